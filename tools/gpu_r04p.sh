set -e
mkdir -p gpurun_out
timeout -k 10 120 tools/microbench/bin/fpops_peak > gpurun_out/r04p_fpops_peak.txt
timeout -k 10 300 python3 -u tools/fpops/census.py --peaks gpurun_out/r04p_fpops_peak.txt > gpurun_out/r04p_fp_census.json 2> gpurun_out/r04p_fp_census.err
