set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/profile_round.sh r04s || exit 11
timeout -k 10 120 tools/microbench/bin/fpops_peak > gpurun_out/r04s_fpops_peak.txt || exit 12
timeout -k 10 300 python3 -u tools/fpops/census.py --peaks gpurun_out/r04s_fpops_peak.txt > gpurun_out/r04s_fp_census.json 2> gpurun_out/r04s_fp_census.err || exit 13
