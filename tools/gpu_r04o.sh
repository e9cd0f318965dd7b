set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 -u bench.py > gpurun_out/r04o_bench.json 2> gpurun_out/r04o_bench.err
