set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r04w_bench_n1.json 2> gpurun_out/r04w_bench.err || exit 11
