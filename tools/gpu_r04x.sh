set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --g1-log2 24 --steps 2 --warmup 1 --bn254-log2 0 --no-cpu-baseline > gpurun_out/r04x_bench_gloo2.json 2> gpurun_out/r04x_bench_gloo2.err || exit 11
