set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread --durations=15 > gpurun_out/r04u_pytest_gpu.txt 2>&1 || exit 11
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04u_smoke.txt 2>&1 || exit 12
timeout -k 10 300 python bench.py > gpurun_out/r04u_bench_n1.json 2> gpurun_out/r04u_bench.err || exit 13
