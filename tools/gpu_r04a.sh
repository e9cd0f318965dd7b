set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04a_pytest_gpu.txt 2>&1 || exit 11
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04a_smoke.txt 2>&1 || exit 12
timeout -k 10 300 python bench.py > gpurun_out/r04a_bench_n1.json 2> gpurun_out/r04a_bench.err || exit 13
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --g1-log2 24 --steps 2 --warmup 1 --bn254-log2 0 --no-cpu-baseline > gpurun_out/r04a_bench_gloo2.json 2> gpurun_out/r04a_bench_gloo2.err || exit 14
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r04a_stages -o run -- python3 tools/e2e_breakdown.py > gpurun_out/r04a_stages_calls.json 2> gpurun_out/r04a_stages.err || exit 15
python3 tools/stage_summary.py gpurun_out/r04a_stages gpurun_out/r04a_stages_calls.json > gpurun_out/r04a_e2e_stages.json 2>&1 || exit 16
