set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_oracle_port.py -x -q --timeout 600 --timeout-method thread -k "load or Load" > gpurun_out/r04k_pytest_load.txt 2>&1 || exit 11
timeout -k 10 300 python bench.py --steps 1 --no-cpu-baseline --bn254-log2 0 --e2e-log2 0 --no-host-api > gpurun_out/r04k_bench.json 2> gpurun_out/r04k_bench.err || exit 12
timeout -k 10 200 tools/microbench/bin/loader_ceiling > gpurun_out/r04k_loader_ceiling.txt 2>&1 || exit 13
