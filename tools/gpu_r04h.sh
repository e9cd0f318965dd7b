set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_oracle_port.py -x -v --timeout 900 --timeout-method thread --durations=0 > gpurun_out/r04h_pytest_port.txt 2>&1 || exit 11
