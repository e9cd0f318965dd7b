set -o pipefail
mkdir -p gpurun_out
bash tools/asan_gpu_tests.sh || exit 11
