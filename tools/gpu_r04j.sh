set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 tools/microbench/bin/loader_ceiling > gpurun_out/r04j_loader_ceiling.txt 2>&1 || exit 11
