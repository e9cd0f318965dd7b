set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_preprocess.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04t_pytest_preprocess.txt 2>&1 || exit 11
timeout -k 10 300 python -u tools/e2e_breakdown.py --shards 2 > gpurun_out/r04t_e2e_2shards.json 2> gpurun_out/r04t_e2e.err || exit 12
timeout -k 10 300 python -u tools/e2e_breakdown.py --shards 1 > gpurun_out/r04t_e2e_1shard.json 2>> gpurun_out/r04t_e2e.err || exit 13
