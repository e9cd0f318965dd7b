set -o pipefail
mkdir -p gpurun_out/ab_file3
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_preprocess.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04g_pytest_gpu.txt 2>&1 || exit 11
for r in 1 2 3; do
  KZGPOT_LIB=$PWD/kzg-setup-powersoftau_amd/build_exp_old/libkzgpot.so timeout -k 10 120 python3 tools/e2e_breakdown.py > gpurun_out/ab_file3/old_$r.json 2>/dev/null || exit 12
  timeout -k 10 120 python3 tools/e2e_breakdown.py > gpurun_out/ab_file3/new_$r.json 2>/dev/null || exit 13
done
