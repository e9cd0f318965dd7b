set -o pipefail
mkdir -p gpurun_out/ab_file
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_preprocess.py tests/test_cli_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04e_pytest_gpu.txt 2>&1 || exit 11
for r in 1 2 3; do
  KZGPOT_LIB=$PWD/kzg-setup-powersoftau_amd/build_exp_old/libkzgpot.so timeout -k 10 120 python3 tools/e2e_breakdown.py > gpurun_out/ab_file/old_$r.json 2>/dev/null || exit 12
  timeout -k 10 120 python3 tools/e2e_breakdown.py > gpurun_out/ab_file/new_$r.json 2>/dev/null || exit 13
done
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r04e_stages -o run -- python3 tools/e2e_breakdown.py > gpurun_out/r04e_stages_calls.json 2> gpurun_out/r04e_stages.err || exit 14
python3 tools/stage_summary.py gpurun_out/r04e_stages gpurun_out/r04e_stages_calls.json > gpurun_out/r04e_e2e_stages.json 2>&1 || exit 15
