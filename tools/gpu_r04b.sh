set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cp gpurun_out/r04b_pytest_gpu.txt /dev/null 2>/dev/null; true
bash tools/pmc_fetch_probe.sh r04b kzg-setup-powersoftau_amd/build/libkzgpot.so kzg-setup-powersoftau_amd/build_exp_nt/libkzgpot.so || exit 12
PHASES_ONLY=1 timeout -k 10 400 bash tools/ab_libs.sh cur=kzg-setup-powersoftau_amd/build/libkzgpot.so nt=kzg-setup-powersoftau_amd/build_exp_nt/libkzgpot.so || exit 13
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --bn254-log2 0 --e2e-log2 0 > gpurun_out/r04b_bench_hostapi.json 2> gpurun_out/r04b_bench.err || exit 14
