set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/pmc_fetch_probe.sh r04c kzg-setup-powersoftau_amd/build/libkzgpot.so || exit 11
bash tools/pmc_loader_stalls.sh || exit 12
timeout -k 10 300 python bench.py > gpurun_out/r04c_bench_n1.json 2> gpurun_out/r04c_bench.err || exit 13
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r04c_stages -o run -- python3 tools/e2e_breakdown.py > gpurun_out/r04c_stages_calls.json 2> gpurun_out/r04c_stages.err || exit 14
python3 tools/stage_summary.py gpurun_out/r04c_stages gpurun_out/r04c_stages_calls.json > gpurun_out/r04c_e2e_stages.json 2>&1 || exit 15
