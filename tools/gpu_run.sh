#!/usr/bin/env bash
# One parametrised GPU-box runner (replaces round 4's one-off tools/gpu_r04*.sh launch scripts):
#
#   gpurun --timeout 1200 -- bash tools/gpu_run.sh TAG STEP [STEP ...]
#
# runs the named steps in order from the repo root, each under its own time limit, writing
# gpurun_out/TAG_<step>.* ; the first failing step ends the run with exit code 10 + its position
# (nothing more touches the GPU after a failure, a fault or a time limit). Steps:
#   pytest        the whole GPU suite (pytest -m gpu)
#   quicktests    the CLI, C-ABI stream and preprocess GPU tests only
#   smoke         __graft_entry__.smoke()
#   bench         python bench.py (the default line: config 4 + every row + cpu_baseline)
#   bench_quick   bench.py without the CPU baseline and the e2e rows (kernel numbers only)
#   stages        e2e stage trace: rocprofv3 marker + kernel + memory-copy trace of
#                 tools/e2e_breakdown.py, summarised by tools/stage_summary.py
#   codec_stalls  per-wave stall split of the G1 / G2 codec kernels (tools/pmc_codec_stalls.sh)
#   profile       tools/profile_round.sh TAG (kernel trace --stats + FETCH/WRITE/SQ PMC passes)
#   asan          tools/asan_gpu_tests.sh (host-ASan library under the C-ABI GPU tests)
#   loader_stalls tools/pmc_loader_stalls.sh
#   loader_ceiling tools/microbench/bin/loader_ceiling (the loader's pattern variants, TB/s)
#   gloo2         bench.py --gpus 2 --dist-backend gloo (the N > 1 launch path on one GPU)
#   gloo8         bench.py --gpus 8 --dist-backend gloo at reduced sizes: the driver's world-8 control
#                 flow (8 spawned ranks, the rendezvous-store wait, rank 0's e2e at 8 shards, the exit
#                 code) on the one GPU of the box
#   overlap       tools/overlap_probe.py (copies on a second stream beside a codec launch, normal and
#                 highest stream priority: do RCCL-like copy kernels progress during the decode?)
#   gather1       bench.py --gather-at-1 (the library's RCCL path at one rank)
#   port          tests/test_gpu_oracle_port.py alone (every point vs the GPU port of the oracle)
#   campaign      tools/random_campaign.py for 9 minutes (SEED0=... for fresh seeds)
#   campaign_g2   the same on the G2 ops only, with fresh seeds
#   ab_codec      tools/ab_codec.sh (alternating A/B of two library builds)
#   census        tools/microbench/bin/fpops_peak + tools/fpops/census.py
set -o pipefail
tag=${1:?usage: gpu_run.sh TAG STEP [STEP ...]}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/$tag
pos=0
for step in "$@"; do
  pos=$((pos + 1))
  echo "[gpu_run] $(date +%T) $tag: $step"
  case $step in
    pytest) timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
              --durations=15 > ${o}_pytest_gpu.txt 2>&1 ;;
    quicktests) timeout -k 10 600 python -u -m pytest tests/test_cli_gpu.py tests/test_gpu_capi_stream.py \
                  tests/test_gpu_preprocess.py -x -v --timeout 300 --timeout-method thread > ${o}_quicktests.txt 2>&1 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > ${o}_smoke.txt 2>&1 ;;
    bench) timeout -k 10 600 python -u bench.py > ${o}_bench_n1.json 2> ${o}_bench.err ;;
    bench_quick) timeout -k 10 400 python -u bench.py --no-cpu-baseline --e2e-log2 0 --no-host-api \
                   > ${o}_bench_quick.json 2> ${o}_bench_quick.err ;;
    stages) timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace --memory-copy-trace --output-format csv \
              -d ${o}_stages -o run -- python3 tools/e2e_breakdown.py > ${o}_stages_calls.json 2> ${o}_stages.err &&
            python3 tools/stage_summary.py ${o}_stages ${o}_stages_calls.json > ${o}_e2e_stages.json 2>&1 ;;
    codec_stalls) timeout -k 10 400 bash tools/pmc_codec_stalls.sh $tag &&
                  python3 tools/codec_stall_summary.py ${o}_codec_stalls > ${o}_codec_stalls.json ;;
    profile) timeout -k 10 900 bash tools/profile_round.sh $tag ;;
    asan) timeout -k 10 700 bash tools/asan_gpu_tests.sh ;;
    loader_ceiling) timeout -k 10 400 tools/microbench/bin/loader_ceiling > ${o}_loader_ceiling.txt 2>&1 ;;
    loader_stalls) timeout -k 10 400 bash tools/pmc_loader_stalls.sh ;;
    gloo2) timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --g1-log2 24 --steps 2 --warmup 1 \
             --bn254-log2 0 --no-cpu-baseline > ${o}_bench_gloo2.json 2> ${o}_bench_gloo2.err ;;
    gloo8) t0=$(date +%s%N); timeout -k 10 600 python bench.py --gpus 8 --dist-backend gloo --g1-log2 23 --g2-log2 13 \
             --steps 2 --warmup 1 --bn254-log2 23 --e2e-log2 18 --no-cpu-baseline > ${o}_bench_gloo8.json \
             2> ${o}_bench_gloo8.err; rc=$?; echo "wall_ms $(( ($(date +%s%N) - t0) / 1000000 )) rc $rc" \
             > ${o}_bench_gloo8.wall; (exit $rc) ;;
    overlap) timeout -k 10 180 python -u tools/overlap_probe.py > ${o}_overlap.json 2> ${o}_overlap.err ;;
    gather1) timeout -k 10 400 python bench.py --gather-at-1 --steps 2 --no-cpu-baseline --no-next-rows \
               > ${o}_bench_gather_at_1.json 2> ${o}_bench_gather_at_1.err ;;
    port) timeout -k 10 1000 python -u -m pytest tests/test_gpu_oracle_port.py -x -v --timeout 900 \
            --timeout-method thread --durations=0 > ${o}_pytest_port.txt 2>&1 ;;
    campaign) timeout -k 10 660 python3 -u tools/random_campaign.py --budget 540 --seed0 ${SEED0:-1000} > ${o}_random_campaign.json \
                2> ${o}_random_campaign.err ;;
    campaign_g2) timeout -k 10 660 python3 -u tools/random_campaign.py --budget 540 --seed0 200000 \
                   --ops g2_decompress,g2_transcode > ${o}_random_campaign_g2.json 2> ${o}_random_campaign_g2.err ;;
    ab_codec) timeout -k 10 900 bash tools/ab_codec.sh ;;
    census) timeout -k 10 120 tools/microbench/bin/fpops_peak > ${o}_fpops_peak.txt &&
            timeout -k 10 300 python3 -u tools/fpops/census.py --peaks ${o}_fpops_peak.txt > ${o}_fp_census.json \
              2> ${o}_fp_census.err ;;
    *) echo "[gpu_run] unknown step $step" >&2; exit 2 ;;
  esac
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "[gpu_run] $tag: step $step failed with $rc" >&2
    exit $((10 + pos))
  fi
done
echo "[gpu_run] $(date +%T) $tag: done"
