#!/usr/bin/env bash
# Round profile on one MI355X (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of the default bench command (same command as the bench line,
#      minus the drop-in binaries' wall-clock rows)
#   2. three separate --pmc passes (FETCH_SIZE / WRITE_SIZE / SQ_*) of a 1-step bench that also runs
#      the next rows (config 3's 2^20 G2, config 5's 2^28 BN254, loader, transcode)
# Outputs under gpurun_out/prof_<tag>/; copy the summaries into profiles/ afterwards
# (tools/pmc_summary.py turns the three PMC CSVs into profiles/pmc_traffic.json, per dispatch, largest
# grid per kernel; tools/trace_summary.py splits the kernel trace by launch size).
set -euo pipefail
tag=${1:-round}
out=$GRAFT_REPO_ROOT/gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
step="bench.py --steps 1 --warmup 0 --no-verify --no-cpu-baseline --e2e-log2 0"

# --no-cli: the bench's drop-in binary rows start child processes, which must never start from a
# process the profiler's preloaded library has put on the GPU, and whose _exit would drop their
# trace data anyway; every other row of the default line runs
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run \
  -- python3 bench.py --no-cli > "$out/bench_traced.json" 2> "$out/trace.err"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run \
  -- python3 $step > /dev/null 2> "$out/fetch.err"
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run \
  -- python3 $step > /dev/null 2> "$out/write.err"
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d "$out/sq" -o run -- python3 $step > /dev/null 2> "$out/sq.err"
# per-phase VALU split of the checked codecs (tools/codec_phases.py -> pmc_summary.py --phases)
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$out/phases" -o run \
  -- python3 tools/codec_phases.py > "$out/codec_phases.json" 2> "$out/phases.err"
find "$out" -name "*.csv" | sort
