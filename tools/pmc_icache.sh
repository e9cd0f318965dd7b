#!/usr/bin/env bash
# Instruction-fetch counters of the G1 / G2 codec kernels (run through gpurun from the repo root):
# does the ~290 KB k_g1_codec / k_g2_codec code stream through the 64 KB SQC instruction cache?
# Usage: bash tools/pmc_icache.sh [tag] [lib ...]   (each lib: a libkzgpot.so to A/B; default: this tree)
set -uo pipefail
tag=${1:-icache}
shift || true
libs=("$@")
[ ${#libs[@]} -eq 0 ] && libs=("")
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag
mkdir -p "$out"
export TMPDIR=/tmp
rocprofv3 -L > "$out/avail.txt" 2>&1 || true
grep -oE "SQC?_[A-Z_]*(ICACHE|IFETCH|WAIT_INST|INST_LEVEL)[A-Z_]*" "$out/avail.txt" | sort -u > "$out/icache_counters.txt" || true
step="bench.py --steps 1 --warmup 0 --no-verify --no-cpu-baseline --bn254-log2 0 --e2e-log2 0 --g1-log2 22"
i=0
for lib in "${libs[@]}"; do
  i=$((i + 1))
  if [ -n "$lib" ]; then export KZGPOT_LIB=$lib; else unset KZGPOT_LIB; fi
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU \
    --output-format csv -d "$out/lib$i" -o run -- python3 $step > "$out/lib$i.json" 2> "$out/lib$i.err" || exit $?
done
