#!/usr/bin/env bash
# PMC passes over tools/fetch_probe.py for one or more library builds (run through gpurun from the
# repo root). Usage: bash tools/pmc_fetch_probe.sh TAG LIB [LIB ...]
set -uo pipefail
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out/fetch_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$out/avail.txt" 2>&1 || true
i=0
for lib in "$@"; do
  i=$((i + 1))
  export KZGPOT_LIB=$GRAFT_REPO_ROOT/$lib
  echo "$lib" > "$out/lib$i.name"
  mkdir -p "$out/lib$i"
  for pass in "FETCH_SIZE" "WRITE_SIZE" "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_INSTS_VALU" \
              "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum SQC_TC_INST_REQ SQC_TC_DATA_READ_REQ"; do
    p=$(echo "$pass" | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$out/lib$i/$p" -o run \
      -- python3 tools/fetch_probe.py --log2s ${LOG2S:-20,22} > "$out/lib$i/$p.json" 2> "$out/lib$i/$p.err" || exit $?
  done
done
