#!/usr/bin/env bash
# Per-wave stall attribution of the loader against its staged pattern: the
# loader_ceiling microbenchmark's copy16 / slab_nt / product (k_load_direct) / staged k_load kernels under two SQ PMC
# passes (run through gpurun from the repo root; build tools/microbench/bin/loader_ceiling first).
set -uo pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/loader_stalls
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
            "SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$out/p$i" -o run \
    -- tools/microbench/bin/loader_ceiling > "$out/p$i.txt" 2> "$out/p$i.err" || exit $?
done
