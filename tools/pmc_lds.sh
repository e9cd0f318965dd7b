#!/usr/bin/env bash
# LDS bank conflicts of the kernels that use LDS (k_load's staged slabs, the codecs' parking lot):
# one --pmc pass over a 1-step bench that runs the loader row. Output: gpurun_out/pmc_lds/.
set -euo pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_lds
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$out" -o run -- python3 bench.py --steps 1 --warmup 0 --no-verify --no-cpu-baseline \
  --e2e-log2 0 --bn254-log2 0 --g1-log2 24 > /dev/null 2> "$out/err.txt"
