#!/usr/bin/env bash
# Per-wave stall split of the checked codecs (why k_g2_codec sits further
# below its VALU roof than k_g1_codec): three SQ PMC passes and an instruction-fetch pass (the G2
# ladder's doubling loop is ~63 KB of code against the 64 KB instruction cache a CU pair shares)
# over tools/codec_phases.py, which
# launches k_g1_codec / k_g2_codec (and their split halves) on 2^20 synthetic points. Run through
# gpurun from the repo root (tools/gpu_run.sh TAG codec_stalls); summarise with
#   python3 tools/codec_stall_summary.py gpurun_out/TAG_codec_stalls > profiles/TAG_codec_stalls.json
set -uo pipefail
tag=${1:-round}
out=$GRAFT_REPO_ROOT/gpurun_out/${tag}_codec_stalls
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
            "SQ_WAVES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_FLAT GRBM_GUI_ACTIVE" \
            "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$out/p$i" -o run \
    -- python3 tools/codec_phases.py --reps 2 > "$out/p$i.txt" 2> "$out/p$i.err" || exit $?
done
