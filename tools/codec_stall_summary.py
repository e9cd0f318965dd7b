"""Per-wave stall split of the checked codec kernels from tools/pmc_codec_stalls.sh's three SQ
passes over tools/codec_phases.py (2^20 points per launch):

    python3 tools/codec_stall_summary.py gpurun_out/TAG_codec_stalls > profiles/TAG_codec_stalls.json

Per kernel (its dispatches summed):
  * the wave-cycle split SQ_WAIT_ANY (parked on s_waitcnt) / SQ_WAIT_INST_ANY (ready, not issued)
    / SQ_ACTIVE_INST_ANY (issuing), and the share of wave cycles issuing VALU / LDS / scalar;
  * SIMD cycles per VALU instruction (GRBM_GUI_ACTIVE summed over the 8 XCDs x 128 SIMDs per XCD /
    SQ_INSTS_VALU) — the number the cycle-weighted VALU roof prices at 4.06 (G1) / 4.1 (G2);
  * the fraction of SIMD cycles the VALU spends issuing at the 4-cycle wave64 rate: 4 x SQ_INSTS_VALU /
    the SIMD cycles (on gfx950 SQ_ACTIVE_INST_VALU counts exactly one per VALU instruction, so it
    adds nothing to SQ_INSTS_VALU; the measured r05a ratio is 1.000 for every codec kernel);
  * the EXEC utilisation of VALU work: SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU) (1.0 = no
    divergence: every VALU instruction ran all 64 lanes);
  * per wave: VALU (int32 / int64 split), SALU, SMEM, LDS, branch instructions, LDS bank conflicts.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

SIMDS_PER_XCD = 32 * 4
WANT = [("k_g1_codec", r"k_g1_codec\("), ("k_g2_codec", r"k_g2_codec\("),
        ("k_g1_decompress", r"k_g1_decompress\("), ("k_g2_decompress", r"k_g2_decompress\("),
        ("k_g1_check<ArkInPlace>", r"k_g1_check<\(kzgpot::Src\)0>"), ("k_g2_check<ArkInPlace>", r"k_g2_check<\(kzgpot::Src\)0>")]


def collect(root):
    """{kernel: {counter: sum over its dispatches}}; GRBM_GUI_ACTIVE is taken once per dispatch and
    pass (it is the same clock in every pass), averaged over the passes that carry it."""
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    grbm = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        p = os.path.relpath(f, root).split(os.sep)[0]
        for r in csv.DictReader(open(f)):
            label = next((k for k, pat in WANT if re.search(pat, r["Kernel_Name"])), None)
            if label is None:
                continue
            name, v = r["Counter_Name"], float(r["Counter_Value"])
            if name == "GRBM_GUI_ACTIVE":
                grbm[label][p] += v
            else:
                tot[label][name] += v
    for label, per_pass in grbm.items():
        tot[label]["GRBM_GUI_ACTIVE"] = sum(per_pass.values()) / len(per_pass)
    return tot


def summarise(c):
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    # SQ_WAVES appears in passes 2 and 3: both count the same waves
    waves = c.get("SQ_WAVES", 0) / 2 or 1
    simd_cycles = c.get("GRBM_GUI_ACTIVE", 0) * SIMDS_PER_XCD
    valu = c.get("SQ_INSTS_VALU", 0) or 1
    act_valu = c.get("SQ_ACTIVE_INST_VALU", 0)
    return {
        "waves": waves,
        "wait_any_frac": c.get("SQ_WAIT_ANY", 0) / wc,
        "wait_inst_any_frac": c.get("SQ_WAIT_INST_ANY", 0) / wc,
        "active_inst_any_frac": c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        "active_valu_frac_of_wave_cycles": act_valu / wc,
        "active_lds_frac_of_wave_cycles": c.get("SQ_ACTIVE_INST_LDS", 0) / wc,
        "active_scalar_frac_of_wave_cycles": c.get("SQ_ACTIVE_INST_SCA", 0) / wc,
        "active_misc_frac_of_wave_cycles": c.get("SQ_ACTIVE_INST_MISC", 0) / wc,
        "wait_inst_lds_frac": c.get("SQ_WAIT_INST_LDS", 0) / wc,
        "simd_cycles_per_valu": simd_cycles / valu if simd_cycles else None,
        "valu_issue_frac_at_4_cycles": 4 * valu / simd_cycles if simd_cycles else None,
        "active_valu_per_valu_inst": act_valu / valu,
        "valu_exec_utilisation": c.get("SQ_THREAD_CYCLES_VALU", 0) / (64 * act_valu) if act_valu else None,
        "wave_quad_cycles_per_valu": wc / valu,
        "per_wave": {k: c.get(n, 0) / waves for k, n in (
            ("valu", "SQ_INSTS_VALU"), ("valu_int32", "SQ_INSTS_VALU_INT32"), ("valu_int64", "SQ_INSTS_VALU_INT64"),
            ("salu", "SQ_INSTS_SALU"), ("smem", "SQ_INSTS_SMEM"), ("lds", "SQ_INSTS_LDS"),
            ("branch", "SQ_INSTS_BRANCH"), ("salu_cycles", "SQ_INST_CYCLES_SALU"))},
        "lds_bank_conflict_per_lds_inst": c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, c.get("SQ_INSTS_LDS", 0)),
        "lds_in_flight_per_wave": c.get("SQ_INST_LEVEL_LDS", 0) / wc,
        # the instruction-fetch pass (round 6): SQC instruction-cache misses per wave and per
        # 1,000 VALU instructions, and the miss rate of the instruction fetches
        **({"icache_misses_per_wave": c["SQC_ICACHE_MISSES"] / waves,
            "icache_misses_per_kvalu": 1000 * c["SQC_ICACHE_MISSES"] / valu,
            "icache_miss_rate": c["SQC_ICACHE_MISSES"] / max(1, c.get("SQC_ICACHE_HITS", 0) + c["SQC_ICACHE_MISSES"]),
            "ifetch_per_valu": c.get("SQ_IFETCH", 0) / valu} if "SQC_ICACHE_MISSES" in c else {}),
        "raw": dict(c),
    }


def main():
    root = sys.argv[1]
    tot = collect(root)
    out = {"source": f"tools/pmc_codec_stalls.sh -> {root} (tools/codec_phases.py, 2^20 points per launch)",
           "kernels": {label: summarise(c) for label, c in tot.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
