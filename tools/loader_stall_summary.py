"""Per-wave stall attribution of the loader kernels against their staged pattern, from
tools/pmc_loader_stalls.sh's two SQ passes over tools/microbench/bin/loader_ceiling:

    python3 tools/loader_stall_summary.py gpurun_out/loader_stalls > profiles/<tag>_loader_stalls.json

Per kernel (all its dispatches summed): the wave-cycle split SQ_WAIT_ANY (parked on s_waitcnt:
global or LDS data not back yet) / SQ_WAIT_INST_ANY (ready but not issued) / SQ_ACTIVE_INST_ANY
(issuing), the cycles with a VMEM / LDS instruction issuing, LDS bank conflicts per LDS
instruction, the mean number of VMEM instructions in flight per wave, and the TCP (L1) stalls.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

WANT = {"k_copy16": "copy16 (plain 16-B copy, 192 B/pt)", "k_slab<true, true, false>": "slab_nt (the staged pattern, no arithmetic)",
        "k_load_direct<2, 128, true>": "k_load_direct<2, 128> (product G1 since round 6)",
        "k_load_direct<4, 32, true>": "k_load_direct<4, 32> (product G2 since round 6)",
        "k_load_direct<2, 128>": "k_load_direct<2, 128> (r06h-r06n form)",
        "k_load_direct<4, 32>": "k_load_direct<4, 32> (r06h-r06n form)",
        "k_load<2, 128, true, 1>": "k_load<G1> (staged, product to round 5)",
        "k_load<4, 32, true, 2>": "k_load<G2> 32 (staged, product rounds 4-6)",
        "k_load<4, 128, true, 2>": "k_load<G2> 128 (staged, product to round 3)",
        "k_load_dd<2, 128, 0>": "k_load_dd<2, 128> (direct output, experiment)",
        "k_load_dd<4, 32, 0>": "k_load_dd<4, 32> (direct output, experiment)"}


def main():
    root = sys.argv[1]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = re.sub(r"^(void )?(kzgpot::)?", "", r["Kernel_Name"]).split("(")[0]
            for pat, label in WANT.items():
                if name == pat:
                    tot[label][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {"source": f"tools/pmc_loader_stalls.sh -> {root}", "kernels": {}}
    for label, c in tot.items():
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        lds = c.get("SQ_INSTS_LDS", 0) or 1
        out["kernels"][label] = {
            "wait_any_frac": c.get("SQ_WAIT_ANY", 0) / wc,
            "wait_inst_any_frac": c.get("SQ_WAIT_INST_ANY", 0) / wc,
            "active_inst_any_frac": c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            "active_vmem_frac": c.get("SQ_ACTIVE_INST_VMEM", 0) / wc,
            "active_lds_frac": c.get("SQ_ACTIVE_INST_LDS", 0) / wc,
            "wait_inst_lds_frac": c.get("SQ_WAIT_INST_LDS", 0) / wc,
            "active_valu_frac": c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
            "lds_bank_conflict_per_lds_inst": c.get("SQ_LDS_BANK_CONFLICT", 0) / lds,
            "vmem_in_flight_per_wave": c.get("SQ_INST_LEVEL_VMEM", 0) / wc,
            "valu_per_wave": c.get("SQ_INSTS_VALU", 0) / max(1, c.get("SQ_WAVES", 1)),
            "vmem_rd_per_wave": c.get("SQ_INSTS_VMEM_RD", 0) / max(1, c.get("SQ_WAVES", 1)),
            "vmem_wr_per_wave": c.get("SQ_INSTS_VMEM_WR", 0) / max(1, c.get("SQ_WAVES", 1)),
            "tcp_pending_stall_cycles": c.get("TCP_PENDING_STALL_CYCLES_sum"),
            "tcp_tcr_stall_cycles": c.get("TCP_TCR_TCP_STALL_CYCLES_sum"),
            "raw": dict(c),
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
