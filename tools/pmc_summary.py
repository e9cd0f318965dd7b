"""Summarise rocprofv3 --pmc CSVs of a bench.py run into profiles/pmc_traffic.json.

    python tools/pmc_summary.py FETCH.csv WRITE.csv SQ.csv [--out profiles/pmc_traffic.json] [--source "..."]

Per kernel (averaged over its dispatches): HBM bytes per point from FETCH_SIZE / WRITE_SIZE with the
gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md (FETCH_SIZE and WRITE_SIZE are KiB;
FETCH_SIZE reports half the bytes of a 16-B/lane streaming read, so fetch bytes = 2 x 1024 x
FETCH_SIZE), VALU instructions per point, and register counts. bench.py reads the G1 codec entry
(`k_g1_decompress` + `k_g1_check`) for its `roofline.traffic`.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json

KERNELS = {
    "k_g1_decompress": "kzgpot::k_g1_decompress(",
    "k_g1_check": "kzgpot::k_g1_check<(kzgpot::Src)0>",
    "k_g2_decompress": "kzgpot::k_g2_decompress(",
    "k_g2_check": "kzgpot::k_g2_check<(kzgpot::Src)0>",
    "k_g1_load": "kzgpot::k_load<2, 256>",
    "k_g2_load": "kzgpot::k_load<4, 128>",
}


def read(path):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            for key, pat in KERNELS.items():
                if pat in row["Kernel_Name"]:
                    per[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
                    meta[key] = (int(row["Grid_Size"]), int(row["VGPR_Count"]), int(row["Accum_VGPR_Count"]))
    return per, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("sq")
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--source", default="rocprofv3 --pmc passes of bench.py --steps 1 --warmup 0 --no-verify")
    a = ap.parse_args()
    fetch, meta = read(a.fetch)
    write, _ = read(a.write)
    sq, _ = read(a.sq)
    avg = lambda v: sum(v) / len(v)  # noqa: E731
    out = {"source": a.source,
           "correction": "FETCH_SIZE/WRITE_SIZE are KiB; gfx950 FETCH_SIZE reports 1/2 of a 16-B/lane streaming "
                         "read, so bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM)",
           "kernels": {}}
    for k in KERNELS:
        if k not in meta:
            continue
        pts, vgpr, agpr = meta[k]
        fb = 2 * 1024 * avg(fetch[k]["FETCH_SIZE"]) if fetch[k].get("FETCH_SIZE") else None
        wb = 1024 * avg(write[k]["WRITE_SIZE"]) if write[k].get("WRITE_SIZE") else None
        e = {"points": pts, "fetch_bytes": fb, "write_bytes": wb,
             "bytes_per_point": ((fb or 0) + (wb or 0)) / pts, "vgpr": vgpr, "agpr": agpr}
        if sq[k].get("SQ_INSTS_VALU"):
            # chip-wide count of wave64 VALU instructions / waves = the instruction stream one lane runs
            e["valu_insts_per_wave"] = avg(sq[k]["SQ_INSTS_VALU"]) / (pts / 64)
        for c in ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE", "SQ_WAVES"):
            if sq[k].get(c):
                e[c.lower()] = avg(sq[k][c])
        out["kernels"][k] = e
    if "k_g1_decompress" in out["kernels"] and "k_g1_check" in out["kernels"]:
        out["g1_bytes_per_point"] = (out["kernels"]["k_g1_decompress"]["bytes_per_point"]
                                     + out["kernels"]["k_g1_check"]["bytes_per_point"])
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for k, e in out["kernels"].items():
        print(f"{k:18s} {e['bytes_per_point']:8.1f} B/pt  vgpr {e['vgpr']}")


if __name__ == "__main__":
    main()
