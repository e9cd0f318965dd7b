"""Summarise rocprofv3 --pmc CSVs of a bench.py run into profiles/pmc_traffic.json.

    python tools/pmc_summary.py FETCH.csv WRITE.csv SQ.csv [--out profiles/pmc_traffic.json] [--source "..."]
                               [--mix profiles/r02_valu_mix.json]

Per kernel, from its LARGEST dispatch (the bench runs the codec kernels at several sizes: config 4's
2^27 G1 / 2^16 G2, config 3's 2^20, config 5's 2^28 BN254; counts are normalised per dispatch, so
no average mixes sizes):
  * HBM bytes per point from FETCH_SIZE / WRITE_SIZE with the gfx950 correction of
    /opt/skills/guides/MI355X_MICROARCH.md (FETCH_SIZE and WRITE_SIZE are KiB; FETCH_SIZE reports
    half the bytes of a 16-B/lane streaming read, so fetch bytes = 2 x 1024 x FETCH_SIZE);
  * VALU instructions per wave (SQ_INSTS_VALU / waves = the instruction stream one lane runs for
    its point) and SIMD cycles per VALU instruction (GRBM_GUI_ACTIVE x SIMDs per XCD / SQ_INSTS_VALU);
  * registers: the CSV's VGPR columns (rocprofv3 reports the arch VGPR field in its own units) and
    the code object's .vgpr_count / .group_segment_fixed_size / waves per SIMD, taken from
    profiles/r02_valu_mix.json (tools/valu_mix.py) so DESIGN's occupancy claims can be checked.
bench.py reads the G1 codec entry (`k_g1_codec`, or `k_g1_decompress` + `k_g1_check` for the split
kernels) for `roofline.traffic` and
the per-kernel instruction counts for its `valu` roofs.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os

KERNELS = {
    "k_g1_codec": "kzgpot::k_g1_codec(",
    "k_g1_decompress": "kzgpot::k_g1_decompress(",
    "k_g1_check": "kzgpot::k_g1_check<(kzgpot::Src)0>",
    "k_g2_codec": "kzgpot::k_g2_codec(",
    "k_g2_decompress": "kzgpot::k_g2_decompress(",
    "k_g2_check": "kzgpot::k_g2_check<(kzgpot::Src)0>",
    "k_g1_load": "kzgpot::k_load_direct<2,",  # round 6 (was k_load<2, 128, true, 1>)
    "k_g2_load": "kzgpot::k_load_direct<4,",  # round 6 (was k_load<4, 32> from round 4, k_load<4, 128> before)
    "k_bn254_g1_decompress": "kzgpot::k_bn254_g1_decompress(",
    "k_g1_transcode": "kzgpot::k_g1_check<(kzgpot::Src)1>",
    "k_g2_transcode": "kzgpot::k_g2_check<(kzgpot::Src)1>",
}
LANES_PER_POINT = {"k_g1_load": 2, "k_g2_load": 4}  # the loaders run one coordinate per lane (load_kernels.hip)
SIMDS_PER_XCD = 32 * 4  # GRBM_GUI_ACTIVE is summed over the 8 XCDs (one clock each); 32 CUs x 4 SIMDs per XCD


def read(path):
    """kernel -> dispatch id -> {counter: value, "_grid": threads, "_vgpr": .., "_agpr": ..}"""
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    with open(path) as f:
        for row in csv.DictReader(f):
            for key, pat in KERNELS.items():
                if pat in row["Kernel_Name"]:
                    d = per[key][row.get("Dispatch_Id") or row.get("Correlation_Id")]
                    d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                    d["_grid"] = int(row["Grid_Size"])
                    d["_vgpr"] = int(row.get("VGPR_Count") or row.get("Arch_VGPR_Count") or 0)
                    d["_agpr"] = int(row.get("Accum_VGPR_Count") or 0)
    return per


def largest(dispatches):
    """The dispatches of the largest grid (several identical ones are averaged)."""
    if not dispatches:
        return None
    g = max(d["_grid"] for d in dispatches.values())
    ds = [d for d in dispatches.values() if d["_grid"] == g]
    keys = set().union(*ds)
    return {k: sum(d.get(k, 0.0) for d in ds) / len(ds) for k in keys}


def phases(sq):
    """VALU instructions per wave (= per point's instruction stream) of each codec phase, from the
    SQ pass of tools/codec_phases.py: phase 1 = k_gX_decompress (flags, field checks, square
    root(s), sign rule, emit), phase 2 = k_gX_check<ArkInPlace> (record re-read, Montgomery
    conversion, endomorphism ladder), against the fused k_gX_codec that does both in one pass."""
    res = {}
    for g in ("g1", "g2"):
        row = {}
        for name, key in (("fused", f"k_{g}_codec"), ("phase1_decompress", f"k_{g}_decompress"),
                          ("phase2_check", f"k_{g}_check")):
            d = largest(sq.get(key))
            if d and d.get("SQ_INSTS_VALU"):
                row[name] = {"kernel": KERNELS[key], "points": int(d["_grid"]),
                             "valu_insts_per_wave": d["SQ_INSTS_VALU"] / (d["_grid"] / 64)}
        if {"fused", "phase1_decompress"} <= set(row):
            f, p1 = row["fused"]["valu_insts_per_wave"], row["phase1_decompress"]["valu_insts_per_wave"]
            row["fused_minus_phase1"] = f - p1
            row["phase1_share_of_fused"] = p1 / f
        res[g] = row
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("sq")
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--mix", default="profiles/r02_valu_mix.json")
    ap.add_argument("--source", default="rocprofv3 --pmc passes of bench.py --steps 1 --warmup 0 --no-verify")
    ap.add_argument("--phases", help="SQ pass CSV of tools/codec_phases.py: split each codec's VALU stream by phase")
    a = ap.parse_args()
    fetch, write, sq = read(a.fetch), read(a.write), read(a.sq)
    mix = json.load(open(a.mix)) if os.path.exists(a.mix) else {"kernels": {}}
    out = {"source": a.source,
           "correction": "FETCH_SIZE/WRITE_SIZE are KiB; gfx950 FETCH_SIZE reports 1/2 of a 16-B/lane streaming "
                         "read, so bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM)",
           "normalisation": "per dispatch, largest grid of each kernel",
           "kernels": {}}
    for k, pat in KERNELS.items():
        f, w, s = largest(fetch.get(k)), largest(write.get(k)), largest(sq.get(k))
        base = f or w or s
        if base is None:
            continue
        lpp = LANES_PER_POINT.get(k, 1)
        pts = int(base["_grid"]) // lpp
        fb = 2 * 1024 * f["FETCH_SIZE"] if f and "FETCH_SIZE" in f else None
        wb = 1024 * w["WRITE_SIZE"] if w and "WRITE_SIZE" in w else None
        e = {"points": pts, "lanes_per_point": lpp, "fetch_bytes": fb, "write_bytes": wb,
             "bytes_per_point": ((fb or 0) + (wb or 0)) / pts,
             "csv_vgpr": int(base["_vgpr"]), "csv_agpr": int(base["_agpr"])}
        md = next((m for name, m in mix["kernels"].items() if pat in name), None)
        if md:
            e.update({"code_object_vgpr": md.get("vgpr"), "code_object_agpr": md.get("agpr"),
                      "lds_bytes_per_block": md.get("lds_bytes"), "waves_per_simd": md.get("waves_per_simd"),
                      "avg_simd_cycles_per_valu_at_roof": md.get("avg_cycles_per_valu")})
        if s and s.get("SQ_INSTS_VALU"):
            e["valu_insts_per_wave"] = s["SQ_INSTS_VALU"] / (pts * lpp / 64)  # one lane's stream
            e["valu_insts_per_point"] = e["valu_insts_per_wave"] * lpp
            if s.get("GRBM_GUI_ACTIVE"):
                e["simd_cycles_per_valu"] = s["GRBM_GUI_ACTIVE"] * SIMDS_PER_XCD / s["SQ_INSTS_VALU"]
        for c in ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE", "SQ_WAVES"):
            if s and c in s:
                e[c.lower()] = s[c]
        out["kernels"][k] = e
    if "k_g1_codec" in out["kernels"]:  # the fused one-pass kernel (default since round 2)
        out["g1_bytes_per_point"] = out["kernels"]["k_g1_codec"]["bytes_per_point"]
    elif "k_g1_decompress" in out["kernels"] and "k_g1_check" in out["kernels"]:
        out["g1_bytes_per_point"] = (out["kernels"]["k_g1_decompress"]["bytes_per_point"]
                                     + out["kernels"]["k_g1_check"]["bytes_per_point"])
    if a.phases:
        out["phases"] = phases(read(a.phases))
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for k, e in out["kernels"].items():
        print(f"{k:22s} {e['points']:>10d} pts {e['bytes_per_point']:8.1f} B/pt  "
              f"valu/wave {e.get('valu_insts_per_wave', 0):9.0f}  cyc/valu {e.get('simd_cycles_per_valu', 0):.2f}")


if __name__ == "__main__":
    main()
