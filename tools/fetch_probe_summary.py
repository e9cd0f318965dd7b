"""Bytes per point and I-cache misses per point of tools/fetch_probe.py's launches, per library
build, from tools/pmc_fetch_probe.sh's passes (gfx950 FETCH_SIZE correction: fetch bytes =
2 x 1024 x FETCH_SIZE for 16-B/lane streaming reads, MI355X_MICROARCH.md; WRITE_SIZE exact).

    python3 tools/fetch_probe_summary.py gpurun_out/fetch_<tag> > profiles/<tag>_fetch_probe.json
"""
import collections
import csv
import glob
import json
import os
import sys

NAMES = {"kzgpot::k_g1_codec(": "k_g1_codec", "kzgpot::k_g2_codec(": "k_g2_codec",
         "kzgpot::k_g2_decompress(": "k_g2_decompress (unchecked)",
         "kzgpot::k_g1_check<(kzgpot::Src)1>": "k_g1_check<PairingBE> (transcode)",
         "kzgpot::k_g2_check<(kzgpot::Src)1>": "k_g2_check<PairingBE> (transcode)"}
ALG = {"k_g1_codec": (48, 96), "k_g2_codec": (96, 192), "k_g2_decompress (unchecked)": (96, 192),
       "k_g1_check<PairingBE> (transcode)": (96, 96), "k_g2_check<PairingBE> (transcode)": (192, 192)}


def read(path):
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    with open(path) as f:
        for r in csv.DictReader(f):
            for pat, key in NAMES.items():
                if pat in r["Kernel_Name"]:
                    d = per[key][int(r.get("Dispatch_Id") or r.get("Correlation_Id"))]
                    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                    d["_grid"] = int(r["Grid_Size"])
    # per (kernel, grid size): the last dispatch (fetch_probe.py launches each twice per size)
    out = {}
    for k, v in per.items():
        for did in sorted(v):
            out[(k, v[did]["_grid"])] = v[did]
    return out


def main():
    root = sys.argv[1]
    out = {"source": f"tools/pmc_fetch_probe.sh -> {root}", "builds": {}}
    for name_file in sorted(glob.glob(os.path.join(root, "lib*.name"))):
        lib = open(name_file).read().strip()
        d = name_file[:-5]
        f = read(glob.glob(os.path.join(d, "FETCH_SIZE", "**", "*counter_collection.csv"), recursive=True)[0])
        w = read(glob.glob(os.path.join(d, "WRITE_SIZE", "**", "*counter_collection.csv"), recursive=True)[0])
        ic = read(glob.glob(os.path.join(d, "SQC_ICACHE_MISSES", "**", "*counter_collection.csv"), recursive=True)[0])
        rq_files = glob.glob(os.path.join(d, "TCC_EA0_RDREQ_sum", "**", "*counter_collection.csv"), recursive=True)
        rq = read(rq_files[0]) if rq_files else {}
        rows = {}
        for (k, n) in sorted(f):
            rd = 2 * 1024 * f[(k, n)]["FETCH_SIZE"] / n
            wr = 1024 * w[(k, n)]["WRITE_SIZE"] / n if (k, n) in w else None
            c = ic.get((k, n), {})
            r = rq.get((k, n), {})
            row = {"points": n, "fetch_B_per_point": round(rd, 3), "write_B_per_point": None if wr is None else round(wr, 3),
                   "algorithmic_read_write": ALG[k], "fetch_excess_B_per_point": round(rd - ALG[k][0], 3),
                   "fetch_excess_MB_per_launch": round((rd - ALG[k][0]) * n / 1e6, 3),
                   "icache_misses_per_point": round(c["SQC_ICACHE_MISSES"] / n, 3) if "SQC_ICACHE_MISSES" in c else None,
                   "valu_per_wave": round(c.get("SQ_INSTS_VALU", 0) / max(1, c.get("SQ_WAVES", 1))) if c else None}
            if r:
                tot = r.get("TCC_EA0_RDREQ_sum", 0)
                b32, b128 = r.get("TCC_EA0_RDREQ_32B_sum", 0), r.get("TCC_EA0_RDREQ_128B_sum", 0)
                row["rdreq"] = {"total": tot, "32B": b32, "128B": b128, "64B": tot - b32 - b128,
                                "dram": r.get("TCC_EA0_RDREQ_DRAM_sum"),
                                "bytes_by_size_per_point": round((32 * b32 + 128 * b128 + 64 * (tot - b32 - b128)) / n, 3),
                                "sqc_inst_req": r.get("SQC_TC_INST_REQ"), "sqc_data_read_req": r.get("SQC_TC_DATA_READ_REQ")}
            rows[f"{k} @ {n}"] = row
        out["builds"][lib] = rows
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
