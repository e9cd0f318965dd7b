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
    # the last dispatch of each kernel (fetch_probe.py launches each twice)
    return {k: v[max(v)] for k, v in per.items()}


def main():
    root = sys.argv[1]
    out = {"source": f"tools/pmc_fetch_probe.sh -> {root}", "builds": {}}
    for name_file in sorted(glob.glob(os.path.join(root, "lib*.name"))):
        lib = open(name_file).read().strip()
        d = name_file[:-5]
        f = read(glob.glob(os.path.join(d, "FETCH_SIZE", "**", "*counter_collection.csv"), recursive=True)[0])
        w = read(glob.glob(os.path.join(d, "WRITE_SIZE", "**", "*counter_collection.csv"), recursive=True)[0])
        ic = read(glob.glob(os.path.join(d, "SQC_ICACHE_MISSES", "**", "*counter_collection.csv"), recursive=True)[0])
        rows = {}
        for k in NAMES.values():
            if k not in f:
                continue
            n = f[k]["_grid"]
            rd = 2 * 1024 * f[k]["FETCH_SIZE"] / n
            wr = 1024 * w[k]["WRITE_SIZE"] / n if k in w else None
            miss = ic.get(k, {}).get("SQC_ICACHE_MISSES")
            rows[k] = {"points": n, "fetch_B_per_point": round(rd, 2), "write_B_per_point": None if wr is None else round(wr, 2),
                       "algorithmic_read_write": ALG[k], "fetch_excess_B_per_point": round(rd - ALG[k][0], 2),
                       "icache_misses_per_point": None if miss is None else round(miss / n, 3),
                       "valu_per_wave": None if k not in ic else round(ic[k].get("SQ_INSTS_VALU", 0) / max(1, ic[k].get("SQ_WAVES", 1)))}
        out["builds"][lib] = rows
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
