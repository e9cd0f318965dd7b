"""Field-operation census of the codec kernels, set against each primitive's measured peak.

    make -C tools/fpops all      # the census library and the peak microbenchmark (CPU, ~3 min)
    tools/microbench/bin/fpops_peak > gpurun_out/fpops_peak.txt                       # on the GPU
    python3 tools/fpops/census.py --peaks gpurun_out/fpops_peak.txt > profiles/<tag>_fp_census.json

1. Runs every codec op of tools/fpops/build/libfp_census.so (the product kernels compiled with
   fp381.hpp's KZG_FPOP hook counting each Montgomery reduction by kind) on N valid synthetic
   points, checks the output bytes against the generator's, and divides the counts by N.
2. Reads the chip-wide peak of each primitive from tools/microbench/fpops_peak's output.
3. Times each codec op here through the product library (same box, right after the peaks), and
   states its field-op rate: reductions per second, and the fraction of the kernel's time that its reductions would take at their peak rates
   (sum_k count_k / peak_k x points per second; the rest is additions, normalisations, selects,
   loads and stores).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import re
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "kzg-setup-powersoftau_amd"))
from kzgpot import device as D  # noqa: E402

KINDS = ["fp_mul", "fp_sqr", "fp_mul_sum2", "fp_mul_sum3", "fp_mul_addsqr", "f30_mul", "f30_sqr"]
NO_CHECK, REF, SPLIT = 0x1, 0x2, 0x4
OP = {"g1_decompress": 0, "g2_decompress": 1, "g1_transcode": 2, "g2_transcode": 3, "bn254_g1_decompress": 6}


def lib():
    so = ctypes.CDLL(os.path.join(HERE, "build", "libfp_census.so"))
    so.fp_census_run.restype = ctypes.c_int
    so.fp_census_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                 ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong),
                                 ctypes.POINTER(ctypes.c_ulonglong)]
    return so


def census(so, op, src, n, out, want, flags):
    counts = (ctypes.c_ulonglong * 8)()
    key = ctypes.c_ulonglong(0)
    out.zero_()
    rc = so.fp_census_run(OP[op], src.data_ptr(), n, out.data_ptr(), flags, None, counts, ctypes.byref(key))
    if rc:
        raise RuntimeError(f"{op}: fp_census_run failed ({rc})")
    per = {k: counts[i] / n for i, k in enumerate(KINDS) if counts[i]}
    return {"op": op, "flags": flags, "points": n, "per_point": per, "reductions_per_point": sum(per.values()),
            "all_accepted": key.value == (1 << 64) - 1, "bit_exact": bool(torch.equal(out, want))}


def parse_peaks(path):
    """{kind: {"best": G ops/s, "best_at_2_waves": G ops/s}} from fpops_peak's output."""
    pk = {}
    for line in open(path):
        m = re.match(r"(\S+)\s+chains (\d) waves/SIMD<=(\d):\s+([\d.]+) ms\s+([\d.]+) G ops/s", line)
        if not m:
            continue
        k, occ, g = m.group(1), int(m.group(3)), float(m.group(5))
        e = pk.setdefault(k, {"best": 0.0, "best_at_2_waves": 0.0})
        e["best"] = max(e["best"], g)
        if occ == 2:
            e["best_at_2_waves"] = max(e["best_at_2_waves"], g)
    return pk


def live_rates(dev, log2):
    """points/s of each default-flag codec op, timed here through the product library
    (libkzgpot.so's _dev entry points) on 2^log2 synthetic points, after the peak microbenchmark
    on the same box: one clock for both sides of the ratio."""
    n = 1 << log2
    out = {}
    key = torch.empty(1, dtype=torch.int64, device=dev)
    for op, kind, rin, rout in (("g1_decompress", "g1", 48, 96), ("g2_decompress", "g2", 96, 192),
                                ("g1_transcode", "g1", 96, 96), ("g2_transcode", "g2", 192, 192),
                                ("bn254_g1_decompress", "bn254", 32, 64)):
        m = n if kind != "g2" else n // 4
        comp, ark = D.synth(kind, 31, 0, m, dev)
        if op.endswith("transcode"):
            comp = (ark.view(m, 2, 48).flip(-1) if kind == "g1" else ark.view(m, 2, 2, 48).flip(2).flip(-1))
            comp = comp.contiguous().view(-1)
        dst = torch.empty(m * rout, dtype=torch.uint8, device=dev)
        D.codec_dev(op, comp, dst, key)  # warm-up (and the clock ramp)
        D.codec_dev(op, comp, dst, key)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        D.codec_dev(op, comp, dst, key)
        e[1].record()
        torch.cuda.synchronize()
        if D.read_key(key) != (1 << 64) - 1 or not torch.equal(dst, ark):
            raise RuntimeError(f"{op}: live-rate run not bit-exact")
        out[op] = m / (e[0].elapsed_time(e[1]) * 1e-3)
        del comp, ark, dst
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2", type=int, default=12)
    ap.add_argument("--peaks", required=True)
    ap.add_argument("--rate-log2", type=int, default=24, help="points for the live rate runs (G2: / 4)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n = 1 << a.log2
    so = lib()
    g1c, g1a = D.synth("g1", 21, 0, n, dev)
    g2c, g2a = D.synth("g2", 22, 0, n, dev)
    bnc, bna = D.synth("bn254", 23, 0, n, dev)
    g1p = g1a.view(n, 2, 48).flip(-1).contiguous().view(-1)           # pairing uncompressed G1
    g2p = g2a.view(n, 2, 2, 48).flip(2).flip(-1).contiguous().view(-1)  # x.c1 x.c0 y.c1 y.c0, BE
    o1, o2, ob = torch.empty_like(g1a), torch.empty_like(g2a), torch.empty_like(bna)
    rows = []
    for name, flags in (("endomorphism (default)", 0), ("reference mul_bits(r)", REF), ("unchecked", NO_CHECK),
                        ("split phases", SPLIT)):
        rows.append({"case": f"g1_decompress {name}", **census(so, "g1_decompress", g1c, n, o1, g1a, flags)})
        rows.append({"case": f"g2_decompress {name}", **census(so, "g2_decompress", g2c, n, o2, g2a, flags)})
    rows.append({"case": "g1_transcode", **census(so, "g1_transcode", g1p, n, o1, g1a, 0)})
    rows.append({"case": "g2_transcode", **census(so, "g2_transcode", g2p, n, o2, g2a, 0)})
    rows.append({"case": "bn254_g1_decompress (9 x 29-bit limbs)", **census(so, "bn254_g1_decompress", bnc, n, ob, bna, 0)})

    peaks = parse_peaks(a.peaks)
    pps = live_rates(dev, a.rate_log2)
    for r in rows:
        if r["flags"] != 0 or r["op"] not in pps:
            continue
        p = pps[r["op"]]
        r["points_per_s"] = p
        r["reductions_per_s"] = r["reductions_per_point"] * p
        if r["op"].startswith("bn254"):
            continue  # the peaks are the BLS12-381 primitives'
        t_peak = sum(c / (peaks[k]["best_at_2_waves"] * 1e9) for k, c in r["per_point"].items())
        r["reduction_time_at_peak_ns_per_point"] = t_peak * 1e9
        r["kernel_ns_per_point"] = 1e9 / p
        r["reduction_fraction_of_kernel_time"] = t_peak * p
    print(json.dumps({"points": n, "peaks_G_per_s": peaks, "peaks_source": os.path.basename(a.peaks),
                      "rates": "timed here through libkzgpot.so, 2^%d points (G2 2^%d)" % (a.rate_log2, a.rate_log2 - 2),
                      "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
