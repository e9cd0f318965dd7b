"""The host-buffer entry point under a trace (where does the FFI boundary's PCIe overhead go?):
kzgpot_g1_decompress (or `--kind g2`) on 2^`--log2` pageable points, called twice (the first sizes the staging
and faults the output in), as bench.py's host_api row does. Run it under
    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -o run -- python3 tools/host_api_trace.py
and summarise with `--summarise DIR`: the codec kernels' busy union and gaps over the timed call,
and the copies' total and longest durations."""
from __future__ import annotations

import argparse
import csv
import ctypes
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))


def run(log2, kind, register=False):
    import numpy as np
    import torch

    from kzgpot import _lib
    from kzgpot import device as D

    dev = torch.device("cuda", 0)
    n = 1 << log2
    rout = 96 if kind == "g1" else 192
    comp, _ = D.synth(kind, 7, 0, n, dev, with_expected=False)
    host_in = comp.cpu().numpy()
    torch.cuda.synchronize()
    lib = _lib.load()
    out = np.empty(n * rout, np.uint8)
    call = lib.kzgpot_g1_decompress if kind == "g1" else lib.kzgpot_g2_decompress
    reg_ms = None
    if register:  # page-lock the caller's buffers first (hipHostRegister), as an integrator could
        hip = ctypes.CDLL("libamdhip64.so")
        t0 = time.time_ns()
        for buf in (host_in, out):
            rc = hip.hipHostRegister(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(buf.nbytes), ctypes.c_uint(0))
            if rc:
                raise RuntimeError(f"hipHostRegister: {rc}")
        reg_ms = (time.time_ns() - t0) / 1e6
    fb = ctypes.c_int64()
    res = {}
    for name in ("first", "timed"):
        out[:] = 0
        t0 = time.time_ns()
        rc = call(host_in.ctypes.data, ctypes.c_size_t(n), out.ctypes.data, 0, ctypes.byref(fb))
        t1 = time.time_ns()
        res[name] = {"rc": rc, "first_bad": fb.value, "ms": (t1 - t0) / 1e6, "t0_ns": t0, "t1_ns": t1}
        time.sleep(0.2)  # separates the calls in the trace
    # the same points device-resident (bench.py host_api_rows' comparison), event-timed
    d_out = torch.empty(n * rout, dtype=torch.uint8, device=dev)
    key = torch.empty(1, dtype=torch.int64, device=dev)
    D.codec_dev(f"{kind}_decompress", comp, d_out, key)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    D.codec_dev(f"{kind}_decompress", comp, d_out, key)
    e[1].record()
    torch.cuda.synchronize()
    res["device_resident_ms"] = e[0].elapsed_time(e[1])
    res["overhead_frac"] = res["timed"]["ms"] / res["device_resident_ms"] - 1
    res["lib"] = _lib.LIB_PATH
    res["kind"], res["points"], res["registered"], res["register_ms"] = kind, n, register, reg_ms
    print(json.dumps(res))


def summarise(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(("k", r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(("c", r.get("Direction", "copy"), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    codec = sorted((s, e) for k, nm, s, e in rows if k == "k" and "k_g1_codec" in nm)
    # the timed call: the second group of codec launches (a gap > 100 ms separates the calls)
    groups, cur = [], [codec[0]]
    for iv in codec[1:]:
        if iv[0] - cur[-1][1] > 100_000_000:
            groups.append(cur)
            cur = []
        cur.append(iv)
    groups.append(cur)
    g = groups[-1]
    t0, t1 = g[0][0], max(e for _, e in g)
    union, last, gaps = 0, t0, []
    for s, e in g:
        if s > last:
            gaps.append((s - last) / 1e6)
            union += 0
        union += max(0, e - max(s, last))
        last = max(last, e)
    copies = [(nm, s, e) for k, nm, s, e in rows if k == "c" and s >= t0 - 50_000_000 and e <= t1 + 50_000_000]
    blits = [(nm, s, e) for k, nm, s, e in rows if k == "k" and "k_g1_codec" not in nm and t0 - 50_000_000 <= s <= t1]
    out = {"codec_launches": len(g), "codec_span_ms": (t1 - t0) / 1e6, "codec_busy_union_ms": union / 1e6,
           "gaps_ms": [round(x, 3) for x in gaps],
           "codec_durations_ms": [round((e - s) / 1e6, 3) for s, e in g],
           "copies": len(copies), "copy_ms_total": sum(e - s for _, s, e in copies) / 1e6,
           "copy_first_ms": (copies[0][2] - copies[0][1]) / 1e6 if copies else None,
           "copy_before_first_codec_ms": (t0 - min(s for _, s, _ in copies)) / 1e6 if copies else None,
           "copy_after_last_codec_ms": (max(e for _, _, e in copies) - t1) / 1e6 if copies else None,
           "other_kernels": len(blits), "other_kernel_names": sorted({nm[:60] for nm, _, _ in blits}),
           "other_kernel_ms_total": sum(e - s for _, s, e in blits) / 1e6}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2", type=int, default=25)
    ap.add_argument("--kind", choices=["g1", "g2"], default="g1")
    ap.add_argument("--register", action="store_true", help="hipHostRegister the host buffers first")
    ap.add_argument("--summarise")
    a = ap.parse_args()
    if a.summarise:
        summarise(a.summarise)
    else:
        run(a.log2, a.kind, a.register)
