"""Where the end-to-end preprocess time goes (C ABI, host buffers, 1 GPU): with / without the
BLAKE2b digests, and the τG1 section alone through the host-buffer codec API.

    python tools/e2e_breakdown.py [--n-log2 21]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-log2", type=int, default=21)
    a = ap.parse_args()
    import numpy as np
    import torch
    import kzgpot
    from kzgpot import _lib
    from kzgpot import device as D

    dev = torch.device("cuda", 0)
    n = 1 << a.n_log2
    parts = [torch.zeros(64, dtype=torch.uint8, device=dev)]
    for i, (kind, cnt) in enumerate((("g1", 2 * n - 1), ("g2", n), ("g1", n), ("g1", n), ("g2", 1))):
        parts.append(D.synth(kind, 100 + i, 0, cnt, dev)[0])
    parts.append(torch.zeros(3 * 192 + 6 * 96, dtype=torch.uint8, device=dev))
    tr = torch.cat(parts).cpu().numpy()
    lib = _lib.load()
    out = np.ones(kzgpot.output_size(a.n_log2, kzgpot.MODE_FASTKZG), np.uint8)
    res = {}
    for mode, mname in ((kzgpot.MODE_KZG, "kgz"), (kzgpot.MODE_FASTKZG, "fastkgz")):
        for dig in (False, True):
            sec, idx = ctypes.c_int(-1), ctypes.c_int64(-1)
            din, dout = ctypes.create_string_buffer(129), ctypes.create_string_buffer(129)
            t = time.perf_counter()
            r = lib.kzgpot_preprocess_buffer_ex(tr.ctypes.data, tr.size, out.ctypes.data, mode, a.n_log2, 1, None,
                                                din if dig else None, dout if dig else None, ctypes.byref(sec),
                                                ctypes.byref(idx))
            res[f"{mname}_{'digests' if dig else 'no_digests'}_s"] = time.perf_counter() - t
            assert r == 0
    g1 = tr[64:64 + (2 * n - 1) * 48]
    o1 = np.ones((2 * n - 1) * 96, np.uint8)
    fb = ctypes.c_int64()
    t = time.perf_counter()
    lib.kzgpot_g1_decompress(g1.ctypes.data, ctypes.c_size_t(2 * n - 1), o1.ctypes.data, 0, ctypes.byref(fb))
    res["tau_g1_host_api_s"] = time.perf_counter() - t
    g2 = tr[64 + (2 * n - 1) * 48:64 + (2 * n - 1) * 48 + n * 96]
    o2 = np.ones(n * 192, np.uint8)
    t = time.perf_counter()
    lib.kzgpot_g2_decompress(g2.ctypes.data, ctypes.c_size_t(n), o2.ctypes.data, 0, ctypes.byref(fb))
    res["tau_g2_host_api_s"] = time.perf_counter() - t
    d = ctypes.create_string_buffer(64)
    t = time.perf_counter()
    lib.kzgpot_blake2b(tr.ctypes.data, ctypes.c_size_t(tr.size), d)
    res["blake2b_transcript_s"] = time.perf_counter() - t
    print(json.dumps(res))


if __name__ == "__main__":
    main()
