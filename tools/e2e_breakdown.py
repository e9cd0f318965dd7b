"""The end-to-end preprocess calls of bench.py's next_rows, one after another, for a stage trace:

    rocprofv3 --marker-trace --kernel-trace --memory-copy-trace --output-format csv -d DIR -o run \
        -- python3 tools/e2e_breakdown.py [--n-log2 21] > calls.json
    python3 tools/stage_summary.py DIR calls.json > profiles/<tag>_e2e_stages.json

Each C-ABI call (kzgpot_preprocess_buffer_ex without / with the two BLAKE2b digests,
kzgpot_preprocess_ex file to file, for kgz and fastkzg) is timed here with perf_counter and
bracketed inside the library by the roctx range "kzgpot.preprocess" (csrc/trace.hpp);
stage_summary.py splits each such range into its stages (H2D staging, kernels, D2H, the digests,
pread / pwrite) from the three traces. Reference: preprocess-kgz.rs:69-199,
preprocess-fastkgz.rs:70-213 (the two `main`s these calls replace).
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-log2", type=int, default=21)
    ap.add_argument("--shards", type=int, default=1)
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
        parts.append(D.synth(kind, 100 + i, 0, cnt, dev, with_expected=False)[0])
    parts.append(torch.zeros(3 * 192 + 6 * 96, dtype=torch.uint8, device=dev))
    # The transcript comes to the host through a pinned buffer: the pageable `.cpu()` of round 4
    # was the copy whose completion rocprofiler-sdk never received (profiles/r04a/r04c stage
    # traces: "1 completion callbacks were not delivered" for correlation id 14, this process's
    # main thread, between the generator's kernels 13 and 15 — before the first library call).
    dt = torch.cat(parts)
    host = torch.empty(dt.numel(), dtype=torch.uint8, pin_memory=True)
    host.copy_(dt)
    torch.cuda.synchronize()
    tr = host.numpy().copy()
    del parts, dt, host
    import hashlib

    tr_digest = hashlib.blake2b(tr.tobytes()).hexdigest()
    lib = _lib.load()
    out = np.ones(kzgpot.output_size(a.n_log2, kzgpot.MODE_FASTKZG), np.uint8)
    tmpdir = tempfile.mkdtemp(prefix="kzgpot_stages_")
    src = os.path.join(tmpdir, "powersoftau")
    tr.tofile(src)
    calls = []
    sec, idx = ctypes.c_int(-1), ctypes.c_int64(-1)
    # warm-up: staging buffers sized, output pages faulted in (as bench.py's rows run after others)
    lib.kzgpot_preprocess_buffer_ex(tr.ctypes.data, tr.size, out.ctypes.data, kzgpot.MODE_FASTKZG, a.n_log2,
                                    a.shards, None, None, None, ctypes.byref(sec), ctypes.byref(idx))
    for mode, mname in ((kzgpot.MODE_KZG, "kgz"), (kzgpot.MODE_FASTKZG, "fastkgz")):
        for kind in ("buffer_no_digest", "buffer_digests", "file_transcript_digest", "file_digests"):
            din, dout = ctypes.create_string_buffer(129), ctypes.create_string_buffer(129)
            dig = kind != "buffer_no_digest"
            t = time.perf_counter()
            if kind.startswith("buffer"):
                r = lib.kzgpot_preprocess_buffer_ex(tr.ctypes.data, tr.size, out.ctypes.data, mode, a.n_log2,
                                                    a.shards, None, din if dig else None, dout if dig else None,
                                                    ctypes.byref(sec), ctypes.byref(idx))
            elif kind == "file_transcript_digest":  # the reference's digest work: the transcript check only
                dst = os.path.join(tmpdir, "out")
                r = lib.kzgpot_preprocess_ex(src.encode(), dst.encode(), mode, a.n_log2, a.shards, tr_digest.encode(),
                                             None, None, ctypes.byref(sec), ctypes.byref(idx))
            else:
                dst = os.path.join(tmpdir, "out")
                r = lib.kzgpot_preprocess_ex(src.encode(), dst.encode(), mode, a.n_log2, a.shards, None, din, dout,
                                             ctypes.byref(sec), ctypes.byref(idx))
            dt = time.perf_counter() - t
            if kind.startswith("file"):
                os.unlink(dst)
            calls.append({"call": f"{mname}_{kind}", "seconds": dt, "rc": r})
    os.unlink(src)
    os.rmdir(tmpdir)
    d = ctypes.create_string_buffer(64)
    t = time.perf_counter()
    lib.kzgpot_blake2b(tr.ctypes.data, ctypes.c_size_t(tr.size), d)
    bl = time.perf_counter() - t
    print(json.dumps({"n_log2": a.n_log2, "shards": a.shards, "transcript_bytes": int(tr.size),
                      "blake2b_transcript_alone_s": bl, "blake2b_GBs": tr.size / bl / 1e9, "calls": calls,
                      "kzgpot": kzgpot.version()}))


if __name__ == "__main__":
    main()
