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


def tiled_transcript(n_log2, golden=os.path.join(ROOT, "tests", "golden", "transcript_n1024.bin"), n0=1024):
    """A response-layout transcript at N = 2^n_log2 whose sections repeat the N = 2^10 golden
    transcript's sections (all valid, subgroup-checked points)."""
    src = open(golden, "rb").read()
    n = 1 << n_log2
    out, o = [bytes(64)], 64
    for cnt0, cnt, rec in ((2 * n0 - 1, 2 * n - 1, 48), (n0, n, 96), (n0, n, 48), (n0, n, 48), (1, 1, 96)):
        sec = src[o:o + cnt0 * rec]
        o += cnt0 * rec
        out.append((sec * (-(-cnt // cnt0)))[:cnt * rec])
    out.append(src[o:])
    return b"".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-log2", type=int, default=21)
    ap.add_argument("--shards", type=int, default=1)
    a = ap.parse_args()
    import numpy as np
    import kzgpot
    from kzgpot import _lib

    # The transcript is built on the host, with no torch in the process: every memory copy in the
    # trace is then the library's own. (Rounds 4-5 generated it on the GPU and copied it back
    # through torch; rocprofiler-sdk never received that one copy's completion — correlation id 14
    # on the main thread, a ROCclr blit copy between the generator's kernels and the first library
    # call, pageable or pinned alike: "1 completion callbacks were not delivered",
    # profiles/r05a_stages_note.txt.) The sections tile the config-1 transcript's valid points
    # (tests/golden/transcript_n1024.bin): the same per-point work as distinct points.
    tr = np.frombuffer(tiled_transcript(a.n_log2), np.uint8)
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
