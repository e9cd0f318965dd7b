"""Development probe: golden vectors + N=1024 transcript + rough kernel throughput on one GPU."""
import ctypes
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))
import torch  # noqa: E402  (loads the HIP runtime first)

import kzgpot  # noqa: E402
from kzgpot import _lib  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")


def golden(name, op, flags_extra):
    V = json.load(open(os.path.join(G, name + ".json")))["vectors"]
    bad = 0
    for v in V:
        flags = flags_extra | (0 if v["check"] else kzgpot.NO_SUBGROUP_CHECK)
        r = kzgpot.run_codec(op, bytes.fromhex(v["in"]), flags, want_status=True)
        ok = r.status[0] == v["status"] and (v["out"] is None or r.out.hex() == v["out"])
        if v["out"] is None and r.out != bytes(len(r.out)):
            ok = False
        if not ok:
            bad += 1
            print("  MISMATCH", name, hex(flags), v["note"], "got", r.status[0], "want", v["status"])
    print(f"{name} flags={flags_extra}: {len(V)} vectors, {bad} mismatches", flush=True)
    return bad


def main():
    print("devices", kzgpot.device_count(), kzgpot.version(), flush=True)
    bad = 0
    for extra in (0, kzgpot.SUBGROUP_REF):
        bad += golden("g1_decompress", "g1_decompress", extra)
        bad += golden("g2_decompress", "g2_decompress", extra)
        bad += golden("g1_transcode", "g1_transcode", extra)
        bad += golden("g2_transcode", "g2_transcode", extra)
    meta = json.load(open(os.path.join(G, "transcript_n1024.json")))
    tr = open(os.path.join(G, "transcript_n1024.bin"), "rb").read()
    for mode, key in ((kzgpot.MODE_KZG, "kgz_blake2b"), (kzgpot.MODE_FASTKZG, "fastkgz_blake2b")):
        t = time.time()
        out = kzgpot.preprocess_buffer(tr, 10, mode)
        ok = hashlib.blake2b(out).hexdigest() == meta[key]
        print(f"preprocess mode={mode}: digest {'OK' if ok else 'MISMATCH'} ({time.time() - t:.2f}s)", flush=True)
        bad += not ok

    # throughput probe: tile the valid golden G1 points to 2^n records, device buffers
    lib = _lib.load()
    V = [v for v in json.load(open(os.path.join(G, "g1_decompress.json")))["vectors"] if v["status"] == 0 and v["check"]]
    pts = b"".join(bytes.fromhex(v["in"]) for v in V)
    for op, rin, rout, fn, vecs in (("g1", 48, 96, lib.kzgpot_g1_decompress_dev, pts),):
        n = 1 << int(os.environ.get("PROBE_LOG2", "20"))
        reps = n // (len(vecs) // rin) + 1
        host = torch.frombuffer(bytearray((vecs * reps)[: n * rin]), dtype=torch.uint8)
        d_in = host.cuda()
        d_out = torch.empty(n * rout, dtype=torch.uint8, device="cuda")
        key = torch.empty(1, dtype=torch.int64, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        for flags in (0, kzgpot.SUBGROUP_REF, kzgpot.NO_SUBGROUP_CHECK):
            fn(d_in.data_ptr(), n, d_out.data_ptr(), flags, key.data_ptr(), None, stream)
            torch.cuda.synchronize()
            t = time.time()
            iters = 2
            for _ in range(iters):
                fn(d_in.data_ptr(), n, d_out.data_ptr(), flags, key.data_ptr(), None, stream)
            torch.cuda.synchronize()
            dt = (time.time() - t) / iters
            k = int(key.item()) & 0xFFFFFFFFFFFFFFFF
            fb = ctypes.c_int64()
            rc = lib.kzgpot_decode_bad_key(k, ctypes.byref(fb))
            print(f"{op} n={n} flags={flags}: {dt * 1e3:.1f} ms  {n / dt / 1e6:.2f} M pt/s  rc={rc}", flush=True)
    print("TOTAL MISMATCHES", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
