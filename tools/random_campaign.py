"""Random-input parity campaign: the product kernels against the GPU port of the oracle
(tests/gpu_oracle, sharing nothing with csrc/) on many seeds of random records, bytes and every
per-point status compared — the random-at-scale tests of tests/test_gpu_oracle_port.py, run for
longer than a test suite can.

    python3 tools/random_campaign.py [--budget 600] > profiles/<tag>_random_campaign.json

Per op and seed: 2^log2 random records shaped as the tests shape them (G1 / G2 compressed with the
compression bit set and random x: about half on the curve and, being random, outside the
subgroup; pairing-uncompressed G1 / G2 with random SWFlags, almost all off the curve; loader
records with random SWFlags; BN254 compressed with random flags). Ops rotate until the time budget
is spent; a mismatch stops the run and is reported with its first indices.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))
from kzgpot import device as D  # noqa: E402

PORT = os.path.join(ROOT, "tests", "gpu_oracle", "build", "liboracle_gpu.so")
OPS = {"g1_decompress": (0, 48, 96), "g2_decompress": (1, 96, 192), "g1_transcode": (2, 96, 96),
       "g2_transcode": (3, 192, 192), "bn254_g1_decompress": (4, 32, 64), "g1_load": (5, 96, 104),
       "g2_load": (6, 192, 200)}


def fix_g1(r):
    r[:, 0] = 0x80 | (r[:, 0] & 0x7F)


def fix_g2(r):
    r[:, 0] = 0x80 | (r[:, 0] & 0x3F)
    r[:, 48] &= 0x1F


def fix_g1_unc(r):
    r[:, 0] &= 0x1F
    r[:, 48] &= 0xDF


def fix_g2_unc(r):
    for k in (0, 48, 144):
        r[:, k] &= 0x1F
    r[:, 96] &= 0xDF


def fix_g1_load(r):
    r[:, 47] &= 0x1F
    r[:, 95] &= 0xDF


def fix_g2_load(r):
    for k in (47, 95, 143):
        r[:, k] &= 0x1F
    r[:, 191] &= 0xDF


def fix_bn(r):
    r[:, 31] &= 0xDF


# (op, log2 records per seed, shaping, flags); flags 2 = the reference mul_bits(r) subgroup test
PLAN = [("g1_decompress", 22, fix_g1, 0), ("g2_decompress", 18, fix_g2, 0), ("g1_transcode", 18, fix_g1_unc, 0),
        ("g2_transcode", 16, fix_g2_unc, 0), ("g1_load", 22, fix_g1_load, 0), ("g2_load", 21, fix_g2_load, 0),
        ("bn254_g1_decompress", 22, fix_bn, 0), ("g1_decompress", 18, fix_g1, 2), ("g2_decompress", 16, fix_g2, 2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget", type=float, default=600.0, help="seconds")
    ap.add_argument("--seed0", type=int, default=1000, help="first seed (a second campaign takes new ones)")
    ap.add_argument("--ops", default=None, help="comma-separated op names to run (default: the whole plan)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    port = ctypes.CDLL(PORT)
    port.oracle_gpu_run.restype = ctypes.c_int
    port.oracle_gpu_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint32, ctypes.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream
    totals = {}
    t0, seed, ok = time.time(), a.seed0, True
    plan = [p for p in PLAN if not a.ops or p[0] in a.ops.split(",")]
    while ok and time.time() - t0 < a.budget:
        for op, log2, fix, flags in plan:
            if time.time() - t0 >= a.budget:
                break
            code, rin, rout = OPS[op]
            n = 1 << log2
            seed += 1
            g = torch.Generator(device="cuda").manual_seed(seed)
            r = torch.randint(0, 256, (n, rin), dtype=torch.uint8, device=dev, generator=g)
            fix(r)
            d_in = r.view(-1)
            out = torch.empty(n * rout, dtype=torch.uint8, device=dev)
            st = torch.empty(n, dtype=torch.uint8, device=dev)
            key = torch.empty(1, dtype=torch.int64, device=dev)
            D.codec_dev(op, d_in, out, key, flags, d_status=st)
            pout = torch.full((n * rout,), 0x5A, dtype=torch.uint8, device=dev)
            pst = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
            if port.oracle_gpu_run(code, d_in.data_ptr(), n, pout.data_ptr(), pst.data_ptr(), flags & 1, stream):
                raise RuntimeError(f"port failed on {op}")
            torch.cuda.synchronize()
            name = f"{op}{' (mul_bits(r) mode)' if flags & 2 else ''}"
            t = totals.setdefault(name, {"records": 0, "seeds": 0, "status_histogram": {}, "mismatches": 0})
            bad = (st != pst) | (out.view(n, rout) != pout.view(n, rout)).any(dim=1)
            nbad = int(bad.sum())
            t["records"] += n
            t["seeds"] += 1
            t["mismatches"] += nbad
            for k, v in zip(*torch.unique(pst, return_counts=True)):
                t["status_histogram"][int(k)] = t["status_histogram"].get(int(k), 0) + int(v)
            if nbad:
                t["first_mismatches"] = bad.nonzero()[:8].flatten().tolist()
                t["seed_of_mismatch"] = seed
                ok = False
            print(f"{time.time() - t0:7.1f}s {name} seed {seed}: {n} records, {nbad} mismatches", file=sys.stderr,
                  flush=True)
            del r, out, st, pout, pst
    print(json.dumps({"budget_s": a.budget, "seed0": a.seed0, "elapsed_s": time.time() - t0, "all_equal": ok,
                      "status_codes": "0 ok, 1 compression mode, 2 unexpected info, 3 not in field, 4 not on curve, "
                                      "5 not in subgroup, 6 unexpected flags",
                      "ops": totals}, indent=1))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
