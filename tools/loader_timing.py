"""Per-launch timing of the loader kernels (k_load<G1> / k_load<G2>) on 2^LOG2 records, to explain
the bench's G1 loader row sitting below the microbenchmark (tools/microbench/loader_ceiling.hip).

    python3 tools/loader_timing.py [--log2 27] [--launches 12] > gpurun_out/loader_timing.json

Sources: the synthetic generator's real ark records (what bench.py feeds the loaders) and random
canonical records (the microbenchmark's input). Each launch is bracketed by its own pair of
events on the launch stream; the output buffer is either fresh or pre-touched by a memset.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kzg-setup-powersoftau_amd"))
from kzgpot import device as D  # noqa: E402


def random_canonical(n, rec, dev):
    r = torch.randint(0, 256, (n * rec,), dtype=torch.uint8, device=dev).view(n, rec // 48, 48)
    r[:, :, 47] %= 0x1a  # top byte < 0x1a: the 381-bit little-endian word is < p, no SWFlags bits
    return r.view(-1)


def time_launches(op, src, out, key, launches):
    """Per-launch ms (own event pair) and the shader clock over each launch (clock probes)."""
    ms, clk = [], []
    for _ in range(launches):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        c0 = D.clock_probe(src.device)
        ev[0].record()
        D.codec_dev(op, src, out, key)
        ev[1].record()
        clk.append((c0, D.clock_probe(src.device)))
        ms.append(ev)
    torch.cuda.synchronize()
    mhz = []
    for a, b in clk:
        c = D.clock_mhz(a, b)
        mhz.append(round(c["mean"]) if c else None)
    return [round(a.elapsed_time(b), 4) for a, b in ms], mhz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2", type=int, default=27)
    ap.add_argument("--launches", type=int, default=12)
    ap.add_argument("--idle", type=float, default=0.0, help="seconds of idle GPU before each row")
    ap.add_argument("--order", default="g1,g2", help="loader order within each source")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n = 1 << a.log2
    key = torch.empty(1, dtype=torch.int64, device=dev)
    res = {"points": n, "launches": a.launches, "rows": []}
    comp, real = D.synth("g1", 11, 0, n, dev)
    del comp
    srcs = {"real ark records": real, "random canonical": random_canonical(n, 96, dev)}
    torch.cuda.synchronize()
    for name, src in srcs.items():
        shapes = {"g1": ("g1_load", 96, 104, n), "g2": ("g2_load", 192, 200, n // 2)}
        for op, rin, rout, m in (shapes[k] for k in a.order.split(",")):
            for pre in (False, True):
                out = torch.empty(m * rout, dtype=torch.uint8, device=dev)
                if pre:
                    out.zero_()
                torch.cuda.synchronize()
                time.sleep(a.idle)
                ms, mhz = time_launches(op, src[:m * rin], out, key, a.launches)
                steady = sorted(ms[2:])
                med = steady[len(steady) // 2]
                res["rows"].append({"source": name, "op": op, "out_pretouched": pre, "idle_s": a.idle, "ms": ms, "shader_mhz": mhz,
                                    "median_after_2_ms": med, "median_TBps": (rin + rout) * m / med / 1e9,
                                    "mean_TBps": (rin + rout) * m * len(ms) / sum(ms) / 1e9,
                                    "all_accepted": D.read_key(key) == (1 << 64) - 1})
                print(json.dumps(res["rows"][-1]), file=sys.stderr, flush=True)
                del out
                torch.cuda.empty_cache()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
