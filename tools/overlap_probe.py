"""Does a copy on another stream make progress while a codec launch holds the GPU? (Readiness for
the driver's N > 1 run, DESIGN §6: each rank's in-place RCCL all-gather of chunk c runs on the
communicator's stream while chunk c + 1 decodes; RCCL moves data with its own kernels, which must
find CU slots beside the codec's 2^17+ queued workgroups, or the pipeline serialises.)

On one GPU, stand-ins for RCCL's copy kernels: device-to-device copies (ROCm runs them as blit
kernels) of `--copy-mib` MiB, the per-chunk receive volume of an N = 8 rank being ~1.3 GiB,
issued on a second stream right after a codec launch of 2^`--log2` G1 points, with the second
stream at normal and at the highest priority. Reported (event-timed on each stream): the codec's
time alone and with the copies beside it, and each copy's time alone and beside the codec —
a copy that waits for the codec to finish shows a time close to the codec's.

    python3 tools/overlap_probe.py [--log2 25] [--copy-mib 1344] [--copies 4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2", type=int, default=25)
    ap.add_argument("--copy-mib", type=int, default=1344)
    ap.add_argument("--copies", type=int, default=4)
    a = ap.parse_args()
    import torch

    from kzgpot import device as D

    dev = torch.device("cuda", 0)
    n = 1 << a.log2
    comp, _ = D.synth("g1", 7, 0, n, dev, with_expected=False)
    out = torch.empty(n * 96, dtype=torch.uint8, device=dev)
    key = torch.empty(1, dtype=torch.int64, device=dev)
    nb = a.copy_mib << 20
    src = torch.empty(nb, dtype=torch.uint8, device=dev).fill_(1)
    dst = torch.empty(nb, dtype=torch.uint8, device=dev)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    s_codec = torch.cuda.Stream(device=dev)

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def codec_alone():
        e0, e1 = ev(), ev()
        with torch.cuda.stream(s_codec):
            e0.record()
            D.codec_dev("g1_decompress", comp, out, key)
            e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    def copies_alone(s):
        ts = []
        with torch.cuda.stream(s):
            for _ in range(a.copies):
                e0, e1 = ev(), ev()
                e0.record()
                dst.copy_(src)
                e1.record()
                ts.append((e0, e1))
        torch.cuda.synchronize()
        return [x.elapsed_time(y) for x, y in ts]

    def together(s):
        c0, c1 = ev(), ev()
        ts = []
        with torch.cuda.stream(s_codec):
            c0.record()
            D.codec_dev("g1_decompress", comp, out, key)
            c1.record()
        with torch.cuda.stream(s):
            for _ in range(a.copies):
                e0, e1 = ev(), ev()
                e0.record()
                dst.copy_(src)
                e1.record()
                ts.append((e0, e1))
        torch.cuda.synchronize()
        return c0.elapsed_time(c1), [x.elapsed_time(y) for x, y in ts], c0.elapsed_time(ts[-1][1])

    codec_alone()  # warm-up: clocks, code object
    res = {"points": n, "copy_bytes": nb, "copies": a.copies, "priority_range": [lo, hi],
           "codec_alone_ms": codec_alone(), "runs": {}}
    for name, prio in (("normal", 0), ("highest", hi)):
        s = torch.cuda.Stream(device=dev, priority=prio)
        copies_alone(s)
        alone = copies_alone(s)
        c_ms, c_each, last_copy_done = together(s)
        res["runs"][name] = {"stream_priority": prio, "copy_alone_ms": alone, "codec_with_copies_ms": c_ms,
                             "copy_beside_codec_ms": c_each,
                             "last_copy_done_after_codec_start_ms": last_copy_done}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
