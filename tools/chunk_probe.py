"""Where does a chunked host call lose time against one device-resident launch (FFI
boundary row)? Device-resident only, no copies: 2^`--log2` points as one launch, as 2^`--chunk`-point
launches back to back on one stream, and alternating over two streams, event-timed (median of 3).

    python3 tools/chunk_probe.py [--kind g2] [--log2 20] [--chunk 17]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-setup-powersoftau_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", choices=["g1", "g2"], default="g2")
    ap.add_argument("--log2", type=int, default=20)
    ap.add_argument("--chunk", type=int, default=17)
    a = ap.parse_args()
    import torch

    from kzgpot import device as D

    dev = torch.device("cuda", 0)
    n, c = 1 << a.log2, 1 << a.chunk
    rin, rout = (48, 96) if a.kind == "g1" else (96, 192)
    comp, _ = D.synth(a.kind, 7, 0, n, dev, with_expected=False)
    out = torch.empty(n * rout, dtype=torch.uint8, device=dev)
    keys = torch.empty(n // c + 1, dtype=torch.int64, device=dev)
    op = f"{a.kind}_decompress"
    streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]

    def single():
        D.codec_dev(op, comp, out, keys[:1])

    def chunked(nstreams):
        cur = torch.cuda.current_stream()
        for s in streams[:nstreams]:
            s.wait_stream(cur)
        for j in range(n // c):
            with torch.cuda.stream(streams[j % nstreams]):
                D.codec_dev(op, comp[j * c * rin:(j + 1) * c * rin], out[j * c * rout:(j + 1) * c * rout], keys[j:j + 1])
        for s in streams[:nstreams]:
            cur.wait_stream(s)

    def host_paced(nslots, delay_s):
        """run_host's schedule without the copies: launch chunk j on stream j % nslots, then wait
        for chunk j - (nslots - 1) to finish and idle `delay_s` (its output copy and the next input
        copy: ~0.7 ms for a 2^17-point G2 chunk at 56 GB/s)."""
        import time
        cur = torch.cuda.current_stream()
        ss = [torch.cuda.Stream(device=dev) for _ in range(nslots)] if nslots > 2 else streams
        for s in ss:
            s.wait_stream(cur)
        k = n // c
        for j in range(k):
            with torch.cuda.stream(ss[j % nslots]):
                D.codec_dev(op, comp[j * c * rin:(j + 1) * c * rin], out[j * c * rout:(j + 1) * c * rout], keys[j:j + 1])
            if j >= nslots - 1:
                ss[(j - (nslots - 1)) % nslots].synchronize()
                t = time.perf_counter()
                while time.perf_counter() - t < delay_s:
                    pass
        for s in ss:
            cur.wait_stream(s)

    def timed(fn):
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return statistics.median(ts)

    single()
    torch.cuda.synchronize()
    res = {"kind": a.kind, "points": n, "chunk": c}
    res["single_ms"] = timed(single)
    res["one_stream_ms"] = timed(lambda: chunked(1))
    res["two_streams_ms"] = timed(lambda: chunked(2))
    for d in (0.0, 0.0007, 0.0015):
        res[f"host_paced_2slots_{d * 1e3:.1f}ms_ms"] = timed(lambda: host_paced(2, d))
        res[f"host_paced_3slots_{d * 1e3:.1f}ms_ms"] = timed(lambda: host_paced(3, d))
    res["single_again_ms"] = timed(single)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
