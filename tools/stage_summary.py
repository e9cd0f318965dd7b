"""Per-stage breakdown of the end-to-end preprocess calls from one rocprofv3 run with
--marker-trace --kernel-trace --memory-copy-trace (tools/e2e_breakdown.py is the traced program).

    python3 tools/stage_summary.py TRACE_DIR calls.json > profiles/<tag>_e2e_stages.json

For every C-ABI call (the library's roctx range "kzgpot.preprocess", matched in order with the
calls tools/e2e_breakdown.py timed) it reports:
  * `critical_path_ms`: the call cut at the instants its stages hand over — setup (before the first
    section starts), each section's span (first shard thread in to last shard thread out: H2D
    staging, kernels, D2H of that section), the gaps between sections, and the drain after the
    last section (the digests and the writer finishing) — segments that add up to the call;
  * `busy_ms`: per stage, the union of its intervals inside the call (stages overlap: the digest
    threads and the writer run beside the GPU pass), with the GPU's kernel time and the H2D / D2H
    copy time from the kernel and memory-copy traces;
  * `last_to_finish`: the stage whose range ends last before the call returns — the critical path.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys


def find(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    return hits[-1] if hits else None


def rows(path):
    if not path:
        return []
    with open(path) as f:
        return list(csv.DictReader(f))


def col(r, *names):
    for n in names:
        if n in r and r[n] not in (None, ""):
            return r[n]
    return None


def union_ms(iv, lo, hi):
    """Total length of the union of intervals clipped to [lo, hi), in ms (timestamps in ns)."""
    segs = sorted((max(a, lo), min(b, hi)) for a, b in iv if b > lo and a < hi)
    tot, cur_a, cur_b = 0, None, None
    for a, b in segs:
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                tot += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        tot += cur_b - cur_a
    return tot / 1e6


def short_kernel(name):
    m = re.search(r"(k_\w+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:48]


def main():
    d, calls_path = sys.argv[1], sys.argv[2]
    calls = json.load(open(calls_path))
    markers = []
    for r in rows(find(d, "marker_api_trace.csv")):
        name = col(r, "Function", "Message", "Operation")
        a, b = col(r, "Start_Timestamp"), col(r, "End_Timestamp")
        if name and a and b:
            markers.append((name, int(col(r, "Thread_Id") or 0), int(a), int(b)))
    kernels = [(short_kernel(col(r, "Kernel_Name") or ""), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
               for r in rows(find(d, "kernel_trace.csv"))]
    copies = []
    for r in rows(find(d, "memory_copy_trace.csv")):
        direction = (col(r, "Direction", "Operation", "Kind") or "").upper()
        kind = "h2d" if "HOST_TO_DEVICE" in direction else "d2h" if "DEVICE_TO_HOST" in direction else "other"
        copies.append((kind, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    tops = sorted((m for m in markers if m[0] == "kzgpot.preprocess"), key=lambda m: m[2])
    want = calls["calls"]
    tops = tops[-len(want):]  # the first one is e2e_breakdown.py's warm-up call
    out = {"source": "rocprofv3 --marker-trace --kernel-trace --memory-copy-trace of tools/e2e_breakdown.py",
           "n_log2": calls["n_log2"], "shards": calls["shards"],
           "blake2b_transcript_alone_s": calls["blake2b_transcript_alone_s"], "calls": []}
    for call, (_, tid, s, e) in zip(want, tops):
        inside = [m for m in markers if m[3] > s and m[2] < e and m[0] != "kzgpot.preprocess"]
        names = sorted({m[0] for m in inside})
        busy = {n: round(union_ms([(m[2], m[3]) for m in inside if m[0] == n], s, e), 3) for n in names}
        busy["gpu.kernels"] = round(union_ms([(a, b) for _, a, b in kernels], s, e), 3)
        per_kernel = {}
        for k, a, b in kernels:
            if b > s and a < e:
                per_kernel[k] = per_kernel.get(k, 0) + (min(b, e) - max(a, s)) / 1e6
        for kind in ("h2d", "d2h"):
            busy[f"gpu.copy.{kind}"] = round(union_ms([(a, b) for k, a, b in copies if k == kind], s, e), 3)
        sections = {}
        for m in inside:
            if m[0].startswith("kzgpot.section."):
                a, b = sections.get(m[0], (m[2], m[3]))
                sections[m[0]] = (min(a, m[2]), max(b, m[3]))
        path, t = [], s
        for name, (a, b) in sorted(sections.items(), key=lambda kv: kv[1][0]):
            a, b = max(a, s), min(b, e)
            if a > t:
                path.append(["setup" if t == s else "between sections", (a - t) / 1e6])
            path.append([name.replace("kzgpot.", ""), (b - max(a, t)) / 1e6])
            t = max(t, b)
        path.append(["after the last section (digest / writer drain)", (e - t) / 1e6])
        enders = sorted(((m[3], m[0]) for m in inside if m[3] <= e), reverse=True)
        # file calls: kzgpot_preprocess_ex's own range around preprocess_impl (open + mapping the
        # buffers before it; closing, renaming and unmapping after it)
        outer = [m for m in markers if m[0] == "kzgpot.preprocess_file" and m[2] <= s and m[3] >= e]
        file_part = None
        if outer:
            o = outer[0]
            fin = [m for m in markers if m[0] == "kzgpot.file_finish" and o[2] <= m[2] <= o[3]]
            file_part = {"file_call_ms": (o[3] - o[2]) / 1e6, "before_pipeline_ms": (s - o[2]) / 1e6,
                         "after_pipeline_ms": (o[3] - e) / 1e6,
                         "file_finish_ms": sum(m[3] - m[2] for m in fin) / 1e6}
        out["calls"].append({
            "call": call["call"], "seconds_timed_by_caller": call["seconds"], "rc": call["rc"],
            "range_ms": (e - s) / 1e6,
            "critical_path_ms": [[n, round(v, 3)] for n, v in path],
            "critical_path_sum_ms": round(sum(v for _, v in path), 3),
            "busy_ms": busy, "kernel_ms": {k: round(v, 3) for k, v in sorted(per_kernel.items(), key=lambda kv: -kv[1])},
            "last_to_finish": enders[0][1] if enders else None,
            "last_to_finish_before_end_ms": round((e - enders[0][0]) / 1e6, 3) if enders else None,
            "file": file_part,
        })
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
