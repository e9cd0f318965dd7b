"""Per-(kernel, grid size) duration summary of a rocprofv3 --kernel-trace CSV.

    python tools/trace_summary.py run_kernel_trace.csv [--out profiles/r01_kernel_by_size.csv]

rocprofv3's --stats averages every dispatch of a kernel together; the default bench command also
runs the codec kernels at the end-to-end preprocess sizes (2^21-2^23 points), so the headline
2^27-point launches are split out here to compare with bench.py's event-timed `launch_ms`.
"""
from __future__ import annotations

import argparse
import collections
import csv
import re


def short(name: str) -> str:
    m = re.search(r"(k_\w+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out")
    a = ap.parse_args()
    per = collections.defaultdict(list)
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            per[(short(r["Kernel_Name"]), grid)].append(dur)
    rows = [("kernel", "grid_threads", "calls", "avg_ms", "min_ms", "max_ms")]
    for (k, g), d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        rows.append((k, g, len(d), f"{sum(d) / len(d) / 1e6:.3f}", f"{min(d) / 1e6:.3f}", f"{max(d) / 1e6:.3f}"))
    if a.out:
        with open(a.out, "w", newline="") as f:
            csv.writer(f).writerows(rows)
    for r in rows[:16]:
        print(",".join(str(x) for x in r))


if __name__ == "__main__":
    main()
