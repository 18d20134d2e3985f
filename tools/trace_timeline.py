"""Prints the tail of a rocprofv3 kernel trace as a per-queue timeline (start, end,
duration in us relative to the first printed kernel), and the mean gap between
consecutive kernels of each queue.

    python tools/trace_timeline.py <run_kernel_trace.csv> [count]
"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    m = re.search(r"(k_[a-z_]+)", n)
    return m.group(1) if m else n[:24]


rows = list(csv.DictReader(open(sys.argv[1])))
count = int(sys.argv[2]) if len(sys.argv) > 2 else 30
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]) for r in rows)
t0 = ev[-count][0]
for s, e, n, q in ev[-count:]:
    print(f"{(s - t0) / 1000:9.1f} {(e - t0) / 1000:9.1f} {(e - s) / 1000:7.1f} q{q} {n}")
gaps = defaultdict(list)
last = {}
for s, e, n, q in ev[-count:]:
    if q in last:
        gaps[(q, last[q][1], n)].append((s - last[q][0]) / 1000)
    last[q] = (e, n)
for (q, a, b), g in sorted(gaps.items()):
    print(f"q{q} {a} -> {b}: mean gap {sum(g) / len(g):.1f} us over {len(g)}")
