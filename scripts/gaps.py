#!/usr/bin/env python3
"""Inter-kernel gaps per hardware queue from a rocprofv3 kernel trace: frame_copy / schedule -> render.
usage: gaps.py run_kernel_trace.csv"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
byq = collections.defaultdict(list)
for r in rows:
    byq[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
gaps = []
for v in byq.values():
    v.sort()
    for a, b in zip(v, v[1:]):
        if "render_persistent" in b[2] and ("frame_copy" in a[2] or "schedule" in a[2]):
            gaps.append((b[0] - a[1]) / 1e3)
gaps.sort()
print({"copy_to_render_gaps": len(gaps), "median_us": round(statistics.median(gaps), 2),
       "p10_us": round(gaps[len(gaps) // 10], 2), "p90_us": round(gaps[9 * len(gaps) // 10], 2)})
