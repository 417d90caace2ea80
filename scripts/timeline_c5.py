#!/usr/bin/env python3
"""Timeline of a rocprofv3 --kernel-trace CSV: trace launches and BLAS-rebuild kernels per queue (C5 pipeline study).
usage: scripts/timeline_c5.py kernel_trace.csv [last_ms]"""
import csv
import sys


def short(n):
    n = n.split("(")[0]
    for k in ("render_persistent_kernel", "rocprim", "lbvh::", "rtamd::"):
        if k in n:
            return n.split("::")[-1][:28] if k != "rocprim" else "rocprim_sort"
    return n[-28:]


rows = list(csv.DictReader(open(sys.argv[1])))
last = float(sys.argv[2]) if len(sys.argv) > 2 else 60.0
key_q = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get(key_q, "?")) for r in rows]
ev.sort()
t_end = max(e[1] for e in ev)
t0 = t_end - last * 1e6
traces = [e for e in ev if "render_persistent" in e[2]]
print(f"{len(ev)} dispatches, {len(traces)} trace launches; last {last} ms (t=0 at {t0})")
for s, e, n, q in ev:
    if e < t0:
        continue
    if n.startswith("fill") or "fillBuffer" in n or "copyBuffer" in n:
        continue
    print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e3:9.1f} us  q{q:>3}  {n}")
# busy fractions in the window: time with >= 1 trace running, with a rebuild kernel running, with both
import numpy as np
grid = np.arange(t0, t_end, 10_000)   # 10 us
tr = np.zeros(len(grid), bool)
rb = np.zeros(len(grid), bool)
for s, e, n, q in ev:
    m = (grid >= s) & (grid < e)
    if "render_persistent" in n:
        tr |= m
    elif not ("fill" in n or "copy" in n):
        rb |= m
print(f"window: trace running {tr.mean():.2f}, rebuild kernels running {rb.mean():.2f}, both {(tr & rb).mean():.2f}, "
      f"neither {(~tr & ~rb).mean():.2f}")
