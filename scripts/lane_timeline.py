#!/usr/bin/env python3
"""How the overlapped lanes' trace launches interleave (bench.py --launch-times out.npy, L lanes).

    python scripts/lane_timeline.py out.npy L

Launch j ran on lane j % L.  Prints the mean launch duration, each lane's idle gap between its launches
(stop of launch j-L to start of launch j), the time-average number of launches in flight, and the frame
period (span / launches)."""
import json
import sys

import numpy as np

t = np.load(sys.argv[1]).astype(np.float64)
L = int(sys.argv[2])
n = len(t)
dur = t[:, 1] - t[:, 0]
gaps = [t[j, 0] - t[j - L, 1] for j in range(L, n)]
ev = sorted([(a, 1) for a in t[:, 0]] + [(b, -1) for b in t[:, 1]])
inflight, last, acc, c = 0, ev[0][0], 0.0, 0
hist = {}
for x, d in ev:
    hist[c] = hist.get(c, 0.0) + (x - last)
    acc += c * (x - last)
    last = x
    c += d
span = t[:, 1].max() - t[:, 0].min()
print(json.dumps({"launches": n, "lanes": L, "span_ms": round(span, 4), "ms_per_launch": round(span / n, 4),
                  "launch_ms_mean": round(float(dur.mean()), 4), "launch_ms_p90": round(float(np.percentile(dur, 90)), 4),
                  "lane_gap_ms_mean": round(float(np.mean(gaps)), 4) if gaps else None,
                  "lane_gap_ms_p90": round(float(np.percentile(gaps, 90)), 4) if gaps else None,
                  "in_flight_mean": round(acc / span, 3),
                  "in_flight_hist": {k: round(v / span, 3) for k, v in sorted(hist.items())}}))
