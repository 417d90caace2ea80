#!/bin/bash
# r05 session 41: per-kernel cost of the C5 rebuild alone (fused gather library), rocprofv3 kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s41; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/rebuild_alone.py --config C5 --updates 20 > $O/alone.log 2>&1 || { echo fail; tail -5 $O/alone.log; exit 1; }
tail -1 $O/alone.log
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
python3 - $O/kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:25]:
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.1f} total_ms {float(r['TotalDurationNs'])/1e6:8.2f}")
PY
rm -rf $O/prof
