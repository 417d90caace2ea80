#!/bin/bash
# r05 session 21: kernel trace of C5 with the per-frame rebuild (which kernels sit on a frame's critical path)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s21; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- \
    python3 bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
tail -1 $O/kt.log | cut -c1-200
f=$(find $O/kt -name '*kernel_trace.csv' | head -1)
python3 - "$f" > $O/kt_summary.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
# keep the last ~60 ms
tend = max(int(r["End_Timestamp"]) for r in rows)
keep = ("prep_blas", "gather_blas", "render_persistent", "karras", "collapse_all", "tlas_small", "bottom_up_chunk")
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = r["Kernel_Name"].split("(")[0][-48:]
    if not any(k in n for k in keep): continue
    print(f"{(s - t0)/1e3:12.1f} {(e - s)/1e3:9.1f} q{r.get('Queue_Id', r.get('Stream_Id','?'))} {n}")
PY
wc -l $O/kt_summary.txt
rm -f "$f"
