#!/usr/bin/env python3
# Per-lane gaps between trace launches of a one-GPU 1/8 share run from a rocprofv3 --kernel-trace CSV:
#   python scripts/share_gaps.py gpurun_out/st/kt_share/run_kernel_trace.csv   (scripts/r03_share_trace.sh)
import csv,sys,collections,numpy as np
rows=list(csv.DictReader(open(sys.argv[1])))
def short(n):
    for k in ("render_persistent","frame_copy","schedule_kernel","copyBuffer","fillBuffer","instance","assemble"):
        if k in n: return k
    return n[:30]
ks=sorted([(int(r["Start_Timestamp"]),int(r["End_Timestamp"]),short(r["Kernel_Name"]),r["Queue_Id"],int(r["Grid_Size_X"])) for r in rows])
tr=[k for k in ks if k[2]=="render_persistent"]
timed=tr[-241:-41]
t0=min(k[0] for k in timed); t1=max(k[1] for k in timed)
win=[k for k in ks if k[0]>=t0-1 and k[1]<=t1+1]
print("timed span us", (t1-t0)/1e3, "per frame", (t1-t0)/1e3/200, "kernels in window", collections.Counter(k[2] for k in win))
byq=collections.defaultdict(list)
for k in win: byq[k[3]].append(k)
st=collections.defaultdict(list)
for q,v in byq.items():
    prev=None; small=[]
    for k in v:
        if k[2]=="render_persistent":
            if prev is not None:
                st["gap_total"].append(k[0]-prev[1])
                if small:
                    st["end->small_start"].append(small[0][0]-prev[1]); st["small_dur"].append(small[-1][1]-small[0][0]); st["small_end->render"].append(k[0]-small[-1][1])
                    st["n_small"].append(len(small))
            st["render_dur"].append(k[1]-k[0]); st["grid"].append(k[4]*1000//256)
            prev=k; small=[]
        else: small.append(k)
for k,v in st.items():
    v=np.array(v)/1000.0
    print(f"{k:20s} n={len(v):4d} mean {v.mean():8.2f} p10 {np.percentile(v,10):8.2f} p50 {np.median(v):8.2f}  p90 {np.percentile(v,90):8.2f}")
ev=sorted([(k[0],1) for k in timed]+[(k[1],-1) for k in timed])
c=0;last=ev[0][0];acc=0;hist=collections.Counter()
for x,d in ev: acc+=c*(x-last); hist[c]+=x-last; last=x; c+=d
print("in_flight_mean %.2f"%(acc/(t1-t0)), {k:round(v/(t1-t0),3) for k,v in sorted(hist.items())})
# what else runs: other kernels' count in window by queue
