#!/usr/bin/env python3
# When the host enqueues each lane's next frame vs when the lane's previous trace ended (rocprofv3 --hip-trace
# --kernel-trace of scripts/r03_share_hiptrace.sh; reads gpurun_out/st/ht_share/)
import csv,collections,numpy as np
api=list(csv.DictReader(open("gpurun_out/st/ht_share/run_hip_api_trace.csv")))
kt=list(csv.DictReader(open("gpurun_out/st/ht_share/run_kernel_trace.csv")))
def short(n):
    for k in ("render_persistent","frame_copy","schedule_kernel","copyBuffer","fillBuffer"):
        if k in n: return k
    return n[:25]
kmap={r["Correlation_Id"]:r for r in kt}
launches=[]
for r in api:
    if r["Function"]=="hipLaunchKernel" and r["Correlation_Id"] in kmap:
        k=kmap[r["Correlation_Id"]]
        launches.append(dict(name=short(k["Kernel_Name"]),q=k["Queue_Id"],a0=int(r["Start_Timestamp"]),a1=int(r["End_Timestamp"]),g0=int(k["Start_Timestamp"]),g1=int(k["End_Timestamp"])))
launches.sort(key=lambda x:x["a0"])
tr=[l for l in launches if l["name"]=="render_persistent"]
timed=tr[-241:-41]
t0=min(l["a0"] for l in timed)-200000; t1=max(l["g1"] for l in timed)
win=[l for l in launches if t0<=l["a0"]<=t1]
for nm in ("render_persistent","frame_copy","schedule_kernel"):
    d=np.array([(l["a1"]-l["a0"])/1e3 for l in win if l["name"]==nm])
    if len(d): print(f"{nm:20s} api us mean {d.mean():6.2f} p50 {np.median(d):6.2f} p90 {np.percentile(d,90):6.2f} max {d.max():7.1f}")
# per lane: previous render end (GPU) vs host api start of next small kernel on same queue
byq=collections.defaultdict(list)
for l in win: byq[l["q"]].append(l)
A=[];B=[];C=[]
for q,v in byq.items():
    v.sort(key=lambda x:x["a0"])
    prev=None
    for i,l in enumerate(v):
        if l["name"]!="render_persistent":
            if prev: A.append((l["a0"]-prev["g1"])/1e3); B.append((l["g0"]-max(l["a1"],prev["g1"]))/1e3)
        else:
            prev=l
for nm,x in (("host enqueues small after prev trace end (us, <0 = ahead)",A),("small GPU start after max(enqueue, prev end)",B)):
    x=np.array(x); print(nm, "mean %.1f p10 %.1f p50 %.1f p90 %.1f"%(x.mean(),np.percentile(x,10),np.median(x),np.percentile(x,90)))
# host frame period
rs=[l["a0"] for l in timed]; print("host render-launch period us", np.diff(rs).mean()/1e3)
