#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs for the trace kernel into profiles/pmc_latest.json.

Usage: pmc_summary.py OUT.json KERNEL_SUBSTRING DIR [DIR ...]
Each DIR holds one rocprofv3 pass (*counter_collection.csv).  Per-dispatch values are summed
over the counter's instances (XCDs / channels) and averaged over dispatches of the kernel.
HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KB;
on gfx950 FETCH_SIZE reads half the bytes of a wide coalesced stream, so it is doubled.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirs, kernel_sub):
    per = defaultdict(lambda: defaultdict(float))   # counter -> dispatch -> value
    names = set()
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    kn = row.get("Kernel_Name", "")
                    if kernel_sub not in kn:
                        continue
                    names.add(kn)
                    disp = (path, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                    per[row["Counter_Name"]][disp] += float(row["Counter_Value"])
    avg = {c: sum(v.values()) / len(v) for c, v in per.items() if v}
    ndisp = {c: len(v) for c, v in per.items()}
    return avg, ndisp, sorted(names)


def main():
    argv = sys.argv[1:]
    tag = cmd = None
    if "--tag" in argv:
        i = argv.index("--tag")
        with open(argv[i + 1]) as f:
            tag = json.load(f)                    # bench.py --print-pmc-tag: the workload these counters price
        del argv[i:i + 2]
    if "--cmd" in argv:
        i = argv.index("--cmd")
        cmd = argv[i + 1]
        del argv[i:i + 2]
    out, kernel_sub, dirs = argv[0], argv[1], argv[2:]
    avg, ndisp, names = load(dirs, kernel_sub)
    res = {"kernel": names[0] if names else kernel_sub, "kernels_matched": names, "counters_avg_per_dispatch": avg,
           "dispatches": ndisp, "source_dirs": dirs}
    if tag is not None:
        res["tag"] = tag
    if cmd is not None:
        res["command"] = cmd
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        res["fetch_bytes_per_launch_corrected"] = 2.0 * avg["FETCH_SIZE"] * 1024.0
        res["write_bytes_per_launch"] = avg["WRITE_SIZE"] * 1024.0
        res["hbm_bytes_per_launch"] = int(res["fetch_bytes_per_launch_corrected"] + res["write_bytes_per_launch"])
        res["note"] = "hbm_bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count correction)"
    a = avg
    if {"SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"} <= a.keys():
        # waves resident per CU: SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md) over 256 CUs;
        # GRBM_GUI_ACTIVE is summed over 8 XCDs
        gui = a["GRBM_GUI_ACTIVE"] / 8.0
        res["derived_waves_per_cu"] = 4.0 * a["SQ_WAVE_CYCLES"] / gui / 256.0
    if {"SQ_WAIT_ANY", "SQ_WAVE_CYCLES"} <= a.keys():
        res["derived_frac_wave_cycles_waiting"] = a["SQ_WAIT_ANY"] / a["SQ_WAVE_CYCLES"]
    if {"SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES"} <= a.keys():
        res["derived_frac_wave_cycles_valu"] = a["SQ_ACTIVE_INST_VALU"] / a["SQ_WAVE_CYCLES"]
    if {"SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU"} <= a.keys():
        res["derived_valu_lane_utilization"] = a["SQ_THREAD_CYCLES_VALU"] / (64.0 * a["SQ_ACTIVE_INST_VALU"])
    if {"SQ_THREAD_CYCLES_VALU", "SQ_INSTS_VALU"} <= a.keys():
        res["derived_active_lanes_per_valu_inst"] = a["SQ_THREAD_CYCLES_VALU"] / a["SQ_INSTS_VALU"]
    if {"TCC_HIT_sum", "TCC_MISS_sum"} <= a.keys():
        res["derived_l2_hit_rate"] = a["TCC_HIT_sum"] / max(1.0, a["TCC_HIT_sum"] + a["TCC_MISS_sum"])
    if {"TCP_TCC_READ_REQ_LATENCY_sum", "TCP_TCC_READ_REQ_sum"} <= a.keys():
        res["derived_l1_to_l2_read_latency_cycles"] = a["TCP_TCC_READ_REQ_LATENCY_sum"] / max(1.0, a["TCP_TCC_READ_REQ_sum"])
    for lvl, cnt in (("SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM"), ("SQ_INST_LEVEL_LDS", "SQ_INSTS_LDS"),
                     ("SQ_INST_LEVEL_SMEM", "SQ_INSTS_SMEM")):
        if {lvl, cnt} <= a.keys():   # level accumulates in-flight instructions per cycle -> mean latency
            res[f"derived_mean_latency_cycles_{cnt[9:].lower()}"] = a[lvl] / max(1.0, a[cnt])
    if {"SQC_ICACHE_MISSES", "SQC_ICACHE_HITS"} <= a.keys():
        res["derived_icache_miss_rate"] = a["SQC_ICACHE_MISSES"] / max(1.0, a["SQC_ICACHE_MISSES"] + a["SQC_ICACHE_HITS"])
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
