#!/usr/bin/env python3
"""Collect scripts/r03_final.sh / r04_final.sh output (gpurun_out/$FINAL_SRC, default final/) into profiles/:

    python scripts/collect_final.py [OUTDIR=profiles/r03_final]

* profiles/pmc/<config>_<build>[_rebuild].json   the tagged PMC summaries bench.py prices `traffic` with
* OUTDIR/bench_<tag>.json, serial_<tag>.json      the bench lines (pipelined default, serialised --overlap 1)
* OUTDIR/serial_profiled_<tag>.json                the serialised line the rocprofv3-wrapped run printed (the same
                                                   launches its kernel stats average: the summary compares these)
* OUTDIR/kstats_<tag>.csv                          rocprofv3 --kernel-trace --stats of the serialised command
* OUTDIR/summary.json                              per config: frac of the line, frac recomputed from the rocprof
                                                   average (algorithmic bytes / rocprof mean duration / 8 TB/s), the
                                                   measured HBM bytes per launch and their fraction of peak
"""
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "gpurun_out", os.environ.get("FINAL_SRC", "final"))
OUT = os.path.join(REPO, sys.argv[1] if len(sys.argv) > 1 else "profiles/r03_final")
PEAK = 8000.0


def line(path):
    with open(path) as f:
        for ln in f:
            if ln.startswith('{"metric"'):
                return json.loads(ln)
    return None


def main():
    os.makedirs(OUT, exist_ok=True)
    os.makedirs(os.path.join(REPO, "profiles", "pmc"), exist_ok=True)
    summary = {}
    for log in sorted(glob.glob(os.path.join(SRC, "serial_*.log"))):
        tag = os.path.basename(log)[len("serial_"):-4]
        ser = line(log)
        pipe = line(os.path.join(SRC, f"bench_{tag}.log"))
        for name, d in (("serial", ser), ("bench", pipe)):
            if d is not None:
                with open(os.path.join(OUT, f"{name}_{tag}.json"), "w") as f:
                    json.dump(d, f, indent=1)
        stats = glob.glob(os.path.join(SRC, f"kstats_{tag}", "**", "*kernel_stats.csv"), recursive=True)
        rp_avg_ms = None
        if stats:
            shutil.copy(stats[0], os.path.join(OUT, f"kstats_{tag}.csv"))
            import csv
            with open(stats[0]) as f:
                for r in csv.DictReader(f):
                    if "render_persistent_kernel<false" in r["Name"]:
                        rp_avg_ms = float(r["AverageNs"]) / 1e6
                        rp_calls = int(r["Calls"])
        pmc = os.path.join(SRC, f"pmc_{tag}", "summary.json")
        pmc_dst = None
        if os.path.exists(pmc):
            with open(pmc) as f:
                p = json.load(f)
            t = p["tag"]
            pmc_dst = os.path.join(REPO, "profiles", "pmc",
                                   f"{t['config']}_{t['build']}{'_rebuild' if t['rebuild'] else ''}"
                                   f"{'_exact' if t['exact'] else ''}{'' if t['kernel'] else '_grid'}.json")
            shutil.copy(pmc, pmc_dst)
        # the bench line printed by the rocprofv3-wrapped command itself: the very launches rocprof averaged
        prof = line(os.path.join(SRC, f"kstats_{tag}.log"))
        if prof is not None:
            with open(os.path.join(OUT, f"serial_profiled_{tag}.json"), "w") as f:
                json.dump(prof, f, indent=1)
            ser = prof
        roof = ser["roofline"] if ser else None
        s = {"config": ser["config"]["workload"] if ser else None}
        if roof:
            ab = roof["algorithmic_bytes_per_launch"]
            s.update({"algorithmic_bytes_per_launch": ab, "kernel_ms_line": ser["kernel_ms"], "frac_line": roof["frac"]})
            if rp_avg_ms:
                fr = ab / (rp_avg_ms * 1e-3) / 1e9 / PEAK
                s.update({"rocprof_avg_ms": round(rp_avg_ms, 4), "rocprof_calls": rp_calls, "frac_rocprof": round(fr, 4),
                          "frac_rel_diff": round(roof["frac"] / fr - 1.0, 4)})
            if os.path.exists(pmc):
                hb = p["hbm_bytes_per_launch"]
                s.update({"hbm_bytes_per_launch": hb, "fetch_bytes_corrected": int(p["fetch_bytes_per_launch_corrected"]),
                          "write_bytes": int(p["write_bytes_per_launch"]),
                          "hbm_frac_measured_at_rocprof_avg": round(hb / (rp_avg_ms * 1e-3) / 1e9 / PEAK, 5) if rp_avg_ms else None,
                          "pmc_summary": os.path.relpath(pmc_dst, REPO)})
        if pipe:
            s.update({"pipelined_ms_per_frame": pipe["ms_per_step"], "pipelined_mrays_s": pipe["value"],
                      "latency_ms": pipe["frame_latency_ms_median"], "pipelined_line_frac": pipe["roofline"]["frac"],
                      "pipelined_line_traffic": pipe["roofline"]["traffic"], "pipelined_line_limiter": pipe["roofline"]["limiter"]})
        summary[tag] = s
    with open(os.path.join(OUT, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
