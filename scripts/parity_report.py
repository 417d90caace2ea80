#!/usr/bin/env python3
"""Full-frame parity of the benched configuration against the oracle (verdict r3 item 1), as numbers.

For C2 (1080p, 1 spp, depth 2; also at depth 1) and C3 (1080p, 4 spp, depth 4), frames 0 and 37, it renders
  * "bench":  FAST kernel, SAH trees, instance groups, quad traversal, LDS scene, 4 pipelined lanes (NO_SYNC
              frames on four streams into device buffers), i.e. bench.py's configuration;
  * "fast_compat": FAST kernel on the reference's own (median-split) trees — identical trees to the oracle's;
  * "fast_compat_binary": FAST arithmetic on those trees with the binary node-pair traversal (the reference's
              visit order), which separates arithmetic from visit-order ties;
  * "exact_compat": EXACT kernel on those trees (bit-identical by the parity tests);
  * "exact_sah" / "exact_lbvh": the EXACT kernel (the reference's traversal order and arithmetic) on the bench's
              SAH / LBVH trees — what the reference's algorithm itself renders on those trees;
  * "<mode>+opt=v+...": any of the above with extra set_option calls (e.g. "fast_compat+lds_scene=0+kernel=0")
and compares each with the oracle's frame: pixels with any RGBA8 channel |d| > 1 (outliers), max |d|, and the
per-channel float |d| of the linear RGB.  Output: one JSON object (stdout, or --out).
RTAMD_LIB selects the library (variant builds, e.g. RT_SLAB_CONS=0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "real-time-gpu-ray-tracer_amd"))


def compare(rgba, rgb, orgba, orgb):
    import numpy as np
    d = np.abs(rgba.astype(np.int32) - orgba.astype(np.int32)).max(axis=-1)
    out = {"pixels": int(d.size), "outliers_gt1": int((d > 1).sum()), "outlier_frac": float((d > 1).mean()),
           "max_lsb": int(d.max())}
    if rgb is not None:
        fd = np.abs(rgb - orgb)
        out["float_max"] = float(fd.max())
        out["float_ne"] = int((rgb != orgb).any(axis=-1).sum())
        out["float_gt_1e-3"] = int((fd.max(axis=-1) > 1e-3).sum())
    return out


def main():
    import numpy as np
    import torch
    from oracle.oracle import OracleScene
    from rtamd import Renderer, scenes
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2d1,C2,C3")
    ap.add_argument("--frames", default="0,37")
    ap.add_argument("--modes", default="bench,fast_compat,exact_compat")
    ap.add_argument("--out", default=None)
    ap.add_argument("--save-diff", default=None, help="directory: save outlier masks (npz) per case")
    ap.add_argument("--pairs", default="", help="mode pairs a:b compared with each other too (e.g. bench:exact_sah)")
    args = ap.parse_args()
    frames = [int(f) for f in args.frames.split(",")]
    res = {"lib": os.environ.get("RTAMD_LIB", "default"), "cases": []}
    torch.cuda.set_device(0)
    for cname in args.configs.split(","):
        depth_override = None
        base = cname
        if cname.endswith("d1"):
            base, depth_override = cname[:-2], 1
        cfg = scenes.CONFIGS[base]
        scene = scenes.config_scene(cfg)
        W, H = cfg.width, cfg.height
        cam = dict(sample_count=cfg.spp, ray_trace_depth=depth_override or cfg.depth)
        o = OracleScene(scene, build_seed=0)
        o.camera(W, H, **cam)
        oracle = {}
        for f in frames:
            o.update(f)
            t0 = time.time()
            orgb, orgba, _ = o.render(threads=16)
            oracle[f] = (orgb, orgba)
            print(f"oracle {cname} frame {f}: {time.time() - t0:.1f} s", flush=True)
        kept = {}
        for spec in args.modes.split(","):
            mode, *extra = spec.split("+")
            build = {"bench": "sah", "lbvh": "lbvh", "lbvh_nogroup": "lbvh", "sah_nogroup": "sah", "exact_sah": "sah",
                     "exact_lbvh": "lbvh"}.get(mode, "compat")
            r = Renderer(scene)
            if mode == "fast_compat_binary":                 # FAST arithmetic on the reference's binary visit order
                r.set_option("wide", 0)
            if mode.endswith("_nogroup"):                    # one TLAS item per particle, as the reference has them
                r.set_option("group", 0)
            for kv in extra:
                k, v = kv.split("=")
                r.set_option(k, int(v))
            r.build_acceleration_structure(0, mode=build).configure_camera(W, H, **cam)
            got = {}
            if mode == "bench":
                L = 4
                r.set_option("overlap", L)
                lanes = [torch.cuda.Stream(priority=0) for _ in range(L)]
                last = max(frames)
                seq = list(range(0, last + 1))
                rgba_buf = {f: torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda") for f in frames}
                rgb_buf = {f: torch.zeros(W * H * 3, dtype=torch.float32, device="cuda") for f in frames}
                scratch = [torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda") for _ in range(L)]
                for k, f in enumerate(seq):
                    fb = rgba_buf[f] if f in rgba_buf else scratch[k % L]
                    r.render(f, want_rgba=False, rgba8_device=fb.data_ptr(),
                             rgb32_device=rgb_buf[f].data_ptr() if f in rgb_buf else None,
                             stream=lanes[k % L].cuda_stream, sync=False)
                r.synchronize()
                torch.cuda.synchronize()
                for f in frames:
                    got[f] = (rgba_buf[f].cpu().numpy().reshape(H, W, 4), rgb_buf[f].cpu().numpy().reshape(H, W, 3))
            else:
                for f in frames:
                    rgba, rgb, _ = r.render(f, exact=mode.startswith("exact"), want_rgb=True)
                    got[f] = (rgba, rgb)
            r.cleanup()
            kept[spec] = got
            for f in frames:
                c = compare(got[f][0], got[f][1], oracle[f][1], oracle[f][0])
                c.update({"config": cname, "mode": spec, "frame": f, "depth": cam["ray_trace_depth"], "spp": cfg.spp})
                res["cases"].append(c)
                print(json.dumps(c), flush=True)
                if args.save_diff:
                    os.makedirs(args.save_diff, exist_ok=True)
                    d = np.abs(got[f][0].astype(np.int32) - oracle[f][1].astype(np.int32)).max(axis=-1)
                    np.savez_compressed(os.path.join(args.save_diff, f"{cname}_{spec}_{f}.npz"),
                                        yx=np.argwhere(d > 1).astype(np.int32), d=d[d > 1].astype(np.int32))
        for pr in filter(None, args.pairs.split(",")):
            a, b = pr.split(":")
            for f in frames:
                c = compare(kept[a][f][0], kept[a][f][1], kept[b][f][0], kept[b][f][1])
                c.update({"config": cname, "mode": f"{a} vs {b}", "frame": f, "depth": cam["ray_trace_depth"], "spp": cfg.spp})
                res["cases"].append(c)
                print(json.dumps(c), flush=True)
    s = json.dumps(res, indent=1)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(s)
    else:
        print(s)


if __name__ == "__main__":
    main()
