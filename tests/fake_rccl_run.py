"""World > 1 multi-GPU frames on one GPU through the fake RCCL (tests/fake_rccl/fake_rccl.hip).

Run by tests/test_gpu_fake_rccl.py in a child process with RTAMD_RCCL_LIB set (the library resolves RCCL once
per process).  Every rank is a scene of its own on device 0, driven from this thread in the order a real world's
ranks would post their work (senders first, rank 0 last, the same lane sequence on every rank).  The library's
world > 1 branch runs as on 8 GPUs: rank r traces its interleaved tiles into its lane's slab and sends it to
rank 0 (grouped ncclSend / ncclRecv), rank 0 receives the slabs into its lane's gather buffer and assembles the
frame (csrc/rt_api.cpp rt_render).  Prints one JSON line per case; exits non-zero on the first failure.
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "real-time-gpu-ray-tracer_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rtamd import Renderer, abi, scenes  # noqa: E402

W, H, DEPTH, TILE, F = 320, 192, 2, 32, 24


def make(scene):
    return Renderer(scene).build_acceleration_structure(0, mode="sah").configure_camera(W, H, ray_trace_depth=DEPTH)


def world(scene, n, lanes=1, ncomm=1, sync=True):
    """Frames 0..F-1 of an n-rank world; ncomm = lanes in use at attach (one communicator each), lanes >
    ncomm shares them (lane q uses communicator q % ncomm)."""
    rs = [make(scene) for _ in range(n)]
    cid = Renderer.comm_unique_id()
    for k, r in enumerate(rs):
        if ncomm > 1:
            r.set_option("overlap", ncomm)
        r.attach_comm(cid, k, n, TILE, TILE)
        r.set_comm_timeout(20000)
        if lanes != ncomm:
            r.set_option("overlap", lanes if lanes > 1 else 0)
    out = []
    if sync:
        for f in range(F):
            for k in reversed(range(n)):
                rgba, _, st = rs[k].render(f)
                if k == 0:
                    out.append(rgba)
    else:
        streams = [[torch.cuda.Stream() for _ in range(lanes)] for _ in range(n)]
        bufs = [torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda") for _ in range(F)]
        torch.cuda.synchronize()
        for f in range(F):
            for k in reversed(range(n)):
                rs[k].render(f, want_rgba=False, rgba8_device=bufs[f].data_ptr() if k == 0 else None,
                             stream=streams[k][f % lanes].cuda_stream, sync=False)
        for r in rs:
            r.synchronize()
        torch.cuda.synchronize()
        out = [b.cpu().numpy().reshape(H, W, 4) for b in bufs]
    for r in rs:
        r.cleanup()
    return out


def world_c4(n=8, lanes=8, frames=(0, 37)):
    """bench.py's N > 1 configuration at C4's real size (verdict r4 item 4): the C3 scene at 1920x1080, 1 spp, depth 2,
    32x32 tiles over n ranks, 8 lanes (one communicator each, attached after "overlap"), stage_depth 64, every lane
    on a new stream, frames 0..max(frames) pipelined with RT_RENDER_NO_SYNC; rank 0's kept frames against
    single-launch frames of a plain scene."""
    cfg = scenes.CONFIGS["C4"]
    scene = scenes.config_scene(cfg)
    cam = dict(sample_count=cfg.spp, ray_trace_depth=cfg.depth)
    Wc, Hc = cfg.width, cfg.height
    ref_r = Renderer(scene).build_acceleration_structure(0, mode="sah").configure_camera(Wc, Hc, **cam)
    ref = {f: ref_r.render(f)[0] for f in frames}
    ref_r.cleanup()
    rs = [Renderer(scene).build_acceleration_structure(0, mode="sah").configure_camera(Wc, Hc, **cam) for _ in range(n)]
    cid = Renderer.comm_unique_id()
    for k, r in enumerate(rs):
        r.set_option("overlap", lanes)
        r.set_option("stage_depth", 64)
        r.attach_comm(cid, k, n, TILE, TILE)
        r.set_comm_timeout(60000)
    streams = [[torch.cuda.Stream(priority=0) for _ in range(lanes)] for _ in range(n)]
    keep = {f: torch.zeros(Wc * Hc * 4, dtype=torch.uint8, device="cuda") for f in frames}
    scratch = [torch.zeros(Wc * Hc * 4, dtype=torch.uint8, device="cuda") for _ in range(lanes)]
    torch.cuda.synchronize()
    t0 = time.time()
    for f in range(max(frames) + 1):
        buf = keep[f] if f in keep else scratch[f % lanes]
        for k in reversed(range(n)):
            rs[k].render(f, want_rgba=False, rgba8_device=buf.data_ptr() if k == 0 else None,
                         stream=streams[k][f % lanes].cuda_stream, sync=False)
    for r in rs:
        r.synchronize()
    torch.cuda.synchronize()
    bad = [f for f in frames if not np.array_equal(keep[f].cpu().numpy().reshape(Hc, Wc, 4), ref[f])]
    for r in rs:
        r.cleanup()
    return bad, time.time() - t0


def world_c5(n=8, frames=(0, 5)):
    """bench.py's N > 1 configuration of C5 (verdict r5 item 1): 10 M triangles at 3840x2160, 8 -> 4 traced spp, depth 2,
    the GPU LBVH with every BLAS and the TLAS rebuilt each frame ("rebuild" set before the build, as bench.py does:
    no cold records), the scene's own lanes ("overlap" -1 before the attach: 8 communicators; with the rebuild the
    library runs 2 lanes), 32x32 tiles over n ranks, frames 0..max(frames) pipelined with RT_RENDER_NO_SYNC and no
    caller stream — the scene stream's rebuilds, the lane streams' traces and the communicators' sends / receives all
    in flight together; rank 0's kept frames against single-launch frames of a scene built and rebuilt the same way."""
    cfg = scenes.CONFIGS["C5"]
    scene = scenes.config_scene(cfg)
    cam = dict(sample_count=cfg.spp, ray_trace_depth=cfg.depth)
    Wc, Hc = cfg.width, cfg.height

    def c5_scene():
        r = Renderer(scene)
        r.set_option("rebuild", 1)
        return r.build_acceleration_structure(0, mode="lbvh").configure_camera(Wc, Hc, **cam)

    ref_r = c5_scene()
    ref = {f: ref_r.render(f)[0] for f in frames}
    ref_r.cleanup()
    rs = [c5_scene() for _ in range(n)]
    cid = Renderer.comm_unique_id()
    for k, r in enumerate(rs):
        r.set_option("overlap", -1)
        r.attach_comm(cid, k, n, TILE, TILE)
        r.set_comm_timeout(120000)
    keep = {f: torch.zeros(Wc * Hc * 4, dtype=torch.uint8, device="cuda") for f in frames}
    scratch = [torch.zeros(Wc * Hc * 4, dtype=torch.uint8, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    t0 = time.time()
    for f in range(max(frames) + 1):
        buf = keep[f] if f in keep else scratch[f % 2]
        for k in reversed(range(n)):
            rs[k].render(f, want_rgba=False, rgba8_device=buf.data_ptr() if k == 0 else None, sync=False)
    for r in rs:
        r.synchronize()
    torch.cuda.synchronize()
    dt = time.time() - t0
    lanes = int(rs[0].info()["overlap_lanes"])
    bad = [f for f in frames if not np.array_equal(keep[f].cpu().numpy().reshape(Hc, Wc, 4), ref[f])]
    for r in rs:
        r.cleanup()
    return bad, dt, lanes


def main():
    assert os.environ.get("RTAMD_RCCL_LIB"), "run through tests/test_gpu_fake_rccl.py"
    if len(sys.argv) > 1 and sys.argv[1] == "c4":
        torch.cuda.set_device(0)
        bad, dt = world_c4()
        print(json.dumps({"world": 8, "config": "C4", "lanes": 8, "communicators": 8, "stage_depth": 64, "tile": TILE,
                          "frames": [0, 37], "frames_differing": bad, "s": round(dt, 2)}), flush=True)
        assert not bad, bad
        print(json.dumps({"ok": True}), flush=True)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "c5":
        torch.cuda.set_device(0)
        bad, dt, lanes = world_c5()
        print(json.dumps({"world": 8, "config": "C5", "build": "lbvh", "rebuild": True, "lanes": lanes, "communicators": 8,
                          "tile": TILE, "frames": [0, 5], "frames_differing": bad, "s": round(dt, 2)}), flush=True)
        assert not bad, bad
        print(json.dumps({"ok": True}), flush=True)
        return
    torch.cuda.set_device(0)
    scene = scenes.demo_with_particles(12)
    ref_r = make(scene)
    ref = [ref_r.render(f)[0] for f in range(F)]
    ref_r.cleanup()
    assert not np.array_equal(ref[0], ref[F - 1])
    cases = [(2, 1, 1, True), (8, 1, 1, True), (2, 3, 3, False), (8, 4, 2, False), (8, 8, 3, False)]
    for n, lanes, ncomm, sync in cases:
        t0 = time.time()
        got = world(scene, n, lanes, ncomm, sync)
        bad = [f for f in range(F) if not np.array_equal(got[f], ref[f])]
        print(json.dumps({"world": n, "lanes": lanes, "communicators": ncomm, "sync": sync, "frames": F,
                          "frames_differing": bad, "s": round(time.time() - t0, 2)}), flush=True)
        assert not bad, (n, lanes, ncomm, sync, bad)

    # a peer that never posts its send: rank 0's frame must fail with RT_ERR_DEVICE at the deadline, not hang
    rs = [make(scene) for _ in range(2)]
    cid = Renderer.comm_unique_id()
    for k, r in enumerate(rs):
        r.attach_comm(cid, k, 2, TILE, TILE)
    rs[0].set_comm_timeout(1500)
    t0 = time.time()
    try:
        rs[0].render(0)
        raise AssertionError("rank 0's frame completed without its peer")
    except abi.RtError as e:
        msg = str(e)
    dt = time.time() - t0
    print(json.dumps({"case": "peer never sends", "error": msg, "s": round(dt, 2)}), flush=True)
    assert msg.startswith("RT_ERR_DEVICE") and "not complete after 1500 ms" in msg, msg
    assert 1.4 < dt < 15.0, dt
    # the scene was detached by the abort: it renders whole single-GPU frames again
    rs[0].comm = None
    assert np.array_equal(rs[0].render(5)[0], ref[5])
    for r in rs:
        r.cleanup()
    print(json.dumps({"ok": True}), flush=True)


if __name__ == "__main__":
    main()
