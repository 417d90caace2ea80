"""The multi-GPU frame inside the library (rt_scene_attach_comm) on one GPU.

A world-1 communicator runs the whole multi-GPU code path of rt_render — the rank's tiles traced
into the gather buffer, the (empty) RCCL group, the assemble kernel into rank 0's frame — so the
frame must equal the single-launch frame byte for byte, with and without overlapped lanes.
(World > 1 needs one GPU per rank: RCCL rejects two ranks on one device; the driver's 8-GPU bench
runs it, and tests/test_multirank_cpu.py checks the gather protocol with the library's tile
bookkeeping on CPU.)
"""
import numpy as np
import pytest

from rtamd import Renderer, abi, scenes

pytestmark = pytest.mark.gpu


def test_world1_comm_frames_equal_single_launch(gpu_lib):
    import torch
    s = scenes.demo_with_particles(10)
    W, H = 400, 232
    r = Renderer(s).build_acceleration_structure(0, mode="sah").configure_camera(W, H, ray_trace_depth=2)
    ref = [r.render(f)[0] for f in range(6)]
    cid = Renderer.comm_unique_id()
    assert len(cid) == 128
    for tw, th in ((64, 64), (32, 16)):
        r.attach_comm(cid if (tw, th) == (64, 64) else Renderer.comm_unique_id(), 0, 1, tw, th)
        for f in range(3):
            rgba, _, st = r.render(f)
            assert np.array_equal(rgba, ref[f]), (tw, th, f)
            assert st["pixels"] == W * H
        # overlapped lanes on two caller streams, device outputs
        r.set_option("overlap", 2)
        lanes = [torch.cuda.Stream() for _ in range(2)]
        bufs = [torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda") for _ in range(6)]
        torch.cuda.synchronize()
        for f in range(6):
            r.render(f, want_rgba=False, rgba8_device=bufs[f].data_ptr(), stream=lanes[f % 2].cuda_stream,
                     sync=False, keep_counters=True)
        r.synchronize()
        torch.cuda.synchronize()
        for f in range(6):
            assert np.array_equal(bufs[f].cpu().numpy().reshape(H, W, 4), ref[f]), (tw, th, f)
        r.set_option("overlap", 0)
        r.detach_comm()
    assert np.array_equal(r.render(2)[0], ref[2])       # detached: whole-frame launches again


def test_world1_comm_eight_lanes_many_frames(gpu_lib):
    """The multi-GPU share settings (8 lanes, the lane-scaled auto grid, 32x32 tiles): 24 frames cycled over
    8 caller streams without waiting, more frames than frame blocks, so staging buffers and frame blocks are
    reused while other lanes' traces, gathers and assembles are still in flight; every frame must equal its
    single-launch frame (the per-launch completion events order each reuse after the launch that read it)."""
    import torch
    s = scenes.demo_with_particles(12)
    W, H = 352, 208
    r = Renderer(s).build_acceleration_structure(0, mode="sah").configure_camera(W, H, ray_trace_depth=2)
    F, L = 24, 8
    ref = [r.render(f)[0] for f in range(F)]
    r.attach_comm(Renderer.comm_unique_id(), 0, 1, 32, 32)
    r.set_option("overlap", L)
    lanes = [torch.cuda.Stream() for _ in range(L)]
    bufs = [torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda") for _ in range(F)]
    torch.cuda.synchronize()
    for f in range(F):
        r.render(f, want_rgba=False, rgba8_device=bufs[f].data_ptr(), stream=lanes[f % L].cuda_stream, sync=False)
    r.synchronize()
    torch.cuda.synchronize()
    for f in range(F):
        assert np.array_equal(bufs[f].cpu().numpy().reshape(H, W, 4), ref[f]), f
    r.set_option("overlap", 0)
    r.detach_comm()


def test_comm_rejects_tiles_and_rgb(gpu_lib):
    s = scenes.demo_scene()
    r = Renderer(s).build_acceleration_structure(0).configure_camera(64, 64)
    r.attach_comm(Renderer.comm_unique_id(), 0, 1)
    with pytest.raises(abi.RtError, match="tile"):
        r.render(0, tiles=(64, 64, 0, 2))
    with pytest.raises(abi.RtError, match="rgb32"):
        r.render(0, want_rgb=True)
    with pytest.raises(abi.RtError):
        r.attach_comm(Renderer.comm_unique_id(), 1, 1)      # rank outside [0, world)


def test_c4_through_the_comm_path(gpu_lib):
    """C4's scene and settings through the library's multi-GPU path (world 1): the assembled frame
    equals the single-launch frame."""
    cfg = scenes.CONFIGS["C4"]
    s = scenes.config_scene(scenes.CONFIGS["C3"])
    r = Renderer(s).build_acceleration_structure(0, mode="sah").configure_camera(
        cfg.width, cfg.height, sample_count=cfg.spp, ray_trace_depth=cfg.depth)
    full = r.render(0)[0]
    r.attach_comm(Renderer.comm_unique_id(), 0, 1, 64, 64)
    assert np.array_equal(r.render(0)[0], full)


def test_comm_timeout_frames_and_state(gpu_lib):
    """rt_comm_set_timeout: every wait on a multi-GPU frame polls (completion, ncclCommGetAsyncError, the
    deadline); frames that complete are unaffected, and the setting survives a re-attach."""
    s = scenes.demo_with_particles(4)
    W, H = 256, 144
    r = Renderer(s).build_acceleration_structure(0, mode="sah").configure_camera(W, H, ray_trace_depth=2)
    ref = [r.render(f)[0] for f in range(3)]
    r.set_comm_timeout(5000)
    r.attach_comm(Renderer.comm_unique_id(), 0, 1, 32, 32)
    for f in range(3):
        assert np.array_equal(r.render(f)[0], ref[f])
    r.set_comm_timeout(0)
    r.synchronize()
    r.detach_comm().attach_comm(Renderer.comm_unique_id(), 0, 1, 64, 32)
    assert np.array_equal(r.render(2)[0], ref[2])
    r.cleanup()


def _two_gpu_rank(rank, world, id_path, out_path):
    import os
    import sys
    import time
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "real-time-gpu-ray-tracer_amd")]
    import torch
    from rtamd import Renderer as R, scenes as S
    torch.cuda.set_device(rank)
    s = S.demo_with_particles(10)
    W, H = 480, 272
    r = R(s, device=rank).build_acceleration_structure(0, mode="sah").configure_camera(W, H, ray_trace_depth=2)
    ref = [r.render(f)[0] for f in range(6)] if rank == 0 else None
    if rank == 0:
        with open(id_path + ".tmp", "wb") as f:
            f.write(R.comm_unique_id())
        os.replace(id_path + ".tmp", id_path)
    while not os.path.exists(id_path):
        time.sleep(0.01)
    cid = open(id_path, "rb").read()
    r.set_comm_timeout(60000)
    r.attach_comm(cid, rank, world, 32, 32)
    ok = True
    for f in range(3):                                     # synchronous frames
        rgba = r.render(f)[0]
        if rank == 0:
            ok &= bool(np.array_equal(rgba, ref[f]))
    r.set_option("overlap", 3)                            # lanes beyond the attach-time communicators
    lanes = [torch.cuda.Stream() for _ in range(3)]
    bufs = [torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda") for _ in range(6)]
    torch.cuda.synchronize()
    for f in range(6):
        r.render(f, want_rgba=False, rgba8_device=bufs[f].data_ptr(), stream=lanes[f % 3].cuda_stream, sync=False)
    r.synchronize()
    torch.cuda.synchronize()
    if rank == 0:
        for f in range(6):
            ok &= bool(np.array_equal(bufs[f].cpu().numpy().reshape(H, W, 4), ref[f]))
        np.save(out_path, np.array([ok]))
    r.cleanup()


def test_two_gpus_gather_equals_single_launch(gpu_lib, tmp_path):
    """World 2 on two GPUs (skipped on a one-GPU box): the RCCL Send / Recv branch of rt_render, synchronous
    and on three overlapped lanes; rank 0's assembled frames equal its own single-launch frames."""
    import torch
    import torch.multiprocessing as mp
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL rejects two ranks on one device)")
    out = str(tmp_path / "ok.npy")
    mp.spawn(_two_gpu_rank, args=(2, str(tmp_path / "id.bin"), out), nprocs=2, join=True)
    assert bool(np.load(out)[0])
