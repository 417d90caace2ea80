"""SURVEY §8f row 4 on the GPU: a scripted fly-through (rtamd.interactive.run_scripted: input -> rt_camera_move
-> rt_camera_set when moved -> rt_render into device buffers -> limiter, the order of Renderer.cu:232-338)
produces, frame for frame, the image a fresh rt_camera_set + rt_render of the same camera gives."""
import numpy as np
import pytest

from rtamd import Renderer, interactive, scenes

pytestmark = pytest.mark.gpu

SCRIPT = [dict(), dict(key_w=1), dict(key_w=1, dx=40), dict(key_d=1, dy=-25), dict(dx=-120, dy=30, key_space=1),
          dict(key_s=1, key_a=1), dict(d_speed=1, key_w=1), dict(dx=300), dict(key_lshift=1, dy=60), dict(key_w=1, key_d=1)]


@pytest.mark.parametrize("lanes", [1, 3])
def test_scripted_fly_through_equals_per_frame_camera(gpu_lib, lanes):
    import torch
    s = scenes.demo_with_particles(10)
    W, H = 320, 192
    r = Renderer(s).build_acceleration_structure(0, mode="sah").configure_camera(W, H, ray_trace_depth=2)
    if lanes > 1:
        r.set_option("overlap", lanes)
    streams = [torch.cuda.Stream() for _ in range(lanes)]
    bufs = [torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda") for _ in range(len(SCRIPT))]
    torch.cuda.synchronize()                      # torch's fills run on its stream, not the lanes'
    script = [interactive.input_state(**d) for d in SCRIPT]
    cams, _ = interactive.run_scripted(r, script, [b.data_ptr() for b in bufs], streams=[x.cuda_stream for x in streams],
                                       pace=False, mouse_sensitivity=0.002)
    assert len(cams) == len(SCRIPT)
    r.synchronize()
    torch.cuda.synchronize()
    moved = sum(int(np.any(np.frombuffer(bytes(a.center), np.float32) != np.frombuffer(bytes(b.center), np.float32)) or
                    np.any(np.frombuffer(bytes(a.target), np.float32) != np.frombuffer(bytes(b.target), np.float32)))
                for a, b in zip(cams, cams[1:]))
    assert moved >= 8
    fresh = Renderer(s).build_acceleration_structure(0, mode="sah").configure_camera(W, H, ray_trace_depth=2)
    for k, cam in enumerate(cams):
        fresh.set_camera(cam)
        want = fresh.render(k)[0]
        got = bufs[k].cpu().numpy().reshape(H, W, 4)
        assert np.array_equal(got, want), k
    r.cleanup()
    fresh.cleanup()


def test_paced_loop_holds_120_fps(gpu_lib):
    """The full scripted loop with the limiter on: 12 frames take at least 11 frame budgets (8.33 ms)."""
    import time
    import torch
    s = scenes.demo_with_particles(4)
    r = Renderer(s).build_acceleration_structure(0, mode="sah").configure_camera(256, 144, ray_trace_depth=2)
    buf = torch.zeros(256 * 144 * 4, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    script = [interactive.input_state(key_w=1, dx=5)] * 12 + [interactive.input_state(key_quit=1)]
    t0 = time.perf_counter()
    cams, waits = interactive.run_scripted(r, script, [buf.data_ptr()], pace=True)
    r.synchronize()
    dt = time.perf_counter() - t0
    assert len(cams) == 12 and dt >= 11 * 0.00833
    assert sum(w > 0 for w in waits) >= 10                # a small frame is far inside the budget
    r.cleanup()
