"""SURVEY §8f row 4 — the interactive loop's host half without a window: camera control from scripted
key / mouse input (rt_camera_move vs tests/camera_ref.py, a float32 restatement of
SDL_OpenGLWindow::calculateNewPosition, SDL_OpenGLWindow.cu:182-256) and the frame limiter
(rt_frame_pace, Renderer.cu:327-337).  CPU only: no scene, no device."""
import ctypes as C

import numpy as np
import pytest

from rtamd import abi, interactive, scenes
from camera_ref import camera_move, operate_args

KEYS = ("key_w", "key_a", "key_s", "key_d", "key_space", "key_lshift")


def _script(seed, n):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        d = {k: int(rng.random() < 0.3) for k in KEYS}
        if rng.random() < 0.6:
            d["dx"], d["dy"] = int(rng.integers(-400, 400)), int(rng.integers(-300, 300))
        d["d_speed"] = int(rng.choice([0, 0, 0, 1, -1]))
        d["mouse_click"] = int(rng.random() < 0.05)
        out.append(d)
    return out


def test_control_init_matches_get_operate_args(rtlib_path):
    lib = abi.load_library(rtlib_path)
    c = abi.CameraControl()
    assert lib.rt_camera_control_init(C.byref(c), 120.0, 0.001, 80.0, 2, 0.05) == 0
    ref = operate_args()
    assert np.float32(c.pitch_limit) == ref["pitch_limit"]          # PI / degreeToRadian(80) = 2.25
    assert abs(c.pitch_limit - 2.25) < 1e-6
    assert np.float32(c.move_speed) == ref["move_speed"]
    assert c.target_frame_us == 8333 and c.sleep_margin_us == 2000 and c.restrict_frame_count == 1
    assert c.relative_mouse == 1
    assert lib.rt_camera_control_init(C.byref(c), float("inf"), 0.001, 80.0, 2, 0.05) == 0
    assert c.target_frame_us == 0 and c.restrict_frame_count == 0
    assert lib.rt_camera_control_init(C.byref(c), 0.0, 0.001, 80.0, 2, 0.05) == 1
    assert lib.rt_camera_move(None, C.byref(c), None, None) == 1


@pytest.mark.parametrize("seed,pitch_deg", [(0, 80.0), (1, 80.0), (2, 400.0), (3, 600.0)])
def test_scripted_moves_match_restatement(rtlib_path, seed, pitch_deg):
    """400 scripted frames: center / target after every frame equal the restatement bit for bit; a pitch
    limit above 180 degrees (PI / radians < PI / 2) makes the clamp branch fire."""
    abi.load_library(rtlib_path)
    cam = scenes.demo_scene().camera_input()
    ctl = interactive.CameraController(cam, pitch_limit_degree=pitch_deg, mouse_sensitivity=0.004)
    ops = operate_args(pitch_limit_degree=pitch_deg, mouse_sensitivity=0.004)
    c, t, up = list(cam.center.tuple()), list(cam.target.tuple()), list(cam.up.tuple())
    moved_frames = 0
    for d in _script(seed, 400):
        moved = ctl.step(interactive.input_state(**d))
        c, t, m = camera_move(c, t, up, ops, d)
        assert moved == m
        moved_frames += m
        got_c = np.array(ctl.camera.center.tuple(), np.float32)
        got_t = np.array(ctl.camera.target.tuple(), np.float32)
        assert np.array_equal(got_c, np.array(c, np.float32)), (got_c, c)
        assert np.array_equal(got_t, np.array(t, np.float32)), (got_t, t)
        assert np.float32(ctl.ctl.move_speed) == ops["move_speed"]
        assert bool(ctl.ctl.relative_mouse) == ops["relative_mouse"]
    assert moved_frames > 100


def test_clamp_keeps_pitch_and_distance(rtlib_path):
    """Looking far up with a 60-degree limit (stored as PI / radians(600) = 0.3 rad): the view direction's
    pitch is clamped to that value and the target stays at the view distance."""
    abi.load_library(rtlib_path)
    cam = scenes.demo_scene().camera_input()
    ctl = interactive.CameraController(cam, pitch_limit_degree=600.0)
    assert ctl.step(interactive.input_state(dy=-1500))
    c = np.array(ctl.camera.center.tuple()); t = np.array(ctl.camera.target.tuple())
    w = (t - c) / np.linalg.norm(t - c)
    assert abs(np.arcsin(w[1]) - ctl.ctl.pitch_limit) < 1e-5
    assert abs(np.linalg.norm(t - c) - 10.0) < 1e-5                 # demo camera: |target - center| = 10


def test_relative_mouse_toggle(rtlib_path):
    """A click toggles relative mode after the frame's events: motion in the clicked frame still turns the
    camera, motion in the next frame does not, a second click restores it."""
    abi.load_library(rtlib_path)
    cam = scenes.demo_scene().camera_input()
    ctl = interactive.CameraController(cam)
    assert ctl.step(interactive.input_state(dx=10, mouse_click=1))
    assert not ctl.step(interactive.input_state(dx=10))
    assert not ctl.step(interactive.input_state(dx=10, mouse_click=1))
    assert ctl.step(interactive.input_state(dx=10))


def test_speed_steps(rtlib_path):
    abi.load_library(rtlib_path)
    ctl = interactive.CameraController(scenes.demo_scene().camera_input())
    assert abs(ctl.ctl.move_speed - 0.1) < 1e-7
    for _ in range(5):
        ctl.step(interactive.input_state(d_speed=-1))
    assert ctl.ctl.move_speed == 0.0                                # never below zero (Renderer.cu:255-257)
    ctl.step(interactive.input_state(d_speed=3))                    # one step per frame, whatever the count
    assert abs(ctl.ctl.move_speed - 0.05) < 1e-7
    ctl.step(interactive.input_state(key_w=1, d_speed=1))           # the move uses the speed before the step
    assert abs(ctl.camera.center.z - (10.0 - 0.05)) < 1e-6


def test_frame_pacing(rtlib_path):
    """rt_frame_pace holds a frame to the 120-fps budget (8333 us) and returns at once for a late frame."""
    lib = abi.load_library(rtlib_path)
    ctl = interactive.CameraController(scenes.demo_scene().camera_input(), fps_limit=120.0)
    for _ in range(3):
        t0 = ctl.clock_ns()
        ctl.pace(t0)
        dt = ctl.clock_ns() - t0
        assert 8_333_000 <= dt < 8_333_000 + 3_000_000, dt
    t0 = ctl.clock_ns() - 20_000_000                                # a frame that already took 20 ms
    assert ctl.pace(t0) == 0
    free = interactive.CameraController(scenes.demo_scene().camera_input(), fps_limit=float("inf"))
    t0 = free.clock_ns()
    assert free.pace(t0) == 0
    assert lib.rt_frame_pace(None, 0) == 0
