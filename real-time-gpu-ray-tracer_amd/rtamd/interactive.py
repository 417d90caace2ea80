"""The reference's interactive frame loop without a window.

`Renderer::startRender` (src/Global/Renderer.cu:232-338) polls SDL input, moves the camera
(SDL_OpenGLWindow::calculateNewPosition, SDL_OpenGLWindow.cu:182-256), recomputes it (RenderPin.cu:73-95),
updates the instances, renders, presents and caps the frame rate at 120 fps (:327-337).  Here the input is
a script (one `InputState` per frame), the frame goes to a device buffer instead of the GL surface, and the
camera math and the limiter are the library's (rt_camera_move, rt_frame_pace in include/rt.h).
"""
from __future__ import annotations

import ctypes as C
import math

from . import abi

# getOperateArgs(120, 0.001f, 80, 2, 0.05f) — Renderer.cu:224-225
LOOP_DEFAULTS = dict(fps_limit=120.0, mouse_sensitivity=0.001, pitch_limit_degree=80.0, move_speed_n_steps=2,
                     move_speed_change_step=0.05)


def input_state(**keys) -> abi.InputState:
    """One frame of input: key_w/key_a/key_s/key_d/key_space/key_lshift (held), dx/dy (mouse counts),
    d_speed (wheel), mouse_click, key_quit."""
    st = abi.InputState()
    for k, v in keys.items():
        setattr(st, k, int(v))
    return st


class CameraController:
    """OperateArgs + the loop's camera step, over the C ABI."""

    def __init__(self, camera: abi.CameraInput, fps_limit: float = 120.0, mouse_sensitivity: float = 0.001,
                 pitch_limit_degree: float = 80.0, move_speed_n_steps: int = 2, move_speed_change_step: float = 0.05):
        self.lib = abi.load_library()
        self.camera = abi.CameraInput.from_buffer_copy(camera)
        self.ctl = abi.CameraControl()
        abi.check(self.lib, self.lib.rt_camera_control_init(C.byref(self.ctl), float(fps_limit), float(mouse_sensitivity),
                                                            float(pitch_limit_degree), int(move_speed_n_steps),
                                                            float(move_speed_change_step)))

    def step(self, inp: abi.InputState) -> bool:
        """Calculate the new position for this frame's input; True when the camera moved."""
        moved = C.c_uint32()
        abi.check(self.lib, self.lib.rt_camera_move(C.byref(self.camera), C.byref(self.ctl), C.byref(inp), C.byref(moved)))
        return bool(moved.value)

    def pace(self, frame_start_ns: int) -> int:
        return int(self.lib.rt_frame_pace(C.byref(self.ctl), int(frame_start_ns)))

    def clock_ns(self) -> int:
        return int(self.lib.rt_clock_ns())


def run_scripted(renderer, script, frame_buffers, streams=None, pace: bool = True, first_frame: int = 0, **operate):
    """Drive `renderer` through the scripted input the way startRender drives the reference's window:
    per frame, input -> camera move (+ rt_camera_set when it moved) -> rt_render into frame_buffers[k % n]
    (device pointers) on streams[k % len(streams)] (raw hipStream_t values; None: the scene's stream) ->
    limiter.  Stops at a key_quit frame.  Returns the camera inputs each frame used and the nanoseconds the
    limiter waited per frame."""
    args = dict(LOOP_DEFAULTS)
    args.update(operate)
    ctl = CameraController(renderer.camera, **args)
    cams, waits = [], []
    for k, inp in enumerate(script):
        t0 = ctl.clock_ns()
        if inp.key_quit:
            break
        if ctl.step(inp):
            renderer.set_camera(ctl.camera)
        cams.append(abi.CameraInput.from_buffer_copy(ctl.camera))
        buf = frame_buffers[k % len(frame_buffers)]
        st = streams[k % len(streams)] if streams else None
        renderer.render(first_frame + k, want_rgba=False, rgba8_device=buf, stream=st, sync=False)
        waits.append(ctl.pace(t0) if pace and math.isfinite(ctl.ctl.fps_limit) else 0)
    return cams, waits
