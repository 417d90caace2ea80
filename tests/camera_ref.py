"""Test-side restatement (checker only) of the reference's camera control, in float32 scalar steps:
SDL_OpenGLWindow::calculateNewPosition (src/Global/SDL_OpenGLWindow.cu:182-256), Vec3::rotate
(include/Basic/Vec3.cuh:140-159), calculateCameraProperties' U / V / W (src/Global/RenderPin.cu:84-86),
getOperateArgs (include/Global/SDL_OpenGLWindow.cuh:63-74) and the loop's speed step (Renderer.cu:252-258).
Trigonometry goes through libm's cosf / sinf / asinf (what std::cos(float) calls), so values match the C
library bit for bit; every other operation is one float32 rounding in the reference's order."""
import ctypes
import math

import numpy as np

_m = ctypes.CDLL("libm.so.6")
for _n in ("cosf", "sinf", "asinf"):
    getattr(_m, _n).restype = ctypes.c_float
    getattr(_m, _n).argtypes = [ctypes.c_float]

f = np.float32


def cosf(x): return f(_m.cosf(float(x)))
def sinf(x): return f(_m.sinf(float(x)))
def asinf(x): return f(_m.asinf(float(x)))


def add(a, b): return [f(a[i] + b[i]) for i in range(3)]
def sub(a, b): return [f(a[i] - b[i]) for i in range(3)]
def scl(a, s): return [f(a[i] * f(s)) for i in range(3)]


def dot(a, b):
    s = f(0.0)
    for i in range(3):
        s = f(s + f(a[i] * b[i]))
    return s


def cross(a, b):
    return [f(f(a[1] * b[2]) - f(a[2] * b[1])), f(f(a[2] * b[0]) - f(a[0] * b[2])), f(f(a[0] * b[1]) - f(a[1] * b[0]))]


def length(a): return f(np.sqrt(dot(a, a)))


def unit(a):
    k = f(f(1.0) / length(a))
    return [f(a[i] * k) for i in range(3)]


def rotate(v, axis, angle):                          # Vec3.cuh:140-159
    k = unit(axis)
    c, s = cosf(angle), sinf(angle)
    p1 = scl(v, c)
    p2 = scl(cross(k, v), s)
    p3 = scl(scl(k, dot(k, v)), f(f(1.0) - c))
    return add(add(p1, p2), p3)


def operate_args(fps_limit=120.0, mouse_sensitivity=0.001, pitch_limit_degree=80.0, n_steps=2, step=0.05):
    PI = f(math.pi)
    return dict(mouse_sensitivity=f(mouse_sensitivity),
                pitch_limit=f(PI / f(f(f(pitch_limit_degree) * PI) / f(180.0))),
                move_speed=f(f(n_steps) * f(step)), move_speed_change_step=f(step),
                target_frame_us=int(f(1000000.0) / f(fps_limit)) if math.isfinite(fps_limit) else 0,
                relative_mouse=True)


def camera_move(center, target, up, ops, inp):
    """One loop step; returns (center, target, moved) and updates ops (speed, relative mode)."""
    center = [f(x) for x in center]; target = [f(x) for x in target]; up = [f(x) for x in up]
    mdx, mdy = (inp.get("dx", 0), inp.get("dy", 0)) if ops["relative_mouse"] else (0, 0)
    if inp.get("mouse_click"):
        ops["relative_mouse"] = not ops["relative_mouse"]
    cW = unit(sub(target, center))
    cU = unit(cross(cW, up))
    cV = unit(cross(cU, cW))
    rc, rt, moved = center, target, False
    if mdx != 0 or mdy != 0:
        moved = True
        view = sub(target, center)
        W, U, V = unit(cW), unit(cU), unit(cV)
        W = rotate(W, V, f(f(-float(mdx)) * ops["mouse_sensitivity"]))
        W = rotate(W, U, f(f(-float(mdy)) * ops["mouse_sensitivity"]))
        pitch = asinf(W[1])
        lim, corr = ops["pitch_limit"], False
        if pitch > lim:
            pitch, corr = lim, True
        elif pitch < -lim:
            pitch, corr = f(-lim), True
        if corr:
            h = unit([W[0], f(0.0), W[2]])
            W = add(scl(h, cosf(pitch)), [f(0.0), sinf(pitch), f(0.0)])
        rt = add(center, scl(W, length(view)))
    d = [f(0.0)] * 3
    fwd = unit([cW[0], f(0.0), cW[2]])
    if inp.get("key_w"): d = add(d, fwd)
    if inp.get("key_s"): d = sub(d, fwd)
    if inp.get("key_d"): d = add(d, cU)
    if inp.get("key_a"): d = sub(d, cU)
    if inp.get("key_space"): d = add(d, up)
    if inp.get("key_lshift"): d = sub(d, up)
    if dot(d, d) > f(0.0):
        moved = True
        t = scl(unit(d), ops["move_speed"])
        rc, rt = add(rc, t), add(rt, t)
    ds = inp.get("d_speed", 0)
    if ds > 0:
        ops["move_speed"] = f(ops["move_speed"] + ops["move_speed_change_step"])
    elif ds < 0:
        ops["move_speed"] = f(0.0) if ops["move_speed"] < ops["move_speed_change_step"] else \
            f(ops["move_speed"] - ops["move_speed_change_step"])
    return (rc, rt, moved) if moved else (center, target, False)
