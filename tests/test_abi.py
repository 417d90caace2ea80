"""The C-ABI boundary: struct layouts, exported symbols, error behaviour without a GPU, and the
host-side functions that need no device.  CPU-only (no compute calls)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from rtamd import abi, scenes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "rt.h")

STRUCTS = {
    "rt_vec3": abi.Vec3, "rt_sphere": abi.Sphere, "rt_parallelogram": abi.Parallelogram,
    "rt_triangle": abi.Triangle, "rt_rough": abi.Rough, "rt_metal": abi.Metal, "rt_xform": abi.Xform,
    "rt_instance_desc": abi.InstanceDesc, "rt_scene_desc": abi.SceneDesc, "rt_camera_input": abi.CameraInput,
    "rt_render_opts": abi.RenderOpts, "rt_stats": abi.Stats, "rt_hit": abi.Hit, "rt_scene_info": abi.SceneInfo,
    "rt_vtk_info": abi.VtkInfo, "rt_vtk_particle": abi.VtkParticle,
    "rt_camera_control": abi.CameraControl, "rt_input_state": abi.InputState,
}


def _c_layout(tmp_path):
    """sizeof / offsetof of every rt.h struct as compiled by the C compiler."""
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', 'int main(void){']
    for cname, py in STRUCTS.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    # the layout RT_ABI_VERSION 2 promises (rt.h): a caller whose rt_stats differs is built against another ABI
    lines.append('_Static_assert(sizeof(rt_stats) == 96, "rt_stats layout of ABI 2");')
    lines.append(f'_Static_assert(RT_ABI_VERSION == {abi.RT_ABI_VERSION}u, "rt.h and the ctypes mirror disagree");')
    lines.append('return 0;}')
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    return dict(line.rsplit(" ", 1) for line in out.strip().splitlines())


def test_ctypes_mirror_matches_c_layout(tmp_path):
    lay = _c_layout(tmp_path)
    for cname, py in STRUCTS.items():
        assert int(lay[cname]) == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(lay[f"{cname}.{fname}"]) == getattr(py, fname).offset, f"{cname}.{fname}"


def _declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(rt_[a-z_0-9]+)\s*\(", text))
    return sorted(n for n in names if n != "rt_update_fn")


def test_library_exports_every_declared_symbol(rtlib_path):
    declared = _declared_functions()
    assert set(declared) == set(abi.EXPORTED_SYMBOLS)
    lib = C.CDLL(rtlib_path)
    for name in declared:
        assert hasattr(lib, name), f"librtamd.so does not export {name}"
    nm = subprocess.run(["nm", "-D", "--defined-only", rtlib_path], capture_output=True, text=True, check=True).stdout
    for name in declared:
        assert re.search(rf"\bT {name}$", nm, re.M), name


def test_library_is_built_from_this_tree(rtlib_path):
    """The build stamp (rtamd/provenance.py) matches the library and the sources in the tree."""
    from rtamd import provenance
    ok, msg = provenance.check()
    assert ok, msg
    with open(provenance.STAMP) as f:
        import json
        d = json.load(f)
    assert "real-time-gpu-ray-tracer_amd/csrc/trace_kernel.hip" in d["sources"] and "include/rt.h" in d["sources"]


def test_library_loads_and_reports_abi(rtlib_path):
    lib = abi.load_library(rtlib_path)
    assert lib.rt_abi_version() == abi.RT_ABI_VERSION


def test_no_device_is_an_error_not_a_fallback(rtlib_path):
    lib = abi.load_library(rtlib_path)
    if lib.rt_device_count() > 0:
        pytest.skip("a GPU is visible; this checks the no-device path")
    s = scenes.demo_scene()
    desc = s.desc()
    h = C.c_void_p()
    st = lib.rt_scene_create(C.byref(desc), 0, C.byref(h))
    assert st == 2 and not h.value                       # RT_ERR_DEVICE
    assert b"device" in lib.rt_last_error()


def test_invalid_arguments_are_rejected(rtlib_path):
    lib = abi.load_library(rtlib_path)
    h = C.c_void_p()
    assert lib.rt_scene_create(None, 0, C.byref(h)) == 1
    empty = abi.SceneDesc()
    assert lib.rt_scene_create(C.byref(empty), 0, C.byref(h)) == 1
    assert lib.rt_scene_build(None, 0, 0) == 1
    assert lib.rt_render(None, 0, None, None, None, None) == 1
    assert lib.rt_tiles_for_rank(None, 64, 64, 0, 1) == 0


def test_native_demo_update_matches_oracle_copy(rtlib_path, oracle_lib):
    """rt_demo_update (product) and oracle_demo_update are independent restatements of
    Main.cu:6-42; they must agree bit for bit."""
    lib = abi.load_library(rtlib_path)
    ol = oracle_lib.lib()
    for frame in (0, 1, 37, 100, 12345):
        a = (abi.Xform * 7)()
        b = (abi.Xform * 7)()
        lib.rt_demo_update(None, a, 7, frame)
        ol.oracle_demo_update(None, b, 7, frame)
        assert bytes(a) == bytes(b)
        # and they agree with the Python restatement to float32 rounding
        c = (abi.Xform * 7)()
        scenes.demo_update_py(c, 7, frame)
        av = np.frombuffer(bytes(a), np.float32)[:45]
        cv = np.frombuffer(bytes(c), np.float32)[:45]
        assert np.allclose(av, cv, rtol=1e-5, atol=1e-5)
