"""The library's world > 1 multi-GPU frame on one GPU (verdict r3 item 2).

RCCL refuses two ranks on one device, so tests/fake_rccl/fake_rccl.hip stands in for librccl.so.1
(RTAMD_RCCL_LIB, csrc/comm.cpp): an N-rank world inside one process, point-to-point messages matched in
posting order and ordered on the streams as RCCL orders them.  tests/fake_rccl_run.py drives worlds of 2 and
8 scenes through rt_render's RCCL branch — synchronous frames, and pipelined frames on 3-8 overlap lanes with
fewer communicators than lanes (lane q uses communicator q % ncomm) — and checks rank 0's assembled frames
byte-identical to single-launch frames for 24 animated frames; then a peer that never sends: rank 0's frame
returns RT_ERR_DEVICE at rt_comm_set_timeout's deadline instead of hanging, and the detached scene renders
again.  (What is replaced: the reference is single-GPU and exits on any error, src/Global/Global.cu:34-41.)
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
FAKE = os.path.join(REPO, "real-time-gpu-ray-tracer_amd", "lib", "libfake_rccl.so")


def test_world_2_and_8_through_fake_rccl(gpu_lib):
    if not os.path.exists(FAKE):
        subprocess.run(["make", "-s", "-C", os.path.join(HERE, "fake_rccl")], check=True)
    env = dict(os.environ, RTAMD_RCCL_LIB=FAKE, FAKE_RCCL_MAX_WAIT_S="20")
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "fake_rccl_run.py")], env=env, capture_output=True,
                       text=True, timeout=280)
    print(p.stdout[-4000:])
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    worlds = [x for x in lines if "world" in x]
    assert {x["world"] for x in worlds} == {2, 8} and all(not x["frames_differing"] for x in worlds)
    assert any(x.get("case") == "peer never sends" for x in lines) and lines[-1] == {"ok": True}


def test_world_8_at_c4_size_bench_settings(gpu_lib):
    """bench.py's N > 1 settings at C4's real size through the world > 1 branch (verdict r4 item 4): the C3 scene at
    1920x1080, 1 spp, depth 2, 8 ranks, 32x32 tiles, 8 lanes on new streams with one communicator each, stage_depth
    64, frames 0..37 pipelined without waiting; rank 0's frames 0 and 37 equal single-launch frames byte for byte
    (test_gpu_parity_full.py holds those to the oracle)."""
    if not os.path.exists(FAKE):
        subprocess.run(["make", "-s", "-C", os.path.join(HERE, "fake_rccl")], check=True)
    env = dict(os.environ, RTAMD_RCCL_LIB=FAKE, FAKE_RCCL_MAX_WAIT_S="60")
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "fake_rccl_run.py"), "c4"], env=env, capture_output=True,
                       text=True, timeout=280)
    print(p.stdout[-2000:])
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert lines[0]["config"] == "C4" and lines[0]["frames_differing"] == [] and lines[-1] == {"ok": True}


def test_world_8_c5_with_per_frame_rebuild(gpu_lib):
    """C5's 8-GPU configuration through the world > 1 branch (verdict r5 item 1): 8 ranks of the 10 M-triangle scene at
    3840x2160, 8 -> 4 traced spp, depth 2, every BLAS and the TLAS rebuilt on the GPU each frame, the scene's own
    lanes (overlap -1, 8 communicators), 32x32 tiles, frames 0..5 pipelined without waiting and without caller
    streams: rank 0's frames 0 and 5 equal single-launch frames of the same LBVH scene byte for byte (the rebuild on
    the scene stream, the traces on the lane streams and the gathers on the communicators, all in flight together).
    Replaced behaviour: the reference builds its BLASes once and renders on one GPU
    (src/AS/BLAS.cu:4-117, src/Global/Renderer.cu:305-317)."""
    if not os.path.exists(FAKE):
        subprocess.run(["make", "-s", "-C", os.path.join(HERE, "fake_rccl")], check=True)
    env = dict(os.environ, RTAMD_RCCL_LIB=FAKE, FAKE_RCCL_MAX_WAIT_S="120")
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "fake_rccl_run.py"), "c5"], env=env, capture_output=True,
                       text=True, timeout=400)
    print(p.stdout[-2000:])
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert lines[0]["config"] == "C5" and lines[0]["frames_differing"] == [] and lines[-1] == {"ok": True}
    assert lines[0]["lanes"] == 2
