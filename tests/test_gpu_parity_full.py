"""Full 1920x1080 frames of the benched configuration against the oracle, at SURVEY §8(c)'s bars (verdict r3 item 1).

Bars (measured basis: the oracle against itself on different random trees):
  * identical trees (the reference's median-split trees, RT_BUILD_COMPAT_MEDIAN): 0 pixels beyond ULP — here the
    float RGB frame is bit-identical but for <= 1 pixel per frame where a hit lies on a box boundary the reference's
    own slab rounding culls (the FAST culls are conservative), RGBA8 within 1 LSB (gamma);
  * different trees (the bench's SAH trees and instance groups): RGBA8 outliers (any channel |d| > 1) <= 0.01 % of
    pixels at depth <= 2 and <= 0.05 % at depth >= 4; at depth 1 every channel's float |d| <= 1e-3 on >= 99.99 %
    of pixels.
The benched configuration is bench.py's: FAST persistent kernel, SAH trees, instance groups, quad traversal, LDS
scene region, 4 overlapped lanes on new streams, frames pipelined without waiting (RT_RENDER_NO_SYNC) into device
buffers; frames 0 and 37 of the animation (C5: GPU LBVH trees rebuilt every frame, 2 lanes).  Measured on MI355X
(scripts/parity_report.py):
  C2 depth 1: 0 outliers, float |d| 0 on both frames;  C2 depth 2: 34 / 4 outliers (0.0016 %);
  C3 (4 spp, depth 4): 122 / 3 outliers (0.0059 %); C4: 33 / 0;  C5: 4 / 255 (0.0031 %) — since round 5 the quads of
  GPU-built (and the reference's own) trees hold two binary levels visited in the reference's pair order (round 4's
  entry-t order: 1 304 / 1 544, over the bar); FAST on the reference's trees: bit-identical float frames.
Option "fast_math" (hardware reciprocals + FMA contraction, ~8 % faster) is held to its own measured bar: it moves
0.008-0.09 % of pixels even on identical trees (ground-sphere cancellation in Sphere.cu:4-28 and bounce origins).
Reference: src/Global/Kernel.cu:105-147 (render), src/AS/BoundingBox.cu:34-72 (the slab the FAST kernel culls with).
"""
import numpy as np
import pytest

from rtamd import Renderer, scenes

pytestmark = pytest.mark.gpu

THREADS = 16
FRAMES = (0, 37)


def outliers(a, b):
    d = np.abs(a.astype(np.int32) - b.astype(np.int32)).max(axis=-1)
    return int((d > 1).sum()), int(d.max())


def oracle_frames(scene, W, H, cam):
    from oracle.oracle import OracleScene
    o = OracleScene(scene, build_seed=0)
    o.camera(W, H, **cam)
    out = {}
    for f in FRAMES:
        o.update(f)
        orgb, orgba, _ = o.render(threads=THREADS)
        out[f] = (orgb, orgba)
    return out


CASES = {
    "C2d1": ("C2", dict(sample_count=1, ray_trace_depth=1)),
    "C2": ("C2", dict(sample_count=1, ray_trace_depth=2)),
    "C3": ("C3", dict(sample_count=4, ray_trace_depth=4)),
    "C4": ("C4", dict(sample_count=1, ray_trace_depth=2)),     # the C3 scene at 1 spp, depth 2 (one GPU's frame)
    "C5": ("C5", dict(sample_count=8, ray_trace_depth=2)),     # 10 M triangles, 4K, 8 -> 4 traced spp
}
# bench.py's configuration per case: the builder, the per-frame BLAS rebuild, the overlap lanes, lane 0 = the current
# stream (bench.py "classic": a rebuild on a small frame) or every lane a new stream
BENCH = {"C5": ("lbvh", True, 2, False)}

@pytest.fixture(scope="module", params=list(CASES))
def case(request):
    base, cam = CASES[request.param]
    cfg = scenes.CONFIGS[base]
    scene = scenes.config_scene(cfg)
    return request.param, scene, cfg.width, cfg.height, cam, oracle_frames(scene, cfg.width, cfg.height, cam)


def bench_frames(scene, W, H, cam, name="C2", **opts):
    """bench.py's configuration: SAH, 4 overlapped lanes on new streams, frames 0..37 pipelined into device buffers
    (C5: GPU LBVH with every BLAS rebuilt each frame, 2 lanes on new streams)."""
    import torch
    build, rebuild, L, classic = BENCH.get(name, ("sah", False, 4, False))
    r = Renderer(scene)
    if rebuild:                       # set before the build, as bench.py does (the build then leaves out cold records)
        r.set_option("rebuild", 1)
    r.build_acceleration_structure(0, mode=build).configure_camera(W, H, **cam)
    for k, v in opts.items():
        r.set_option(k, v)
    r.set_option("overlap", L)
    lanes = ([torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(L - 1)] if classic
             else [torch.cuda.Stream(priority=0) for _ in range(L)])
    keep = {f: (torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda"),
                torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")) for f in FRAMES}
    scratch = [torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda") for _ in range(L)]
    torch.cuda.synchronize()
    for k in range(max(FRAMES) + 1):
        rgba = keep[k][0] if k in keep else scratch[k % L]
        r.render(k, want_rgba=False, rgba8_device=rgba.data_ptr(), rgb32_device=keep[k][1].data_ptr() if k in keep else None,
                 stream=lanes[k % L].cuda_stream, sync=False)
    r.synchronize()
    torch.cuda.synchronize()
    out = {f: (keep[f][0].cpu().numpy().reshape(H, W, 4), keep[f][1].cpu().numpy().reshape(H, W, 3)) for f in FRAMES}
    r.cleanup()
    return out


def test_bench_configuration_full_frame_within_survey_bars(gpu_lib, case):
    name, scene, W, H, cam, orc = case
    got = bench_frames(scene, W, H, cam, name)
    depth = cam["ray_trace_depth"]
    bar = 0.0001 if depth <= 2 else 0.0005
    for f in FRAMES:
        rgba, rgb = got[f]
        orgb, orgba = orc[f]
        n_out, mx = outliers(rgba, orgba)
        print(f"{name} frame {f}: {n_out} outliers of {W * H} ({100 * n_out / (W * H):.4f} %), max {mx} LSB")
        assert n_out <= bar * W * H, (name, f, n_out, mx)
        if depth == 1:
            fd = np.abs(rgb - orgb).max(axis=-1)
            assert (fd <= 1e-3).mean() >= 0.9999, (name, f, float(fd.max()))


@pytest.mark.parametrize("wide", [0, 1])
def test_fast_kernel_on_reference_trees(gpu_lib, case, wide):
    """Identical trees (the reference's median split), FAST kernel (persistent waves, reciprocal-slab culls, LDS
    scene) with the reference's visit order on binary node pairs ("wide" 0) and on the default quads (two binary
    levels per quad, visited in the same pair order).  The kernel's arithmetic is the reference's wherever a value
    reaches a hit or a pixel; its box culls are conservative (RT_SLAB_CONS), and on these trees every box decision —
    and every pair-order comparison — that lies inside the reciprocal slab's error margin is re-taken with the
    reference's division slab (RT_BOX_EXACT, XBOX instances), so the traversal takes the reference's decisions: the
    float frame is bit-identical (round 4, without the re-test: 1 pixel on 5 of 20 renders, a hit on a box boundary
    the reference's own slab rounding culls; profiles/r04/c5_compat_residual/, profiles/r05/exact_box/)."""
    name, scene, W, H, cam, orc = case
    r = Renderer(scene).set_option("wide", wide).build_acceleration_structure(0, mode="compat").configure_camera(W, H, **cam)
    for f in FRAMES:
        rgba, rgb, _ = r.render(f, want_rgb=True)
        orgb, orgba = orc[f]
        mism = int((rgb != orgb).any(axis=-1).sum())
        print(f"{name} frame {f} wide {wide}: {mism} pixels differ, max {float(np.abs(rgb - orgb).max()):.4f}")
        assert mism == 0, (name, f, mism, float(np.abs(rgb - orgb).max()))
        assert outliers(rgba, orgba)[0] == 0
    r.cleanup()


def test_sah_outliers_split_into_tree_ties_and_fast_culls(gpu_lib, case):
    """Where the SAH frames' outliers against the oracle come from (verdict r5 weak 9).  On the SAH trees bench.py
    renders: (1) FAST in binary pair order ("wide" 0: every decision inside the slab's error margin re-taken with the
    reference's slab) equals the EXACT kernel's float frame bit for bit — so no FAST box decision or arithmetic moves a
    pixel on these trees, and every outlier below is the tree's; (2) EXACT on the SAH trees against the oracle on the
    reference's median-split trees: 283-430 outliers on frames 0 / 37 (0.014-0.021 %, measured) — the reference's q-centred
    parallelogram box (Parallelogram.cu:48-50, reproduced) lets a parallelogram's visibility depend on which tree and
    visit order reach it; (3) the benched default (greedy quads visited by entry t, conservative culls) against EXACT on
    the same trees: a different visit order on the same tree, 300-470 outliers — which happens to land closer to the
    oracle (34 / 122 / 33 outliers, test_bench_configuration_full_frame_within_survey_bars).  Both are held to 0.05 %
    here as a regression bar; the bit-identity (1) is the claim.  C5's GPU-built trees: test_fast_equals_exact_on_
    bench_lbvh_trees."""
    name, scene, W, H, cam, orc = case
    if name == "C5":
        pytest.skip("C5 is benched on GPU-built trees: test_fast_equals_exact_on_bench_lbvh_trees")
    r = Renderer(scene).build_acceleration_structure(0, mode="sah").configure_camera(W, H, **cam)
    for f in FRAMES:
        ergba, ergb, _ = r.render(f, exact=True, want_rgb=True)
        r.set_option("wide", 0)
        _, b0, _ = r.render(f, want_rgb=True)
        r.set_option("wide", 1)
        drgba, drgb, _ = r.render(f, want_rgb=True)
        tree = outliers(ergba, orc[f][1])
        cull = outliers(drgba, ergba)
        n0 = int((b0 != ergb).any(axis=-1).sum())
        nd = int((drgb != ergb).any(axis=-1).sum())
        print(f"{name} SAH frame {f}: FAST binary vs EXACT {n0} px; "
              f"EXACT-SAH vs oracle {tree[0]} outliers (max {tree[1]} LSB); benched FAST vs EXACT-SAH {nd} px differ, "
              f"{cull[0]} outliers (max {cull[1]} LSB)")
        assert n0 == 0, (name, f, n0)
        assert tree[0] <= 0.0005 * W * H and cull[0] <= 0.0005 * W * H, (name, f, tree, cull)
    r.cleanup()


def test_c5_reference_order_on_bench_trees(gpu_lib):
    """C5's benched trees (GPU LBVH, instance group) traversed by the FAST kernel in the reference's visit order
    (binary node pairs): within SURVEY's 0.01 % at depth 2 (measured 4 / 255 outliers of 8 294 400)."""
    cfg = scenes.CONFIGS["C5"]
    scene = scenes.config_scene(cfg)
    W, H, cam = cfg.width, cfg.height, CASES["C5"][1]
    orc = oracle_frames(scene, W, H, cam)
    r = Renderer(scene).set_option("wide", 0).build_acceleration_structure(0, mode="lbvh").configure_camera(W, H, **cam)
    for f in FRAMES:
        rgba, _, _ = r.render(f)
        n_out, mx = outliers(rgba, orc[f][1])
        print(f"C5 binary order frame {f}: {n_out} outliers, max {mx} LSB")
        assert n_out <= 0.0001 * W * H, (f, n_out, mx)
    r.cleanup()


# option "fast_math" on C5: measured 0.056 % / 0.049 % (the quad order's ties plus the arithmetic)
FAST_MATH_BAR = {"C5": 0.0007}


def test_fast_math_option_measured_bar(gpu_lib, case):
    """Option "fast_math" (not the default): its own measured bar, <= 0.02 % outliers at depth <= 2 and <= 0.1 % at
    depth >= 4 on the bench configuration (measured 0.011 % / 0.088 %; C5 0.07 %), and depth 1 within the float bar
    (measured 0)."""
    name, scene, W, H, cam, orc = case
    got = bench_frames(scene, W, H, cam, name, fast_math=1)
    depth = cam["ray_trace_depth"]
    bar = FAST_MATH_BAR.get(name, 0.0002 if depth <= 2 else 0.001)
    for f in FRAMES:
        n_out, mx = outliers(got[f][0], orc[f][1])
        assert n_out <= bar * W * H, (name, f, n_out, mx)
        if depth == 1:
            fd = np.abs(got[f][1] - orc[f][0]).max(axis=-1)
            assert (fd <= 1e-3).mean() >= 0.9999, (name, f, float(fd.max()))


@pytest.mark.parametrize("name", ["C2", "C3", "C5"])
def test_fast_equals_exact_on_bench_lbvh_trees(gpu_lib, name):
    """GPU-built trees (RT_BUILD_LBVH; C5's benched configuration: every BLAS rebuilt each frame, no cold records,
    instance group) in the FAST kernel's quad traversal — two binary levels per quad in the reference's pair order —
    with option "exact_decisions" (round 6): every FAST box decision and pair-order comparison on these trees that
    lies inside the reciprocal slab's error margin is re-taken with the reference's division slab, as on the
    reference's own trees, so the float frames equal the EXACT kernel's on the same trees bit for bit, frames 0 and 37.
    (The default keeps conservative culls: the re-takes cost C5 ~35 % per launch; round 5's C5 frame 37
    had one more outlier against the oracle than the same trees in binary order.)
    Reference: src/AS/BoundingBox.cu:44-66, include/Util/Range.cuh:33-43."""
    base, cam = CASES[name]
    cfg = scenes.CONFIGS[base]
    scene = scenes.config_scene(cfg)
    W, H = cfg.width, cfg.height
    r = Renderer(scene)
    if name == "C5":
        r.set_option("rebuild", 1)            # before the build, as bench.py sets it (no cold records)
    r.set_option("exact_decisions", 1)
    r.build_acceleration_structure(0, mode="lbvh").configure_camera(W, H, **cam)
    assert r.info()["device_bytes"] > 0
    for f in FRAMES:
        _, frgb, _ = r.render(f, want_rgb=True)
        _, ergb, _ = r.render(f, exact=True, want_rgb=True)
        mism = int((frgb != ergb).any(axis=-1).sum())
        print(f"{name} LBVH frame {f}: FAST vs EXACT {mism} pixels differ, max {float(np.abs(frgb - ergb).max()):.4g}")
        assert mism == 0, (name, f, mism)
    r.cleanup()
