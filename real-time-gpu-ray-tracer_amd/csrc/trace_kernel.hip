// trace_kernel.hip — the hot path on gfx950: camera ray -> two-level BVH traversal
// (TLAS -> instance -> BLAS) -> sphere / parallelogram / Moller-Trumbore intersection ->
// Rough/Metal scatter loop -> average -> gamma-2 quantise -> framebuffer write.
//
// Restates the reference kernel `render` (src/Global/Kernel.cu:105-147) and its device
// callees: rayColor (Kernel.cu:6-103), TLAS::hit (src/AS/TLAS.cu:131-201), Instance::hit
// (src/AS/Instance.cu:19-50), BLAS::hit (src/AS/BLAS.cu:119-206), BoundingBox::hit
// (src/AS/BoundingBox.cu:34-72), Sphere/Parallelogram/Triangle::hit (src/Geometry/*.cu),
// Rough/Metal::scatter (include/Material/*.cuh), Color3::castToUchar4 (Color3.cuh:99-114).
//
// This file is compiled three times:
//   RT_EXACT=1, -ffp-contract=off : every float operation in the reference's order with IEEE
//       division, the reference's binary trees and visit order — bit-faithful to the oracle on identical
//       trees, equal work counters (parity mode);
//   RT_EXACT=0 RT_FAST_IEEE=1, -ffp-contract=off (default): the persistent quad-tree kernel with
//       reciprocal-direction slab tests (one explicit FMA per plane, a cull only) and the reference's
//       arithmetic everywhere a value reaches a hit or a pixel — on the reference's trees its frames are
//       bit-identical to the oracle's;
//   RT_EXACT=0 RT_FAST_IEEE=0, -ffp-contract=fast (option "fast_math"): also reciprocal determinant /
//       division, v_rsq, FMA-contracted transforms (parity within the measured tolerance).
//
// Traversal keeps the reference's visit order exactly: node pairs test both children of an
// interior node (BLAS.cu:180-202), the near child (smaller entry t; ties -> left) is visited
// next and the far child is pushed with its entry t; a popped entry is culled iff its entry t
// >= the current tmax, which is exactly when the reference's re-test of the popped node box
// (BLAS.cu:145) fails.  TLAS leaves with two instances push a non-cullable "resume" entry, as
// the reference loops over a leaf's instances without re-testing the leaf box (TLAS.cu:157-173).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.hpp"
#include "../../include/rt.h"

#ifndef RT_EXACT
#error "compile with -DRT_EXACT=0 or 1"
#endif

// RT_FAST_IEEE (FAST builds): 1 = the reference's correctly rounded division and 1/sqrt everywhere except the box
// tests' reciprocal slabs, compiled without FMA contraction (the default FAST kernel: on the reference's own trees
// its frames are bit-identical to the oracle's); 0 = hardware v_rcp / v_rsq and FMA contraction
// (option "fast_math": ~8 % faster on C2 / C3, and ~0.01-0.09 % of pixels differ, measured)
#ifndef RT_FAST_IEEE
#define RT_FAST_IEEE 1
#endif
#if RT_EXACT
#define RT_SUFFIX(n) n##_exact
#elif RT_FAST_IEEE
#define RT_SUFFIX(n) n##_fast
#else
#define RT_SUFFIX(n) n##_fastmath
#endif

namespace rtamd {
namespace RT_SUFFIX(dev) {

constexpr float FZERO = 1e-6f;          // FLOAT_ZERO_VALUE (Global.cuh:147)
constexpr float TMIN = 0.001f;          // Kernel.cu:66
constexpr int BLOCK = 256;              // 4 waves; each wave owns one 8x8 pixel unit
#ifndef RT_LDS_DEPTH
#define RT_LDS_DEPTH 16
#endif
#ifndef RT_LDS_MATERIALS
#define RT_LDS_MATERIALS 64              // the scene region ("lds_scene") needs the rest of the 52 KB
#endif
constexpr int LDS_DEPTH = RT_LDS_DEPTH;         // per-lane stack entries kept in LDS
constexpr int LDS_MATERIALS = RT_LDS_MATERIALS; // persistent kernel: material table in LDS up to this many slots
constexpr int SPILL_DEPTH = 64 - LDS_DEPTH;   // overflow entries in scratch (max depth 64 = reference)
static_assert(LDS_DEPTH % 4 == 0, "half-pages move as 16 B pieces");
#ifndef RT_CHAIN_ROOT_LEAF
#define RT_CHAIN_ROOT_LEAF 1            // quad trees: an entered instance whose BLAS root is a leaf (a sphere, a
                                        // parallelogram, a small mesh) has it tested in the same leaf round
#endif
#ifndef RT_SLAB_CONS
#define RT_SLAB_CONS 1                  // FAST slabs are conservative: the interval [lo, hi] a box test computes with
                                        // reciprocal-FMA planes is widened by a bound on its distance from the
                                        // reference's (mn - q) / d interval before the lo < hi test (and a popped entry's
                                        // lo before its lo < tmax re-test), so a FAST cull never rejects a box the
                                        // reference's slab accepts — but for a parallel axis (|d| < 1e-6) whose origin lies
                                        // exactly on a face of the slab, which planes cannot widen (the reference keeps
                                        // q == min / max, BoundingBox.cu:47; the FAST planes there are the rounding residual
                                        // of o / d): the exact-decision instances (XD_ALL, XBOX) re-take every box test of a
                                        // ray with a parallel axis with the reference's slab; the others keep the exception.
                                        // Entries keep the unwidened lo, so children are still ordered by it
#endif
#ifndef RT_BOX_EXACT
#define RT_BOX_EXACT 1                  // FAST box decisions that lie inside the slabs' error margin (and every box test of a
                                        // ray with a parallel axis) are re-taken with the reference's division slab, as
                                        // are the pair-order comparisons of two entry t's inside the margin: on the
                                        // reference's trees the traversal takes the reference's decisions
#endif
// the persistent kernel's traversal modes (SceneGPU::wide): 0 binary node pairs, 1 greedy quads by entry t (host SAH
// trees), 2 two-level quads in pair order (GPU-built trees), 3 the same with exact decisions (the reference's trees, and
// GPU-built trees with option "exact_decisions").
// Exact-decision level of a traversal instance (template argument XB):
//   XD_CULL: conservative culls only (modes 1 and 2).  One documented exception to "a FAST cull never rejects a box the
//            reference keeps": a ray with a parallel axis (|d| < 1e-6) whose origin lies exactly on a face of that
//            axis's slab (the reference keeps q == min / max, BoundingBox.cu:47; reciprocal planes cannot represent it;
//            tests/test_gpu_box.py pins the misses to exactly that case).  Re-taking such rays' decisions in modes 1 / 2
//            (round 6) cost C2 4.4 % and C3 2.5 % per frame through register pressure alone;
//   XD_ALL : every decision inside the slabs' error margin, every box test of a ray with a parallel axis and (pair
//            order) every comparison of two entry t's inside the margin re-taken with the reference's slab: the traversal
//            takes the reference's decisions.  The binary pairs and mode 3 — FAST then equals EXACT on the same trees
//            (tests/test_gpu_parity_full.py: the reference's trees, and C5's benched LBVH trees with "exact_decisions").
//            For mode 2 by default it cost C5 +34 % per frame (sibling boxes' entry t's often tie exactly:
//            profiles/r06/exact_decisions/).
constexpr int XD_CULL = 0, XD_ALL = 2;
#define XBOX(W) ((RT_BOX_EXACT && ((W) == 0 || (W) == 3)) ? XD_ALL : XD_CULL)
#ifndef RT_NZ_MIN
#define RT_NZ_MIN FZERO                 // |d_axis| below this is clamped to +-1e-20 for the slab reciprocals (prep)
#endif
#ifndef TRI_AHEAD
#define TRI_AHEAD 4                     // triangle records of a leaf requested before the first test (all 4 of a
                                        // full leaf: C2 serialised -2..-7 %, C3 -0.6 %; profiles/r02_ab_tri_ahead.jsonl)
#endif

struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ f3 ld3(const float *p) { return mk(p[0], p[1], p[2]); }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 scl(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ f3 mul(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) {          // Vec3.cuh:113-119
    float s = 0.0f; s += a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s;
}
__device__ __forceinline__ f3 cross(f3 a, f3 b) {           // Vec3.cuh:120-126
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// "fast_math" (RT_FAST_IEEE 0) replaces IEEE division / 1/sqrt by the hardware v_rcp_f32 / v_rsq_f32 (1 ulp);
// EXACT and the default FAST build keep the reference's correctly rounded operations (the box tests' reciprocals
// are the FAST kernels' own: prep / slab4, a cull only).
#define RT_IEEE_PRIM (RT_EXACT || RT_FAST_IEEE)
#define RT_IEEE_TRI RT_IEEE_PRIM
__device__ __forceinline__ float rcp(float x) {              // slab reciprocals (FAST)
#if RT_EXACT
    return 1.0f / x;
#else
    return __builtin_amdgcn_rcpf(x);
#endif
}
__device__ __forceinline__ float fdiv(float a, float b) {
#if RT_IEEE_PRIM
    return a / b;
#else
    return a * __builtin_amdgcn_rcpf(b);
#endif
}
__device__ __forceinline__ f3 unit(f3 a) {                   // Vec3.cuh:129-137
#if RT_IEEE_PRIM
    const float f = 1.0f / sqrtf(dot(a, a));
#else
    const float f = __builtin_amdgcn_rsqf(dot(a, a));
#endif
    return mk(a.x * f, a.y * f, a.z * f);
}
__device__ __forceinline__ float comp(f3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
// unit(e1 x e2) with the arithmetic the BLAS builders store a triangle's normals with (lbvh.hip gather_item,
// host_math.hpp; Triangle.cuh:26-46): correctly rounded 1 / sqrt, no contraction, in every FAST variant
__device__ __forceinline__ f3 tri_face_normal(f3 a, f3 b) {
#pragma clang fp contract(off)
    const f3 c = mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
    float d = 0.0f;
    d += c.x * c.x; d += c.y * c.y; d += c.z * c.z;
    const float f = 1.0f / sqrtf(d);
    return mk(c.x * f, c.y * f, c.z * f);
}

__device__ __forceinline__ bool f_eq(float a, float b) { return fabsf(a - b) < FZERO; }
__device__ __forceinline__ bool in_range(float v, float mn, float mx) {      // Range.cuh:33-43
    return f_eq(v, mn) || f_eq(v, mx) || (v > mn && v < mx);
}

// ---- pinned RNG contract (replaces curand XORWOW, Kernel.cu:114) ----------
constexpr uint64_t GOLDEN64 = 0x9E3779B97F4A7C15ull;
constexpr uint64_t SUBMUL64 = 0xD1B54A32D192ED03ull;
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
struct Rng {
    uint64_t s;
    __device__ __forceinline__ void init(uint64_t seed, uint64_t sub) { s = mix64((seed * GOLDEN64) ^ ((sub + 1ull) * SUBMUL64)); }
    __device__ __forceinline__ float uniform() {                             // (0, 1]
        s += GOLDEN64;
        const uint64_t x = mix64(s);
        return (float)((uint32_t)(x >> 40) + 1u) * 0x1p-24f;
    }
    __device__ __forceinline__ float range(float mn, float mx) { return mn + (mx - mn) * uniform(); }   // Global.cuh:209-211
};
__device__ __forceinline__ f3 random_space_vector(Rng &r) {   // Vec3.cu:54-65 (length 1)
    f3 v; float l2;
    do {
        v.x = r.range(-1.0f, 1.0f);
        v.y = r.range(-1.0f, 1.0f);
        v.z = r.range(-1.0f, 1.0f);
        l2 = dot(v, v);
    } while (l2 < FZERO * FZERO);
    return scl(unit(v), 1.0f);
}
__device__ __forceinline__ f3 random_plane_vector(Rng &r, float maxlen) {   // Vec3.cu:29-36
    float x, y;
    do {
        x = r.range(-1.0f, 1.0f);
        y = r.range(-1.0f, 1.0f);
    } while (x * x + y * y > maxlen * maxlen);
    return mk(x, y, 0.0f);
}

// ---- rays ---------------------------------------------------------------------------
struct RayP {
    f3 o, d;
#if !RT_EXACT
    f3 inv, oinv;      // 1/d and o/d for one-FMA slab planes
#if RT_SLAB_CONS
    float pad;         // the absolute part of a plane distance's error bound: 2^-22 max |o/d| over the non-parallel
                       // axes; negative (sign bit set) when an axis is parallel (|d| < 1e-6)
#endif
#endif
};
template <int XB = XD_CULL>
__device__ __forceinline__ void prep(RayP &r) {
#if !RT_EXACT
    // |d| < 1e-6 (the reference's parallel-axis threshold, BoundingBox.cu:44-50) -> +-1e-20: the plane distances
    // of that axis are +-1e20 * (face - o), so the axis rejects the box exactly when o lies outside the slab and
    // constrains nothing otherwise — the reference's parallel branch, with finite reciprocals (never 0 * inf)
    const auto nz = [](float x) { return fabsf(x) < RT_NZ_MIN ? copysignf(1e-20f, x) : x; };
    r.inv = mk(rcp(nz(r.d.x)), rcp(nz(r.d.y)), rcp(nz(r.d.z)));
    r.oinv = mk(r.o.x * r.inv.x, r.o.y * r.inv.y, r.o.z * r.inv.z);
#if RT_SLAB_CONS
    {   // fmaf(b, inv, -oinv) differs from (b - o) / d by <= 2^-24 |o / d| (oinv's rounding) + ~2^-21.7 |t| (the
        // reciprocal's 1 ulp, the fma's and the reference's roundings); parallel axes only decide inside / outside
        const float px = fabsf(r.d.x) < RT_NZ_MIN ? 0.0f : fabsf(r.oinv.x);
        const float py = fabsf(r.d.y) < RT_NZ_MIN ? 0.0f : fabsf(r.oinv.y);
        const float pz = fabsf(r.d.z) < RT_NZ_MIN ? 0.0f : fabsf(r.oinv.z);
        const float pad = 0x1p-22f * fmaxf(px, fmaxf(py, pz));
        r.pad = pad;
        if (XB != XD_CULL) {   // the exact-decision instances re-take every box test of a ray with a parallel axis
            const bool par = fabsf(r.d.x) < RT_NZ_MIN || fabsf(r.d.y) < RT_NZ_MIN || fabsf(r.d.z) < RT_NZ_MIN;
            r.pad = par ? -pad : pad;
        }
    }
#endif
#else
    (void)r;
#endif
}

// BoundingBox::hit (BoundingBox.cu:34-72), reference arithmetic.  b = {xmin,xmax,ymin,ymax,zmin,zmax}
__device__ __forceinline__ bool slab_ref(const float *b, const f3 &o, const f3 &d, float tmin, float tmax, float &te) {
    float cmin = tmin, cmax = tmax;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float q = comp(o, a), dd = comp(d, a), mn = b[2 * a], mx = b[2 * a + 1];
        if (fabsf(dd) < FZERO) {
            if (q < mn || q > mx) return false;
            continue;
        }
        const float t1 = fdiv(mn - q, dd);
        const float t2 = fdiv(mx - q, dd);
        if (t1 < t2) {
            if (t1 > cmin) cmin = t1;
            if (t2 < cmax) cmax = t2;
        } else {
            if (t2 > cmin) cmin = t2;
            if (t1 < cmax) cmax = t1;
        }
        if (cmin >= cmax) return false;
    }
    te = cmin;
    return true;
}

#if RT_SLAB_CONS && !RT_EXACT
// The reference's slab as one out-of-line copy for the FAST kernels' rare exact re-tests (inlined at every box test it
// would add its divisions to the hot loop's code and registers).  Returns the entry t, or NaN for a miss.
struct BoxArgs { float b[6]; f3 o, d; float tmax; };
__device__ __attribute__((noinline)) float slab_ref_entry(BoxArgs a) {
    float te = 0.0f;
    return slab_ref(a.b, a.o, a.d, TMIN, a.tmax, te) ? te : __builtin_nanf("");
}
// A FAST box decision: each end of the interval [lo, hi] (hi includes tmax) is within |pad| + 2^-20 |t| of the
// reference's (lo, hi >= TMIN > 0 wherever lo < hi can hold), so the widened test cons_lo(lo) < cons_hi(hi) keeps every
// box the reference's slab accepts (a cull is never wrong), and hi - lo > box_margin is an accept the reference shares;
// in between, the XB instances re-take the decision with the reference's slab (RT_BOX_EXACT)
__device__ __forceinline__ float cons_lo(float lo, float pad) { return fmaf(lo, 1.0f - 0x1p-20f, -fabsf(pad)); }
__device__ __forceinline__ float cons_hi(float hi, float pad) { return fmaf(hi, 1.0f + 0x1p-20f, fabsf(pad)); }
__device__ __forceinline__ float box_margin(float lo, float hi, float pad) { return fmaf(lo + hi, 0x1p-20f, 2.0f * fabsf(pad)); }
__device__ __forceinline__ bool ray_parallel(const RayP &r) { return __builtin_signbit(r.pad) != 0; }
#endif
// XB: decisions inside the margin re-taken with the reference's slab (RT_BOX_EXACT: the quad instance for the reference's
// own trees and the binary-pair one, where the traversal then takes exactly the reference's decisions)
template <int XB = XD_CULL>
__device__ __forceinline__ bool slab(const float *b, const RayP &r, float tmin, float tmax, float &te) {
#if RT_EXACT
    return slab_ref(b, r.o, r.d, tmin, tmax, te);
#else
    const float tx1 = fmaf(b[0], r.inv.x, -r.oinv.x), tx2 = fmaf(b[1], r.inv.x, -r.oinv.x);
    const float ty1 = fmaf(b[2], r.inv.y, -r.oinv.y), ty2 = fmaf(b[3], r.inv.y, -r.oinv.y);
    const float tz1 = fmaf(b[4], r.inv.z, -r.oinv.z), tz2 = fmaf(b[5], r.inv.z, -r.oinv.z);
    const float lo = fmaxf(fmaxf(tmin, fminf(tx1, tx2)), fmaxf(fminf(ty1, ty2), fminf(tz1, tz2)));
    const float hi = fminf(fminf(tmax, fmaxf(tx1, tx2)), fminf(fmaxf(ty1, ty2), fmaxf(tz1, tz2)));
    te = lo;
#if RT_SLAB_CONS
    bool h = cons_lo(lo, r.pad) < cons_hi(hi, r.pad);
#if RT_BOX_EXACT
    if ((XB == XD_ALL && h && !(hi - lo > box_margin(lo, hi, r.pad))) || (XB != XD_CULL && ray_parallel(r))) {
        // rare: the reference's decision
        BoxArgs a;
        for (int c = 0; c < 6; c++) a.b[c] = b[c];
        a.o = r.o; a.d = r.d; a.tmax = tmax;
        const float e = slab_ref_entry(a);            // (tmin is TMIN at every call site)
        h = e == e;
        if (h) te = e;
    }
#endif
    return h;
#else
    return lo < hi;
#endif
#endif
}

// ---- primitives (local space) ---------------------------------------------------------
__device__ __forceinline__ bool tri_test(const TriHot &T, const RayP &r, float tmin, float tmax,
                                         float &t, float &u, float &v) {      // Triangle.cu:4-44
    const f3 e1 = ld3(T.e1), e2 = ld3(T.e2), v0 = ld3(T.v0);
    const f3 h = cross(r.d, e2);
    const float det = dot(e1, h);
    if (fabsf(det) < FZERO) return false;
    const f3 s = sub(r.o, v0);
#if RT_IEEE_TRI
    u = dot(s, h) / det;
    if (!in_range(u, 0.0f, 1.0f)) return false;
    const f3 q = cross(s, e1);
    v = dot(r.d, q) / det;
    if (!in_range(v, 0.0f, 1.0f) || u + v > 1.0f) return false;
    t = dot(e2, q) / det;
    return in_range(t, tmin, tmax);
#else
    const float inv = __builtin_amdgcn_rcpf(det);
    const f3 q = cross(s, e1);
    u = dot(s, h) * inv;
    v = dot(r.d, q) * inv;
    t = dot(e2, q) * inv;
    return in_range(u, 0.0f, 1.0f) && in_range(v, 0.0f, 1.0f) && !(u + v > 1.0f) && in_range(t, tmin, tmax);
#endif
}

__device__ __forceinline__ bool sphere_test(const SphereHot &S, const RayP &r, float tmin, float tmax, float &t) {
    const f3 c = ld3(S.center);                                               // Sphere.cu:4-28
    const f3 cq = sub(c, r.o);
    const float a = dot(r.d, r.d);
    const float b = -2.0f * dot(cq, r.d);
    const float cc = dot(cq, cq) - S.radius * S.radius;
    float delta = b * b - 4.0f * a * cc;
    if (delta < 0.0f) return false;
    delta = sqrtf(delta);
    // the far root only when the near one is out of range (the same values; one correctly rounded division less
    // for every ray that hits a sphere from outside, e.g. the ground)
    const float root1 = fdiv(-b - delta, a * 2.0f);
    if (in_range(root1, tmin, tmax)) { t = root1; return true; }
    const float root2 = fdiv(-b + delta, a * 2.0f);
    if (in_range(root2, tmin, tmax)) { t = root2; return true; }
    return false;
}

__device__ __forceinline__ bool quad_test(const QuadHot &Q, const RayP &r, float tmin, float tmax,
                                          float &t, float &al, float &be) {   // Parallelogram.cu:4-36
    const f3 n = ld3(Q.n);
    const float ndd = dot(n, r.d);
    if (fabsf(ndd) < FZERO) return false;
    float ndp = 0.0f;
    ndp += n.x * r.o.x; ndp += n.y * r.o.y; ndp += n.z * r.o.z;
    const float tt = fdiv(Q.d - ndp, ndd);
    if (!in_range(tt, tmin, tmax)) return false;
    const f3 inter = add(r.o, scl(r.d, tt));
    const f3 p = sub(inter, ld3(Q.q));
    const f3 nx = ld3(Q.nx);
    if (fabsf(Q.den) < FZERO) return false;
    al = fdiv(dot(cross(p, ld3(Q.v)), nx), Q.den);
    if (!in_range(al, 0.0f, 1.0f)) return false;                              // (the reference tests both after)
    be = fdiv(dot(cross(ld3(Q.u), p), nx), Q.den);
    if (!in_range(be, 0.0f, 1.0f)) return false;
    t = tt;
    return true;
}

// (M * toMatrix(Point3)).toPoint() / (M * toMatrix(Vec3)).toVector() over rows 1..3 of a 4x4
// (Matrix.cu:71-86); m = 12 floats (3 rows x 4 cols).
__device__ __forceinline__ f3 xf_point(const float *m, f3 p) {
    f3 r;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        float s = 0.0f;
        s += m[4 * i] * p.x; s += m[4 * i + 1] * p.y; s += m[4 * i + 2] * p.z; s += m[4 * i + 3] * 1.0f;
        if (i == 0) r.x = s; else if (i == 1) r.y = s; else r.z = s;
    }
    return r;
}
__device__ __forceinline__ f3 xf_vector(const float *m, f3 v) {
    f3 r;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        float s = 0.0f;
        s += m[4 * i] * v.x; s += m[4 * i + 1] * v.y; s += m[4 * i + 2] * v.z;
#if RT_EXACT
        s += m[4 * i + 3] * 0.0f;     // keeps the sign-of-zero behaviour of the 4x4 product
#endif
        if (i == 0) r.x = s; else if (i == 1) r.y = s; else r.z = s;
    }
    return r;
}

// ---- closest hit -----------------------------------------------------------------------
struct Hit {
    float t;
    uint32_t inst;     // instance index
    uint32_t ptype;    // primitive type
    uint32_t slot;     // leaf-ordered slot in the type's array
    float u, v;
};

struct LaneCount { uint32_t pairs, tri, sq, quad, inst, hits, overflow; };

// Per-lane traversal stack: a window of LDS_DEPTH entries in LDS (layout [depth][BLOCK]: a wave's
// 64 lanes touch 64 consecutive u64 at any depth -> bank-conflict-free ds_*_b64) backed by a
// scratch array.  Push/pop only touch LDS; when the window fills, its bottom half is paged out to
// scratch, and when it empties the most recent half-page is paged back in (rare: median-split
// trees stay within 16 entries up to ~1k instances x 1k triangles).  Capacity LDS_DEPTH +
// SPILL_DEPTH = 64 entries, the reference's stack size (BLAS.cu:129, TLAS.cu:138).
struct SEnt { uint32_t ref; uint32_t tn; };   // node ref, entry t (float bits)
// LDS entries are stored packed as u64 (low = ref, high = entry t bits)
typedef __attribute__((address_space(3))) unsigned long long LdsU2;
__device__ __forceinline__ unsigned long long pack(SEnt e) { return (unsigned long long)e.ref | ((unsigned long long)e.tn << 32); }
__device__ __forceinline__ SEnt unpack(unsigned long long v) { SEnt e; e.ref = (uint32_t)v; e.tn = (uint32_t)(v >> 32); return e; }
constexpr int HALF = LDS_DEPTH / 2;

struct Stack {
    LdsU2 *lds;            // &lds_stack[0][tid]; entry k at lds[k * BLOCK]
    int sp;                // entries in the LDS window
    int spilled;           // entries paged out to scratch
    __device__ __forceinline__ bool empty() const { return sp == 0 && spilled == 0; }
};

// A half-page (HALF entries = 64 B, 16 B-aligned: pages start at multiples of HALF) moves as 16 B pieces; a
// page-in requests all four before the first LDS write.  (A contiguous row per thread in HBM instead of
// lane-swizzled scratch measured 3 % slower with the same WRITE_SIZE: paging is not the write excess)
__device__ __forceinline__ void spill_store(SEnt *dst, const Stack &stk) {
    uint4 *d = reinterpret_cast<uint4 *>(__builtin_assume_aligned(dst, 16));
#pragma unroll
    for (int k = 0; k < HALF; k += 2) {
        const unsigned long long a = stk.lds[k * BLOCK], b = stk.lds[(k + 1) * BLOCK];
        d[k / 2] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    }
}
__device__ __forceinline__ void spill_load(const SEnt *src, Stack &stk) {
    const uint4 *p = reinterpret_cast<const uint4 *>(__builtin_assume_aligned(src, 16));
#pragma unroll
    for (int k = 0; k < HALF; k += 2) {
        const uint4 v = p[k / 2];
        stk.lds[k * BLOCK] = (unsigned long long)v.x | ((unsigned long long)v.y << 32);
        stk.lds[(k + 1) * BLOCK] = (unsigned long long)v.z | ((unsigned long long)v.w << 32);
    }
}
__device__ __forceinline__ void stack_page_out(Stack &stk, SEnt *spill, LaneCount &c) {
    if (stk.spilled + HALF > SPILL_DEPTH) {        // deeper than the reference's 64 entries
        c.overflow++;
        stk.spilled = SPILL_DEPTH - HALF;          // drop the oldest half-page (result flagged)
    }
    spill_store(spill + stk.spilled, stk);
#pragma unroll
    for (int k = 0; k < HALF; k++) stk.lds[k * BLOCK] = stk.lds[(k + HALF) * BLOCK];
    stk.sp = HALF;
    stk.spilled += HALF;
}
__device__ __forceinline__ void stack_page_in(Stack &stk, const SEnt *spill) {
    stk.spilled -= HALF;
    spill_load(spill + stk.spilled, stk);
    stk.sp = HALF;
}
__device__ __forceinline__ void stack_push(Stack &stk, SEnt *spill, uint32_t ref, float tn, LaneCount &c) {
    if (stk.sp == LDS_DEPTH) stack_page_out(stk, spill, c);
    SEnt e;
    e.ref = ref;
    e.tn = __float_as_uint(tn);
    stk.lds[stk.sp * BLOCK] = pack(e);
    stk.sp++;
}
__device__ __forceinline__ SEnt stack_pop(Stack &stk, const SEnt *spill) {   // precondition: !empty()
    if (stk.sp == 0) stack_page_in(stk, spill);
    --stk.sp;
    return unpack(stk.lds[stk.sp * BLOCK]);
}

// Page the bottom half of the LDS window out when fewer than 3 slots are free (sp > HALF; slots >= sp
// are free space, moved along harmlessly).
__device__ __forceinline__ void stack_page_out3(Stack &stk, SEnt *spill, LaneCount &c) {   // sp > HALF
    if (stk.spilled + HALF > SPILL_DEPTH) {
        c.overflow++;
        stk.spilled = SPILL_DEPTH - HALF;
    }
    spill_store(spill + stk.spilled, stk);
#pragma unroll
    for (int k = 0; k < HALF; k++) stk.lds[k * BLOCK] = stk.lds[(k + HALF) * BLOCK];   // slots >= sp: don't care
    stk.sp -= HALF;
    stk.spilled += HALF;
}

// Resumable per-lane traversal state: TLAS::hit (TLAS.cu:131-201) as a state machine so that a
// persistent wave can interleave traversal steps with shading / ray regeneration of other lanes.
constexpr uint32_t REF_NONE = 0xFFFFFFFFu;   // leaf bit + primitive type 3: never a real ref

struct Trav {
    RayP wr, lr;           // world-space ray, instance-space ray of cur_inst
    float tmax;            // currentRange.max
    uint32_t cur;          // node to process next (REF_NONE: stack exhausted)
    float curT;            // entry t of cur (speculative traversal re-checks it)
    uint32_t pleaf;        // postponed leaf (speculative traversal), REF_NONE if none
    uint32_t cur_inst;
    Hit hit;
    bool found;
    bool tracing;
    Stack stk;
};

// A popped entry (or the speculative successor) survives its re-test: the reference re-runs the box test with the
// current tmax, which accepts it iff its entry t < tmax (the exit side passed at the push and tmax only shrinks).
// RT_SLAB_CONS: the entry is widened by its ray's bound first (a BLAS entry belongs to the current instance's ray).
__device__ __forceinline__ bool pop_keep(const Trav &T, float tn, uint32_t ref) {
#if !RT_EXACT && RT_SLAB_CONS
    return cons_lo(tn, (ref & REF_BLAS) ? T.lr.pad : T.wr.pad) < T.tmax;
#else
    (void)ref;
    return tn < T.tmax;
#endif
}

// R: this frame's TLAS root (the persistent kernel holds it in SGPRs, loaded once per wave)
template <int XB = XD_CULL>
__device__ __forceinline__ void trav_init(Trav &T, const TreeRoot &R, const f3 &o, const f3 &d) {
    T.wr.o = o; T.wr.d = d; prep<XB>(T.wr);
    T.lr = T.wr;
    T.tmax = __builtin_huge_valf();
    T.found = false;
    T.stk.sp = 0;
    T.stk.spilled = 0;
    T.cur = R.ref;
    T.cur_inst = 0;
    T.pleaf = REF_NONE;
    float te = 0.0f;
    T.tracing = slab<XB>(R.box, T.wr, TMIN, T.tmax, te);                 // root pop test (TLAS.cu:150)
    T.curT = te;
}
template <int XB = XD_CULL>
__device__ __forceinline__ void trav_init(Trav &T, const SceneGPU &sc, const f3 &o, const f3 &d) {
    trav_init<XB>(T, *sc.tlas_root, o, d);
}

// The frame's TLAS root as wave-uniform values (SGPRs): read once per wave instead of per ray.
template <bool WIDE>
__device__ __forceinline__ TreeRoot uniform_root(const SceneGPU &sc) {
    const float4 *p = reinterpret_cast<const float4 *>(WIDE ? sc.tlas_root_wide : sc.tlas_root);
    const float4 a = p[0], b = p[1];
    auto u = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
    TreeRoot R;
    R.box[0] = u(a.x); R.box[1] = u(a.y); R.box[2] = u(a.z); R.box[3] = u(a.w);
    R.box[4] = u(b.x); R.box[5] = u(b.y);
    R.ref = (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(b.z));
    R.height = 0;
    return R;
}

// Process T.cur (one node pair, one TLAS leaf instance or one BLAS leaf), then choose the next node:
// the near child, or a popped entry surviving the re-test; clears T.tracing when the stack is dry.
// XB (FAST builds): box decisions inside the slab error margin re-taken with the reference's slab (rt_trace_rays and
// the grid kernel: the binary pairs in the reference's order, so their decisions are the reference's)
template <bool COUNT, int XB = XD_CULL>
__device__ __forceinline__ void trav_step(Trav &T, const SceneGPU &sc, SEnt *spill, LaneCount &cnt) {
    const uint32_t cur = T.cur;
    if (!(cur & REF_LEAF)) {
        // interior node pair: test both children (TLAS.cu:175-197 / BLAS.cu:178-202)
        const bool blas = (cur & REF_BLAS) != 0;
        const NodePair *P = (blas ? sc.blas_pairs : sc.tlas_pairs) + (cur & REF_INDEX_MASK);
        const float4 *P4 = reinterpret_cast<const float4 *>(P);
        const float4 A = P4[0], B = P4[1], Cc = P4[2];
        const uint4 D = reinterpret_cast<const uint4 *>(P)[3];
        const float b0[6] = {A.x, A.y, A.z, A.w, B.x, B.y};
        const float b1[6] = {B.z, B.w, Cc.x, Cc.y, Cc.z, Cc.w};
        if (COUNT) cnt.pairs++;
        float e0 = 0.0f, e1 = 0.0f;
        const RayP &r = blas ? T.lr : T.wr;
        const bool h0 = slab<XB>(b0, r, TMIN, T.tmax, e0);
        const bool h1 = slab<XB>(b1, r, TMIN, T.tmax, e1);
        if (h0 && h1) {
            // reference: tLeft > tRight -> push left then right (right popped first)
            const bool right_near = e0 > e1;
            stack_push(T.stk, spill, right_near ? D.x : D.y, right_near ? e0 : e1, cnt);
            T.cur = right_near ? D.y : D.x;
            return;
        }
        if (h0) { T.cur = D.x; return; }
        if (h1) { T.cur = D.y; return; }
    } else if (!(cur & REF_BLAS)) {
        // TLAS leaf: its instances in order (TLAS.cu:157-173)
        const uint32_t start = ref_leaf_start(cur), count = ref_leaf_count(cur);
        if (count > 1) stack_push(T.stk, spill, make_leaf_ref(start + 1, count - 1, 0, false), -__builtin_huge_valf(), cnt);
        T.cur_inst = sc.inst_by_slot ? start : sc.tlas_slots[start];
        const InstHot &I = sc.inst_hot[T.cur_inst];
        if (COUNT) cnt.inst++;
        // Instance::hit: ray into local space, d' not renormalised (Instance.cu:26-27)
        T.lr.o = xf_point(I.inv, T.wr.o);
        T.lr.d = xf_vector(I.inv, T.wr.d);
        prep<XB>(T.lr);
        float te;
        if (slab<XB>(I.root_box, T.lr, TMIN, T.tmax, te)) { T.cur = I.root_ref; return; }   // BLAS root pop test
    } else {
        // BLAS leaf: primitives in leaf order (BLAS.cu:153-176)
        const uint32_t start = ref_leaf_start(cur), count = ref_leaf_count(cur), type = ref_leaf_type(cur);
        for (uint32_t k = 0; k < count; k++) {
            const uint32_t slot = start + k;
            float t = 0.0f, u = 0.0f, v = 0.0f;
            bool h;
            if (type == RT_PRIM_TRIANGLE) {
                if (COUNT) cnt.tri++;
                h = tri_test(sc.tri_hot[slot], T.lr, TMIN, T.tmax, t, u, v);
            } else if (type == RT_PRIM_SPHERE) {
                if (COUNT) cnt.sq++;
                h = sphere_test(sc.sph_hot[slot], T.lr, TMIN, T.tmax, t);
            } else {
                if (COUNT) { cnt.sq++; cnt.quad++; }
                h = quad_test(sc.quad_hot[slot], T.lr, TMIN, T.tmax, t, u, v);
            }
            if (h) {
                T.found = true; T.tmax = t;
                T.hit.t = t; T.hit.inst = T.cur_inst; T.hit.ptype = type; T.hit.slot = slot; T.hit.u = u; T.hit.v = v;
            }
        }
    }
    // pop until an entry survives the re-test (entry t < tmax)
    while (!T.stk.empty()) {
        const SEnt e = stack_pop(T.stk, spill);
        if (pop_keep(T, __uint_as_float(e.tn), e.ref)) { T.cur = e.ref; return; }
    }
    T.tracing = false;
}

// ---- speculative while-while traversal (Aila & Laine 2009), reference-order preserving ----------
// Phase 1 (interior loop): every lane walks interior node pairs; the first leaf a lane reaches is
// postponed (pleaf) and the lane keeps walking (speculatively) until it meets a second leaf; the
// wave leaves the loop once every traversing lane holds a postponed leaf.  Phase 2 processes the
// postponed leaves together.  The reference processes a leaf before the nodes that follow it, with
// the tmax the leaf produced.  Speculative steps used the older (larger) tmax, so:
//   * the postponed leaf itself passed its test with the current tmax (no leaf ran in between);
//   * entries pushed speculatively are re-tested at pop (entry t < tmax), as always;
//   * the node the lane stopped at (cur) is re-tested after the leaf: every node reached below a node
//     N has entry t >= N's entry t (child boxes lie inside parent boxes and the slab entry is
//     monotone in the box bounds), so cur fails its re-test whenever the reference would have culled
//     N or any node on the way.
// Hence leaves are processed in the reference order with the reference's tmax: same hits, same
// primitive tests, same instance visits (only extra node-pair tests are speculative).
__device__ __forceinline__ void pop_next(Trav &T, const SEnt *spill) {
    while (!T.stk.empty()) {
        const SEnt e = stack_pop(T.stk, spill);
        const float tn = __uint_as_float(e.tn);
        if (pop_keep(T, tn, e.ref)) { T.cur = e.ref; T.curT = tn; return; }
    }
    T.cur = REF_NONE;
}

// One interior-loop step of a lane whose cur is an interior node, or a leaf to postpone.
#if !RT_EXACT
// Quad node (option "wide", layout.hpp NodeQuad): 4 slab tests on SoA bounds; the hit slots are visited
//   PAIR (quads of two binary levels: the reference's trees, GPU-built trees): in the reference's order — the two
//     halves (binary children) by their boxes' entry t, then the slots of a half by theirs, the nearer first and the
//     left one on ties (BLAS.cu:186-202, TLAS.cu:182-197) — so the closest hit is the reference's, ties included;
//   else (host SAH trees, collapsed greedily): by entry t, nearest first (measured against the oracle: DESIGN §3.4).
// The first is visited next and the others pushed last-first, each with its own entry t for the pop re-test (a
// half's box holds its slots' boxes, so its re-test passes whenever one of theirs does).
// Option "lds_scene" (SceneGPU::lds_quads / lds_insts): the frame's TLAS quads and instance hot records,
// copied into LDS by every workgroup of the persistent quad-tree kernel at its start.  On C2 an average
// ray visits ~1.6 quads (mostly TLAS) and enters ~1 instance, so most of its dependent loads are these.
__shared__ float4 lds_scene[LDS_SCENE_F4];

struct InstRec { float4 i0, i1, i2, box01, box2ref; };   // InstHot as 5 dwordx4 (inv rows, root box, refs)
template <bool LDSS>
__device__ __forceinline__ InstRec load_inst(const SceneGPU &sc, uint32_t i) {
    InstRec r;
    if (LDSS && sc.lds_insts) {
        const float4 *p = lds_scene + sc.lds_quads * LDS_QUAD_F4 + i * LDS_INST_F4;
        r.i0 = p[0]; r.i1 = p[1]; r.i2 = p[2]; r.box01 = p[3]; r.box2ref = p[4];
    } else {
        const float4 *p = reinterpret_cast<const float4 *>(sc.inst_hot + i);
        r.i0 = p[0]; r.i1 = p[1]; r.i2 = p[2]; r.box01 = p[3]; r.box2ref = p[4];
    }
    return r;
}
// the workgroup's copy (before the kernel's first barrier)
__device__ __forceinline__ void lds_scene_fill(const SceneGPU &sc) {
    const uint32_t nq = sc.lds_quads * LDS_QUAD_F4, ni = sc.lds_insts * LDS_INST_F4;
    const float4 *q = reinterpret_cast<const float4 *>(sc.tlas_quads);
    for (uint32_t i = threadIdx.x; i < nq; i += BLOCK) {
        const uint32_t k = i / LDS_QUAD_F4, j = i - k * LDS_QUAD_F4;
        lds_scene[i] = q[k * 8 + j];
    }
    const float4 *h = reinterpret_cast<const float4 *>(sc.inst_hot);
    for (uint32_t i = threadIdx.x; i < ni; i += BLOCK) lds_scene[nq + i] = h[i];
    const auto copy = [](uint32_t at, const void *src, uint32_t n4) {
        if (at == LDS_NONE) return;
        const float4 *p = reinterpret_cast<const float4 *>(src);
        for (uint32_t i = threadIdx.x; i < n4; i += BLOCK) lds_scene[at + i] = p[i];
    };
    copy(sc.lds_icold, sc.inst_cold, sc.instance_count * LDS_ICOLD_F4);
    copy(sc.lds_sph_hot, sc.sph_hot, sc.lds_sph_cold - sc.lds_sph_hot);
    copy(sc.lds_sph_cold, sc.sph_cold, sc.lds_sph_cold - sc.lds_sph_hot);
    copy(sc.lds_q_hot, sc.quad_hot, (sc.lds_q_cold - sc.lds_q_hot));
    copy(sc.lds_q_cold, sc.quad_cold, (sc.lds_q_cold - sc.lds_q_hot) / LDS_QPRIM_F4);
    const float4 *bq = reinterpret_cast<const float4 *>(sc.blas_quads + sc.lds_bq0);   // a group BLAS's top levels
    for (uint32_t i = threadIdx.x; i < sc.lds_bqn * LDS_QUAD_F4; i += BLOCK) {
        const uint32_t k = i / LDS_QUAD_F4, j = i - k * LDS_QUAD_F4;
        lds_scene[sc.lds_bq_at + i] = bq[k * 8 + j];
    }
}
// record k of an array that may be resident in the LDS scene region (at = its dwordx4 offset, LDS_NONE = HBM)
template <typename R>
__device__ __forceinline__ R lds_or_global(uint32_t at, const R *g, uint32_t k) {
    constexpr uint32_t N4 = sizeof(R) / 16;
    R r;
    float4 *d = reinterpret_cast<float4 *>(&r);
    if (at != LDS_NONE) {
#pragma unroll
        for (uint32_t j = 0; j < N4; j++) d[j] = lds_scene[at + k * N4 + j];
    } else {
        const float4 *p = reinterpret_cast<const float4 *>(g + k);
#pragma unroll
        for (uint32_t j = 0; j < N4; j++) d[j] = p[j];
    }
    return r;
}

// one axis of the 4 slot slab tests; pa / pb: that axis's contribution to the entry t of the halves' boxes (a
// half's box is the union of its two slots' boxes, and the plane distances are monotone in the bound, so its near
// plane is the nearer of its slots' near planes)
template <bool PAIR>
__device__ __forceinline__ void slab4(const float4 &lo, const float4 &hi, float inv, float oinv, float4 &tn, float4 &tf,
                                      float &pa, float &pb) {
    const float a0 = fmaf(lo.x, inv, -oinv), b0 = fmaf(hi.x, inv, -oinv);
    const float a1 = fmaf(lo.y, inv, -oinv), b1 = fmaf(hi.y, inv, -oinv);
    const float a2 = fmaf(lo.z, inv, -oinv), b2 = fmaf(hi.z, inv, -oinv);
    const float a3 = fmaf(lo.w, inv, -oinv), b3 = fmaf(hi.w, inv, -oinv);
    const float n0 = fminf(a0, b0), n1 = fminf(a1, b1), n2 = fminf(a2, b2), n3 = fminf(a3, b3);
    tn = make_float4(fmaxf(tn.x, n0), fmaxf(tn.y, n1), fmaxf(tn.z, n2), fmaxf(tn.w, n3));
    tf = make_float4(fminf(tf.x, fmaxf(a0, b0)), fminf(tf.y, fmaxf(a1, b1)), fminf(tf.z, fmaxf(a2, b2)), fminf(tf.w, fmaxf(a3, b3)));
    if (PAIR) {
        pa = fmaxf(pa, fminf(n0, n1));
        pb = fmaxf(pb, fminf(n2, n3));
    }
}
__device__ __forceinline__ float comp4(const float4 &v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w)); }
__device__ __forceinline__ void cswap(float &ta, uint32_t &ra, float &tb, uint32_t &rb) {
    const bool sw = tb < ta;
    const float t = sw ? tb : ta, u = sw ? ta : tb;
    const uint32_t r = sw ? rb : ra, q = sw ? ra : rb;
    ta = t; tb = u; ra = r; rb = q;
}
// The hit decisions and entry t's of a quad's 4 slots (and, PAIR, of its two halves' boxes) for ray r with the current
// tmax: FAST reciprocal slabs, conservative (RT_SLAB_CONS); XB: decisions inside the error margin re-taken with the
// reference's division slab on the node's bounds re-read from Q.  Shared by the traversal step and the box-test entry
// point the parity tests call (rt_box_test, RT_BOX_QUAD_*).
template <bool PAIR, int XB>
__device__ __forceinline__ void quad_decide(const float4 *Q, const float4 &lx, const float4 &hx, const float4 &ly,
                                            const float4 &hy, const float4 &lz, const float4 &hz, const uint4 &R,
                                            const RayP &r, float tmax, float (&t)[4], bool (&h)[4], float &pa, float &pb) {
    bool und[4] = {false, false, false, false};   // und: hit decision inside the error margin
    // XD_ALL: whether an entry t is TMIN for certain — every entry plane below TMIN by more than the error bound, so the
    // reference's is TMIN too.  Two such entries compare equal in both slabs (the ray starts inside both boxes: most
    // nodes around a bounce origin), so their order needs no re-take.
    bool low[4] = {false, false, false, false}, low_a = false, low_b = false;
    const float t0 = XB == XD_ALL ? -__builtin_huge_valf() : TMIN;
    pa = t0; pb = t0;                                // entry t of the two halves' boxes
    {
        float4 tn = make_float4(t0, t0, t0, t0), tf = make_float4(tmax, tmax, tmax, tmax);
        slab4<PAIR>(lx, hx, r.inv.x, r.oinv.x, tn, tf, pa, pb);
        slab4<PAIR>(ly, hy, r.inv.y, r.oinv.y, tn, tf, pa, pb);
        slab4<PAIR>(lz, hz, r.inv.z, r.oinv.z, tn, tf, pa, pb);
        if (XB == XD_ALL) {
            const auto below = [&](float v) { return fmaf(fabsf(v), 0x1p-19f, v + 2.0f * fabsf(r.pad)) < TMIN; };
            low[0] = below(tn.x); low[1] = below(tn.y); low[2] = below(tn.z); low[3] = below(tn.w);
            low_a = below(pa); low_b = below(pb);
            tn = make_float4(fmaxf(tn.x, TMIN), fmaxf(tn.y, TMIN), fmaxf(tn.z, TMIN), fmaxf(tn.w, TMIN));
            pa = fmaxf(pa, TMIN); pb = fmaxf(pb, TMIN);
        }
        t[0] = tn.x; t[1] = tn.y; t[2] = tn.z; t[3] = tn.w;
#if RT_SLAB_CONS
        h[0] = cons_lo(tn.x, r.pad) < cons_hi(tf.x, r.pad); h[1] = cons_lo(tn.y, r.pad) < cons_hi(tf.y, r.pad);
        h[2] = cons_lo(tn.z, r.pad) < cons_hi(tf.z, r.pad); h[3] = cons_lo(tn.w, r.pad) < cons_hi(tf.w, r.pad);
        if (XB == XD_ALL) {
            und[0] = !(tf.x - tn.x > box_margin(tn.x, tf.x, r.pad)); und[1] = !(tf.y - tn.y > box_margin(tn.y, tf.y, r.pad));
            und[2] = !(tf.z - tn.z > box_margin(tn.z, tf.z, r.pad)); und[3] = !(tf.w - tn.w > box_margin(tn.w, tf.w, r.pad));
        }
#else
        h[0] = tn.x < tf.x; h[1] = tn.y < tf.y; h[2] = tn.z < tf.z; h[3] = tn.w < tf.w;
#endif
    }
    // an empty slot repeats its sibling's box (the half's union stays exact) and is never accepted
    h[1] = h[1] && R.y != REF_EMPTY;
    h[3] = h[3] && R.w != REF_EMPTY;
#if RT_SLAB_CONS && RT_BOX_EXACT
    if (XB != XD_CULL) {   // Rare: a hit decision inside the error margin, a ray with a parallel axis, or (pair order) two entry t's the order
        // compares inside the margin — then the boxes involved (a ray with a parallel axis: every box of the node) are
        // re-tested with the reference's slab (a half's box: the union of its slots' boxes), on the node's bounds read
        // again (keeping the 24 bounds live through the step would cost registers on the hot path), one box per
        // iteration so that one copy of the division slab serves all six.  Boxes of the mask m: bit k = slot k, bits 4 / 5
        // = the halves.  Re-taking only the two entries a close comparison involves (round 6) instead of all six boxes
        // took C5 with exact decisions from 13.6 to 11.9 ms per serialised launch.
        const auto close = [&](float a, float b) { return fabsf(a - b) <= box_margin(a, b, r.pad); };
        uint32_t m = ray_parallel(r) ? (PAIR ? 0x3Fu : 0xFu) : 0u;
        if (XB == XD_ALL)
            m |= (h[0] && und[0] ? 1u : 0u) | (h[1] && und[1] ? 2u : 0u) | (h[2] && und[2] ? 4u : 0u) | (h[3] && und[3] ? 8u : 0u);
        if (PAIR && XB == XD_ALL)
            m |= (h[0] && h[1] && !(low[0] && low[1]) && close(t[0], t[1]) ? 0x3u : 0u) |
                 (h[2] && h[3] && !(low[2] && low[3]) && close(t[2], t[3]) ? 0xCu : 0u) |
                 ((h[0] || h[1]) && (h[2] || h[3]) && !(low_a && low_b) && close(pa, pb) ? 0x30u : 0u);
        if (m) {
            const float4 L[6] = {Q[0], Q[1], Q[2], Q[3], Q[4], Q[5]};
#pragma unroll 1
            for (; m; m &= m - 1u) {
                const int j = __builtin_ctz(m);
                const int k0 = j < 4 ? j : 2 * (j - 4), k1 = j < 4 ? j : k0 + 1;     // a slot, or a half's two slots
                float b[6];
#pragma unroll
                for (int c = 0; c < 6; c++) {
                    const float u = comp4(L[c], k0), v = comp4(L[c], k1);
                    b[c] = (c & 1) ? fmaxf(u, v) : fminf(u, v);
                }
                BoxArgs ba;
                for (int c = 0; c < 6; c++) ba.b[c] = b[c];
                ba.o = r.o; ba.d = r.d; ba.tmax = tmax;
                const float te = slab_ref_entry(ba);
                const bool hh = te == te;
                if (j < 4) {
                    const uint32_t rk = j == 0 ? R.x : (j == 1 ? R.y : (j == 2 ? R.z : R.w));
                    const bool live = rk != REF_EMPTY;
                    const bool hk = hh && live;
                    h[0] = j == 0 ? hk : h[0]; h[1] = j == 1 ? hk : h[1]; h[2] = j == 2 ? hk : h[2]; h[3] = j == 3 ? hk : h[3];
                    if (hk) { t[0] = j == 0 ? te : t[0]; t[1] = j == 1 ? te : t[1]; t[2] = j == 2 ? te : t[2]; t[3] = j == 3 ? te : t[3]; }
                } else if (hh) {
                    pa = j == 4 ? te : pa;
                    pb = j == 5 ? te : pb;
                }
            }
        }
    }
#endif
}

template <bool COUNT, bool PAIR, int XB>
__device__ __forceinline__ void wide_interior_step(Trav &T, const SceneGPU &sc, SEnt *spill, LaneCount &cnt) {
    const uint32_t cur = T.cur;
    const bool blas = (cur & REF_BLAS) != 0;
    float4 lx, hx, ly, hy, lz, hz;
    uint4 R;
    // one code path: a generic pointer into the LDS scene region or HBM (flat loads serve both)
    const float4 *Q;
    {
        const uint32_t qi = cur & REF_INDEX_MASK, qb = qi - sc.lds_bq0;
        const bool in_lds = blas ? qb < sc.lds_bqn : sc.lds_quads != 0;
        const uint32_t at = blas ? sc.lds_bq_at + qb * LDS_QUAD_F4 : qi * LDS_QUAD_F4;
        Q = in_lds ? static_cast<const float4 *>(lds_scene + at)
                   : reinterpret_cast<const float4 *>((blas ? sc.blas_quads : sc.tlas_quads) + qi);
        lx = Q[0]; hx = Q[1]; ly = Q[2]; hy = Q[3]; lz = Q[4]; hz = Q[5];
        R = reinterpret_cast<const uint4 *>(Q)[6];
    }
    // the child refs are needed only when a child is hit, so the compiler would issue their load after the slab
    // tests: a second dependent memory round trip per step.  Pinning them here keeps all 7 dwordx4 loads of the
    // node in one round trip.
    asm volatile("" ::"v"(R.x), "v"(R.y), "v"(R.z), "v"(R.w));
    if (COUNT) cnt.pairs += 2;                       // 4 child boxes = 2 node-pair equivalents
    const RayP &r = blas ? T.lr : T.wr;
    float t[4];
    bool h[4];
    float pa, pb;                                    // entry t of the two halves' boxes
    quad_decide<PAIR, XB>(Q, lx, hx, ly, hy, lz, hz, R, r, T.tmax, t, h, pa, pb);
    const float inf = __builtin_huge_valf();
    if (!PAIR) {
        float t0 = h[0] ? t[0] : inf, t1 = h[1] ? t[1] : inf, t2 = h[2] ? t[2] : inf, t3 = h[3] ? t[3] : inf;
        uint32_t r0 = R.x, r1 = R.y, r2 = R.z, r3 = R.w;
        const uint32_t nh = (uint32_t)h[0] + (uint32_t)h[1] + (uint32_t)h[2] + (uint32_t)h[3];
        if (nh == 0) { pop_next(T, spill); return; }
        // sort the 4 (t, ref) ascending; misses (t = inf) sink to the end
        cswap(t0, r0, t1, r1); cswap(t2, r2, t3, r3); cswap(t0, r0, t2, r2); cswap(t1, r1, t3, r3); cswap(t1, r1, t2, r2);
        // the 1..3 far hits go to the three LDS slots above the top without branching on their count (farthest
        // first; the slots past the new top are free space), after one page-out check
        if (nh > 1) {
            if (T.stk.sp > LDS_DEPTH - 3) stack_page_out3(T.stk, spill, cnt);
            SEnt a, b, c;
            a.ref = nh == 4 ? r3 : (nh == 3 ? r2 : r1);
            a.tn = __float_as_uint(nh == 4 ? t3 : (nh == 3 ? t2 : t1));
            b.ref = nh == 4 ? r2 : r1;
            b.tn = __float_as_uint(nh == 4 ? t2 : t1);
            c.ref = r1;
            c.tn = __float_as_uint(t1);
            T.stk.lds[T.stk.sp * BLOCK] = pack(a);
            T.stk.lds[(T.stk.sp + 1) * BLOCK] = pack(b);
            T.stk.lds[(T.stk.sp + 2) * BLOCK] = pack(c);
            T.stk.sp += (int)nh - 1;
        }
        T.cur = r0;
        T.curT = t0;
        return;
    }
    const uint32_t na = (uint32_t)h[0] + (uint32_t)h[1], nb = (uint32_t)h[2] + (uint32_t)h[3];
    if (na + nb == 0) { pop_next(T, spill); return; }
    // The reference's visit order (BLAS.cu:186-202: push far, visit near, the right child first iff tLeft > tRight):
    // inside each half its two slots, then the halves by their boxes' entry t.  A missed slot counts as t = +inf, so
    // it is second in its half, and a half without hits goes second; the hits then come first in each half.
    const float u0 = h[0] ? t[0] : inf, u1 = h[1] ? t[1] : inf, u2 = h[2] ? t[2] : inf, u3 = h[3] ? t[3] : inf;
    const bool sa = u0 > u1, sb = u2 > u3;
    const float a0t = sa ? u1 : u0, a1t = sa ? u0 : u1, b0t = sb ? u3 : u2, b1t = sb ? u2 : u3;
    const uint32_t a0r = sa ? R.y : R.x, a1r = sa ? R.x : R.y, b0r = sb ? R.w : R.z, b1r = sb ? R.z : R.w;
    const bool sr = na == 0 || (nb != 0 && pa > pb);                 // the right half first
    const float n0t = sr ? b0t : a0t, n1t = sr ? b1t : a1t, f0t = sr ? a0t : b0t, f1t = sr ? a1t : b1t;
    const uint32_t n0r = sr ? b0r : a0r, n1r = sr ? b1r : a1r, f0r = sr ? a0r : b0r, f1r = sr ? a1r : b1r;
    const uint32_t nn = sr ? nb : na, nf = sr ? na : nb;             // hits in the near / far half (nn >= 1)
    // the near half's first hit is visited next; the rest go to the three LDS slots above the top, deepest first
    // (far half's second, its first, the near half's second), without branching on their count, after one
    // page-out check
    const uint32_t npush = nn - 1u + nf;
    if (npush > 0) {
        if (T.stk.sp > LDS_DEPTH - 3) stack_page_out3(T.stk, spill, cnt);
        SEnt a, b, c;
        a.ref = nf == 2 ? f1r : (nf == 1 ? f0r : n1r);
        a.tn = __float_as_uint(nf == 2 ? f1t : (nf == 1 ? f0t : n1t));
        b.ref = nf == 2 ? f0r : n1r;
        b.tn = __float_as_uint(nf == 2 ? f0t : n1t);
        c.ref = n1r;
        c.tn = __float_as_uint(n1t);
        T.stk.lds[T.stk.sp * BLOCK] = pack(a);
        T.stk.lds[(T.stk.sp + 1) * BLOCK] = pack(b);
        T.stk.lds[(T.stk.sp + 2) * BLOCK] = pack(c);
        T.stk.sp += (int)npush;
    }
    T.cur = n0r;
    T.curT = n0t;
}
#endif

template <bool COUNT, int WIDE = 0>
__device__ __forceinline__ void spec_interior_step(Trav &T, const SceneGPU &sc, SEnt *spill, LaneCount &cnt) {
    const uint32_t cur = T.cur;
#if !RT_EXACT
    if (WIDE) {
        if (!(cur & REF_LEAF)) wide_interior_step<COUNT, (WIDE >= 2), XBOX(WIDE)>(T, sc, spill, cnt);
        else { T.pleaf = cur; pop_next(T, spill); }        // postpone, keep walking
        return;
    }
#endif
    if (!(cur & REF_LEAF)) {
        const bool blas = (cur & REF_BLAS) != 0;
        const NodePair *P = (blas ? sc.blas_pairs : sc.tlas_pairs) + (cur & REF_INDEX_MASK);
        const float4 *P4 = reinterpret_cast<const float4 *>(P);
        const float4 A = P4[0], B = P4[1], Cc = P4[2];
        const uint4 D = reinterpret_cast<const uint4 *>(P)[3];
        const float b0[6] = {A.x, A.y, A.z, A.w, B.x, B.y};
        const float b1[6] = {B.z, B.w, Cc.x, Cc.y, Cc.z, Cc.w};
        if (COUNT) cnt.pairs++;
        float e0 = 0.0f, e1 = 0.0f;
        const RayP &r = blas ? T.lr : T.wr;
        const bool h0 = slab<XBOX(WIDE)>(b0, r, TMIN, T.tmax, e0);
        const bool h1 = slab<XBOX(WIDE)>(b1, r, TMIN, T.tmax, e1);
        if (h0 && h1) {
            const bool right_near = e0 > e1;          // TLAS.cu:185-192 ordering
            stack_push(T.stk, spill, right_near ? D.x : D.y, right_near ? e0 : e1, cnt);
            T.cur = right_near ? D.y : D.x;
            T.curT = right_near ? e1 : e0;
            return;
        }
        if (h0 || h1) {
            T.cur = h0 ? D.x : D.y;
            T.curT = h0 ? e0 : e1;
            return;
        }
        pop_next(T, spill);
    } else {
        T.pleaf = cur;                                // postpone, keep walking
        pop_next(T, spill);
    }
}

// Process the postponed leaf, then resume at cur (re-tested) — TLAS.cu:157-173 / BLAS.cu:153-176.
// a sphere / parallelogram record: from the LDS scene region in the quad-tree kernel when resident
#if RT_EXACT
#define WIDE_LDS_REC(at, arr, k) (arr)[k]
#else
#define WIDE_LDS_REC(at, arr, k) (WIDE ? lds_or_global((at), (arr), (k)) : (arr)[k])
#endif
// FAST quad trees (RT_CHAIN_ROOT_LEAF): when the entered instance's BLAS root is itself a leaf, its
// primitives are tested in this same round, as BLAS::hit tests a leaf root right after the root box
// (BLAS.cu:140-176) — the speculative successor waits on the stack as before and is popped (re-tested)
// after the tests.  A segment against the demo's spheres / parallelogram then takes one round, not two.
// Returns 1 when a root leaf was chained (it counts as a step of its own in the unit costs, so the
// claim order's cost classes keep the scale they were tuned on).
template <bool COUNT, int WIDE = 0>
__device__ __forceinline__ uint32_t spec_leaf_phase(Trav &T, const SceneGPU &sc, SEnt *spill, LaneCount &cnt) {
    uint32_t leaf = T.pleaf;
    bool chained = false;
    T.pleaf = REF_NONE;
    if (!(leaf & REF_BLAS)) {
        // TLAS leaf: enter the first instance's BLAS; the speculative successor and the leaf's
        // remaining instances wait on the stack (popped in reference order).
        const uint32_t start = ref_leaf_start(leaf), count = ref_leaf_count(leaf);
        if (T.cur != REF_NONE) stack_push(T.stk, spill, T.cur, T.curT, cnt);
        if (count > 1) stack_push(T.stk, spill, make_leaf_ref(start + 1, count - 1, 0, false), -__builtin_huge_valf(), cnt);
        T.cur_inst = sc.inst_by_slot ? start : sc.tlas_slots[start];
        if (COUNT) cnt.inst++;
        float te = 0.0f;
#if !RT_EXACT
        if (WIDE) {
            const InstRec I = load_inst<true>(sc, T.cur_inst);
            // all 5 dwordx4 of the record in one round trip (the root ref is used only when the root box is hit,
            // so its load would otherwise be issued after the slab test)
            asm volatile("" ::"v"(I.i2.x), "v"(I.i2.y), "v"(I.i2.z), "v"(I.i2.w), "v"(I.box2ref.w));
            const float inv[12] = {I.i0.x, I.i0.y, I.i0.z, I.i0.w, I.i1.x, I.i1.y, I.i1.z, I.i1.w,
                                   I.i2.x, I.i2.y, I.i2.z, I.i2.w};
            const float box[6] = {I.box01.x, I.box01.y, I.box01.z, I.box01.w, I.box2ref.x, I.box2ref.y};
            T.lr.o = xf_point(inv, T.wr.o);                    // Instance.cu:26-27
            T.lr.d = xf_vector(inv, T.wr.d);
            prep<XBOX(WIDE)>(T.lr);
            if (slab<XBOX(WIDE)>(box, T.lr, TMIN, T.tmax, te)) {
                T.cur = __float_as_uint(I.box2ref.w);
                T.curT = te;
                if (RT_CHAIN_ROOT_LEAF && (T.cur & REF_LEAF)) { leaf = T.cur; chained = true; }
            } else {
                pop_next(T, spill);
            }
        } else
#endif
        {
            const InstHot &I = sc.inst_hot[T.cur_inst];
            T.lr.o = xf_point(I.inv, T.wr.o);                      // Instance.cu:26-27
            T.lr.d = xf_vector(I.inv, T.wr.d);
            prep<XBOX(WIDE)>(T.lr);
            if (slab<XBOX(WIDE)>(I.root_box, T.lr, TMIN, T.tmax, te)) { T.cur = WIDE ? I.root_ref_wide : I.root_ref; T.curT = te; }
            else pop_next(T, spill);
        }
    }
    if (leaf & REF_BLAS) {                  // the postponed BLAS leaf, or (chained) the entered BLAS's root leaf
        const uint32_t start = ref_leaf_start(leaf), count = ref_leaf_count(leaf), type = ref_leaf_type(leaf);
        if (type == RT_PRIM_TRIANGLE) {
            // every triangle record of the leaf is requested before the first test: one memory round
            // trip per leaf instead of one per triangle (tests still run in leaf order, BLAS.cu:153-176)
            for (uint32_t k0 = 0; k0 < count; k0 += TRI_AHEAD) {
                TriHot H[TRI_AHEAD];           // 3 x 12 B loads per triangle (the pad words stay unread)
                // unconditional loads (slots past the leaf's last triangle re-read that one): a load under
                // `k0 + k < count` would be issued only after the previous triangles' loads were waited for
#pragma unroll
                for (uint32_t k = 0; k < TRI_AHEAD; k++) {
                    const float *src = sc.tri_hot[start + min(k0 + k, count - 1u)].v0;
                    const float3 a = *reinterpret_cast<const float3 *>(src);
                    const float3 b = *reinterpret_cast<const float3 *>(src + 4);
                    const float3 c = *reinterpret_cast<const float3 *>(src + 8);
                    H[k].v0[0] = a.x; H[k].v0[1] = a.y; H[k].v0[2] = a.z;
                    H[k].e1[0] = b.x; H[k].e1[1] = b.y; H[k].e1[2] = b.z;
                    H[k].e2[0] = c.x; H[k].e2[1] = c.y; H[k].e2[2] = c.z;
                }
#pragma unroll
                for (uint32_t k = 0; k < TRI_AHEAD; k++) {
                    if (k0 + k >= count) break;
                    float t = 0.0f, u = 0.0f, v = 0.0f;
                    if (COUNT) cnt.tri++;
                    if (tri_test(H[k], T.lr, TMIN, T.tmax, t, u, v)) {
                        T.found = true; T.tmax = t;
                        T.hit.t = t; T.hit.inst = T.cur_inst; T.hit.ptype = type; T.hit.slot = start + k0 + k;
                        T.hit.u = u; T.hit.v = v;
                    }
                }
            }
        } else {
            for (uint32_t k = 0; k < count; k++) {
                const uint32_t slot = start + k;
                float t = 0.0f, u = 0.0f, v = 0.0f;
                bool h;
                if (type == RT_PRIM_SPHERE) {
                    if (COUNT) cnt.sq++;
                    h = sphere_test(WIDE_LDS_REC(sc.lds_sph_hot, sc.sph_hot, slot), T.lr, TMIN, T.tmax, t);
                } else {
                    if (COUNT) { cnt.sq++; cnt.quad++; }
                    h = quad_test(WIDE_LDS_REC(sc.lds_q_hot, sc.quad_hot, slot), T.lr, TMIN, T.tmax, t, u, v);
                }
                if (h) {
                    T.found = true; T.tmax = t;
                    T.hit.t = t; T.hit.inst = T.cur_inst; T.hit.ptype = type; T.hit.slot = slot; T.hit.u = u; T.hit.v = v;
                }
            }
        }
        if (chained) pop_next(T, spill);                                   // the root leaf is done
        else if (T.cur != REF_NONE && !pop_keep(T, T.curT, T.cur)) pop_next(T, spill);   // re-test the successor
    }
    if (T.cur == REF_NONE) T.tracing = false;
    return chained ? 1u : 0u;
}

#ifndef RT_DIAG
#define RT_DIAG 0
#endif
// Diagnostic builds (make diag -> librtamd_diag.so): wave-uniform cycle stamps per phase.
// claim / hit (diagnostic builds): cycles giving idle lanes their pixels (map, RNG, camera ray, traversal
// init) and sampling scatter directions after the hit records arrived
struct PhaseCycles {
    unsigned long long refill, interior, leaf, shade, iters, refill_iters, claim, hit;
    // lane occupancy (diagnostic builds): lanes stepping per interior iteration, lanes holding a TLAS / BLAS leaf per
    // leaf phase, lanes shaded per shade step (sums; the timeline divides by iters / rounds / shades)
    unsigned long long lanes_interior, lanes_leaf_tlas, lanes_leaf_blas, lanes_shade;
};
__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#if RT_DIAG
#define DIAG_WAIT_VM() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#define DIAG_T(var) const unsigned long long var = stamp()
#define DIAG_ADD(acc, t0) (acc) += stamp() - (t0)
#else
#define DIAG_WAIT_VM() (void)0
#define DIAG_T(var) (void)0
#define DIAG_ADD(acc, t0) (void)0
#endif

// One round: interior loop until every traversing lane holds a leaf, then the leaf phase.
// steps (when `track`): the lane's interior steps + leaf phases, the pixel's cost for the work order
// leaf_early (setting "leaf_early"): the interior loop also ends once no more than this many lanes are still looking
// for a leaf while some hold one; the lanes without a leaf skip the leaf phase and go on descending next round
template <bool COUNT, int WIDE = 0>
__device__ __forceinline__ void spec_round(Trav &T, const SceneGPU &sc, SEnt *spill, LaneCount &cnt,
                                           PhaseCycles &pc, uint32_t &steps, bool track, uint32_t leaf_early) {
    DIAG_T(t0);
    for (;;) {
        if (T.tracing && T.pleaf == REF_NONE && T.cur == REF_NONE) T.tracing = false;   // done, no leaf left
        const uint64_t looking = __ballot(T.tracing && T.pleaf == REF_NONE);
        if (!looking) break;
        if (leaf_early && (uint32_t)__popcll(looking) <= leaf_early && __any(T.tracing && T.pleaf != REF_NONE)) break;
        const bool active = T.tracing && T.cur != REF_NONE && (!(T.cur & REF_LEAF) || T.pleaf == REF_NONE);
        if (RT_DIAG) pc.lanes_interior += (unsigned long long)__popcll(__ballot(active));
        if (active) {
            spec_interior_step<COUNT, WIDE>(T, sc, spill, cnt);
            if (track) steps++;
        }
        if (RT_DIAG) pc.iters++;
    }
    DIAG_ADD(pc.interior, t0);
    if (RT_DIAG) {
        pc.lanes_leaf_tlas += (unsigned long long)__popcll(__ballot(T.tracing && T.pleaf != REF_NONE && !(T.pleaf & REF_BLAS)));
        pc.lanes_leaf_blas += (unsigned long long)__popcll(__ballot(T.tracing && T.pleaf != REF_NONE && (T.pleaf & REF_BLAS)));
    }
    DIAG_T(t1);
    if (T.tracing && T.pleaf != REF_NONE) {
        const uint32_t chained = spec_leaf_phase<COUNT, WIDE>(T, sc, spill, cnt);
        if (track) steps += 1u + chained;
    }
    DIAG_ADD(pc.leaf, t1);
}

template <bool COUNT, int XB = XD_CULL>
__device__ __forceinline__ bool trace(const SceneGPU &sc, const f3 &o, const f3 &d, Hit &hit, Trav &T, SEnt *spill,
                                      LaneCount &cnt) {
    trav_init<XB>(T, sc, o, d);
    while (T.tracing) trav_step<COUNT, XB>(T, sc, spill, cnt);
    hit = T.hit;
    return T.found;
}

// Record fields the shading needs (HitRecord, BasicTypes.cuh:19-31), world space.
struct Surface { f3 p, n; uint32_t material; uint32_t orig; uint32_t member; };   // member: group BLAS (option "group"): instance + 1

// Recompute the hit point / normal of the closest hit exactly as the primitive hit function and
// Instance::hit (Instance.cu:41-45) would have stored them.
// RAW: where a hit triangle's normals / material / caller index come from — 0 its TriCold record, 1 the caller's
// triangle (SceneGPU::raw_tris, GPU-built BLASes without cold records), 2 whichever the scene has (a runtime branch).
// The persistent kernel is instantiated per scene kind (0 / 1): with the branch inlined, host-built scenes' kernel
// lost 2 VGPRs to spills and ~1 % per frame (profiles/r04/cold_records/).
template <bool LDSS = false, int RAW = 2>
__device__ __forceinline__ Surface finalize(const SceneGPU &sc, const f3 &wo, const f3 &wd, const Hit &h) {
#if !RT_EXACT
    const InstCold IC = LDSS ? lds_or_global(sc.lds_icold, sc.inst_cold, h.inst) : sc.inst_cold[h.inst];
#else
    const InstCold &IC = sc.inst_cold[h.inst];
#endif
    f3 lo, ld;
#if !RT_EXACT
    if (LDSS) {
        const InstRec I = load_inst<true>(sc, h.inst);
        const float inv[12] = {I.i0.x, I.i0.y, I.i0.z, I.i0.w, I.i1.x, I.i1.y, I.i1.z, I.i1.w,
                               I.i2.x, I.i2.y, I.i2.z, I.i2.w};
        lo = xf_point(inv, wo); ld = xf_vector(inv, wd);
    } else
#endif
    {
        const InstHot &I = sc.inst_hot[h.inst];
        lo = xf_point(I.inv, wo); ld = xf_vector(I.inv, wd);
    }
    const f3 p = add(lo, scl(ld, h.t));                                        // Ray::at (Ray.cuh:18-20)
    f3 n;
    Surface s;
    if (h.ptype == RT_PRIM_TRIANGLE) {                                         // Triangle.cu:40-42
        f3 n0, n1, n2;
        if (RAW == 1 || (RAW == 2 && sc.raw_tris)) {   // GPU-built BLAS without cold records (layout.hpp SceneGPU)
            const TriHot &H = sc.tri_hot[h.slot];
            s.orig = __float_as_uint(H.pad0);
            s.member = __float_as_uint(H.pad1);
            const rt_triangle &R = sc.raw_tris[s.orig];
            if (R.has_normals) {
                n0 = mk(R.normal[0].x, R.normal[0].y, R.normal[0].z);
                n1 = mk(R.normal[1].x, R.normal[1].y, R.normal[1].z);
                n2 = mk(R.normal[2].x, R.normal[2].y, R.normal[2].z);
            } else {
                n0 = tri_face_normal(ld3(H.e1), ld3(H.e2)); n1 = n0; n2 = n0;
            }
            s.material = R.material_type == RT_MAT_ROUGH ? R.material_index
                                                         : ((sc.rough_count + R.material_index) | MAT_METAL_BIT);
        } else {
            const TriCold &T = sc.tri_cold[h.slot];
            n0 = ld3(T.n0); n1 = ld3(T.n1); n2 = ld3(T.n2);
            s.material = T.material; s.orig = T.orig_index; s.member = T.pad;
        }
        const f3 nn = unit(add(add(scl(n0, (1.0f - h.u) - h.v), scl(n1, h.u)), scl(n2, h.v)));
        n = dot(ld, nn) < 0.0f ? nn : neg(nn);
    } else if (h.ptype == RT_PRIM_SPHERE) {                                    // Sphere.cu:37-39
#if !RT_EXACT
        const SphereHot S = LDSS ? lds_or_global(sc.lds_sph_hot, sc.sph_hot, h.slot) : sc.sph_hot[h.slot];
        const PrimCold C = LDSS ? lds_or_global(sc.lds_sph_cold, sc.sph_cold, h.slot) : sc.sph_cold[h.slot];
#else
        const SphereHot &S = sc.sph_hot[h.slot];
        const PrimCold &C = sc.sph_cold[h.slot];
#endif
        const f3 outward = unit(sub(p, ld3(S.center)));
        n = dot(ld, outward) < 0.0f ? outward : neg(outward);
        s.material = C.material; s.orig = C.orig_index; s.member = 0u;
    } else {                                                                   // Parallelogram.cu:42-43
#if !RT_EXACT
        const float4 qn4 = LDSS && sc.lds_q_hot != LDS_NONE ? lds_scene[sc.lds_q_hot + h.slot * LDS_QPRIM_F4]
                                                              : reinterpret_cast<const float4 *>(sc.quad_hot + h.slot)[0];
        const PrimCold C = LDSS ? lds_or_global(sc.lds_q_cold, sc.quad_cold, h.slot) : sc.quad_cold[h.slot];
        const f3 qn = mk(qn4.x, qn4.y, qn4.z);
#else
        const QuadHot &Q = sc.quad_hot[h.slot];
        const PrimCold &C = sc.quad_cold[h.slot];
        const f3 qn = ld3(Q.n);
#endif
        n = dot(ld, qn) < 0.0f ? qn : neg(qn);
        s.material = C.material; s.orig = C.orig_index; s.member = 0u;
    }
    s.p = xf_point(IC.fwd, p);
    s.n = unit(xf_vector(IC.nrm, n));
    return s;
}

template <bool COUNT>
__device__ f3 ray_color(const SceneGPU &sc, const CameraGPU &cam, f3 o, f3 d, Rng &rng, Trav &T, SEnt *spill,
                        LaneCount &cnt, uint32_t &rays) {                      // Kernel.cu:6-103
    f3 result = mk(1.0f, 1.0f, 1.0f);
    for (uint32_t depth = 0; depth < cam.depth; depth++) {
        Hit h;
        rays++;
        if (trace<COUNT, XD_ALL>(sc, o, d, h, T, spill, cnt)) {
            if (COUNT) cnt.hits++;
            const Surface s = finalize(sc, o, d, h);
            const float4 m = reinterpret_cast<const float4 *>(sc.materials)[s.material & ~MAT_METAL_BIT];
            const f3 albedo = mk(m.x, m.y, m.z);
            f3 out;
            if (!(s.material & MAT_METAL_BIT)) {                               // Rough.cuh:14-29
                out = add(s.n, random_space_vector(rng));
                if (f_eq(dot(out, out), FZERO * FZERO)) out = s.n;
            } else {                                                           // Metal.cuh:15-32
                out = unit(sub(d, scl(s.n, 2.0f * dot(d, s.n))));
                if (m.w > 0.0f) out = add(out, scl(random_space_vector(rng), m.w));
                if (!(dot(out, s.n) > 0.0f)) return result;                    // absorbed: throughput (Kernel.cu:85-87)
            }
            o = s.p; d = out;
            result = mul(result, albedo);
        } else {
            result = mul(result, ld3(cam.background));
            break;
        }
    }
    return result;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

template <bool COUNT>
__global__ __launch_bounds__(BLOCK) void render_kernel(SceneGPU sc, CameraGPU cam, OutputGPU out,
                                                       unsigned long long *counters) {
    __shared__ unsigned long long lds_stack[LDS_DEPTH][BLOCK];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t wunit = blockIdx.x * (BLOCK / 64) + (tid >> 6);
    if (wunit >= out.units) return;                       // wave-uniform

    // 8x8 pixel unit -> pixel + output index
    uint32_t px, py, oi;
    if (out.tile_count == 0) {
        const uint32_t ux = wunit % out.units_x, uy = wunit / out.units_x;
        px = ux * 8 + (lane & 7); py = uy * 8 + (lane >> 3);
        oi = py * cam.width + px;
    } else {
        const uint32_t upr = out.tile_w / 8, upt = upr * (out.tile_h / 8);
        const uint32_t k = wunit / upt, r = wunit % upt;
        const uint32_t t = out.tile_rank + k * out.tile_count;
        const uint32_t lx = (r % upr) * 8 + (lane & 7), ly = (r / upr) * 8 + (lane >> 3);
        px = (t % out.tiles_x) * out.tile_w + lx;
        py = (t / out.tiles_x) * out.tile_h + ly;
        oi = k * out.tile_w * out.tile_h + ly * out.tile_w + lx;
    }
    const bool valid = px < cam.width && py < cam.height;

    Trav T;
    T.stk.lds = (LdsU2 *)&lds_stack[0][tid];
    alignas(16) SEnt spill[SPILL_DEPTH];
    LaneCount cnt = {0, 0, 0, 0, 0, 0, 0};
    uint32_t rays = 0;

    if (valid) {
        const uint32_t pixel = cam.pitch * py + px;                            // Kernel.cu:109
        Rng rng;
        rng.init((uint64_t)pixel ^ cam.frame_seed, pixel);                      // Kernel.cu:114
        f3 result = mk(0.0f, 0.0f, 0.0f);
        const f3 po = ld3(cam.pixel_origin), dx = ld3(cam.dx), dy = ld3(cam.dy), cc = ld3(cam.center);
        for (uint32_t si = 0; si < cam.sqrt_s; si++) {
            for (uint32_t sj = 0; sj < cam.sqrt_s; sj++) {                      // Kernel.cu:119-139
                const float ox = (((float)sj + rng.uniform()) * cam.recip_sqrt) - 0.5f;
                const float oy = (((float)si + rng.uniform()) * cam.recip_sqrt) - 0.5f;
                const f3 sp = add(add(po, scl(dx, (float)px + ox)), scl(dy, (float)py + oy));
                f3 origin = cc;
                if (cam.focus_radius > 0.0f) {
                    const f3 dv = random_plane_vector(rng, cam.focus_radius);
                    origin = add(add(cc, scl(ld3(cam.cu), dv.x)), scl(ld3(cam.cv), dv.y));
                }
                const f3 dir = unit(sub(sp, origin));
                result = add(result, ray_color<COUNT>(sc, cam, origin, dir, rng, T, spill, cnt, rays));
            }
        }
        result = scl(result, cam.recip_sqrt * cam.recip_sqrt);                  // Kernel.cu:143
        if (out.rgb) {
            out.rgb[3 * (size_t)oi + 0] = result.x;
            out.rgb[3 * (size_t)oi + 1] = result.y;
            out.rgb[3 * (size_t)oi + 2] = result.z;
        }
        // Color3::castToUchar4, gamma 2 (Color3.cuh:99-114)
        const float cr = fminf(fmaxf(sqrtf(result.x), 0.0f), 0.999f);
        const float cg = fminf(fmaxf(sqrtf(result.y), 0.0f), 0.999f);
        const float cb = fminf(fmaxf(sqrtf(result.z), 0.0f), 0.999f);
        const uint32_t packed = (uint32_t)(uint8_t)(256.0f * cr) | ((uint32_t)(uint8_t)(256.0f * cg) << 8) |
                                ((uint32_t)(uint8_t)(256.0f * cb) << 16) | (255u << 24);
        reinterpret_cast<uint32_t *>(out.rgba)[oi] = packed;
    }

    // one atomic per wave per counter
    const uint32_t wr = wave_sum(rays);
    const uint32_t wp = wave_sum(valid ? 1u : 0u);
    if (COUNT) {
        const uint32_t a = wave_sum(cnt.pairs), b = wave_sum(cnt.tri), c = wave_sum(cnt.sq), d = wave_sum(cnt.inst),
                       e = wave_sum(cnt.overflow), f = wave_sum(cnt.quad), g = wave_sum(cnt.hits);
        if (lane == 0) {
            atomicAdd(&counters[CNT_PAIRS], (unsigned long long)a);
            atomicAdd(&counters[CNT_TRI], (unsigned long long)b);
            atomicAdd(&counters[CNT_SPHQUAD], (unsigned long long)c);
            atomicAdd(&counters[CNT_INST], (unsigned long long)d);
            atomicAdd(&counters[CNT_OVERFLOW], (unsigned long long)e);
            atomicAdd(&counters[CNT_QUAD], (unsigned long long)f);
            atomicAdd(&counters[CNT_HITS], (unsigned long long)g);
        }
    }
    if (lane == 0) {
        atomicAdd(&counters[CNT_RAYS], (unsigned long long)wr);
        atomicAdd(&counters[CNT_PIXELS], (unsigned long long)wp);
    }
}

// ---- persistent-wave megakernel ------------------------------------------------------------
// One launch of (#CUs x resident blocks) workgroups.  Each lane owns one pixel at a time and runs its
// whole path (samples x bounces) as a sequence of ray segments; a segment is traversed step by
// step (trav_step).  A wave keeps stepping while most lanes are traversing; when `threshold` lanes
// have finished their segment (or are idle), the wave leaves the traversal loop and shades those
// lanes together (scatter -> next segment, or next sample, or pixel write + a new pixel from the
// work queue).  Lanes are refilled from a per-wave pool of 64 consecutive work items claimed with
// one atomic per pool (ballot-compacted lane refill).  Each pixel's RNG stream
// is consumed in exactly the reference order, so the image equals the grid kernel's bit for bit.
// XCD (XCC) of the executing wave, 0..7, and the raw HW_ID register (CU / SE / SIMD of the wave).
__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v;
}
__device__ __forceinline__ uint32_t hw_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
    return v;
}

__device__ __forceinline__ bool map_item(const OutputGPU &out, const CameraGPU &cam, uint32_t item,
                                         uint32_t &px, uint32_t &py, uint32_t &oi) {
    // multiply-shift divisions (FastDiv, host-precomputed): this runs per refilled lane and per sample
    const uint32_t wunit = item >> 6, l = item & 63u;
    if (out.tile_count == 0) {
        const uint32_t uy = out.div_units_x.div(wunit), ux = wunit - uy * out.units_x;
        px = ux * 8 + (l & 7); py = uy * 8 + (l >> 3);
        oi = py * cam.width + px;
    } else {
        const uint32_t k = out.div_upt.div(wunit), r = wunit - k * out.div_upt.d;
        const uint32_t t = out.tile_rank + k * out.tile_count;
        const uint32_t ry = out.div_upr.div(r), rx = r - ry * out.div_upr.d;
        const uint32_t lx = rx * 8 + (l & 7), ly = ry * 8 + (l >> 3);
        const uint32_t ty = out.div_tiles_x.div(t), tx = t - ty * out.tiles_x;
        px = tx * out.tile_w + lx;
        py = ty * out.tile_h + ly;
        oi = k * out.tile_w * out.tile_h + ly * out.tile_w + lx;
    }
    return px < cam.width && py < cam.height;
}

// Camera ray of sample `sample` of pixel (px, py) (Kernel.cu:119-135), consuming the pixel's RNG.
// Evaluated without FMA contraction in both builds, so FAST and EXACT start every path from the same
// camera ray.
__device__ __forceinline__ void camera_ray(const CameraGPU &cam, uint32_t px, uint32_t py, uint32_t sample, Rng &rng,
                                           f3 &o, f3 &d) {
#pragma clang fp contract(off)
    const uint32_t si = sample / cam.sqrt_s, sj = sample % cam.sqrt_s;
    const float ox = (((float)sj + rng.uniform()) * cam.recip_sqrt) - 0.5f;
    const float oy = (((float)si + rng.uniform()) * cam.recip_sqrt) - 0.5f;
    const f3 sp = add(add(ld3(cam.pixel_origin), scl(ld3(cam.dx), (float)px + ox)), scl(ld3(cam.dy), (float)py + oy));
    o = ld3(cam.center);
    if (cam.focus_radius > 0.0f) {
        const f3 dv = random_plane_vector(rng, cam.focus_radius);
        o = add(add(o, scl(ld3(cam.cu), dv.x)), scl(ld3(cam.cv), dv.y));
    }
    d = unit(sub(sp, o));
}

__device__ __forceinline__ void write_pixel(const OutputGPU &out, uint32_t oi, f3 result) {
    if (out.rgb) {
        out.rgb[3 * (size_t)oi + 0] = result.x;
        out.rgb[3 * (size_t)oi + 1] = result.y;
        out.rgb[3 * (size_t)oi + 2] = result.z;
    }
    const float cr = fminf(fmaxf(sqrtf(result.x), 0.0f), 0.999f);       // Color3::castToUchar4
    const float cg = fminf(fmaxf(sqrtf(result.y), 0.0f), 0.999f);
    const float cb = fminf(fmaxf(sqrtf(result.z), 0.0f), 0.999f);
    const uint32_t packed = (uint32_t)(uint8_t)(256.0f * cr) | ((uint32_t)(uint8_t)(256.0f * cg) << 8) |
                            ((uint32_t)(uint8_t)(256.0f * cb) << 16) | (255u << 24);
    reinterpret_cast<uint32_t *>(out.rgba)[oi] = packed;
}

// Option "reorder": a unit's cost for the next launch's claim order (schedule.hip) is the traversal
// work of its 64 pixels (interior steps + leaf phases + 1 per pixel).  A wave's lanes refill from
// the unit it claimed, so a unit's total work is the time it holds a wave; units over the particle
// cluster hold one for up to ~0.4 ms against ~20 us for a sky unit (C2, measured), and the launch
// ends with whichever wave claimed the last heavy units.
// A lane keeps one pending (unit, cost) sum and flushes it with a no-return atomic just before the
// wave's next claim atomic, whose returned value the wave waits for anyway, so the flush adds no wait of
// its own (vector memory counters retire in order: a returning atomic's wait also covers the stores and
// atomics issued before it).  A lane that finishes a pixel of another unit before that flushes its old
// sum at once.  Measured: per-shade-step atomics made each next node load wait for their memory-side
// completion (~11 % of C2 throughput, profiles/r02_ab_unit_cost.jsonl).
// a unit's recorded cost is the sum over its paths (round 3's "cost_max", 64 x its longest path, ordered C2 slower)
__device__ __forceinline__ void unit_cost_flush(uint32_t *cost, uint32_t unit, uint32_t c) { atomicAdd(cost + unit, c); }
// the pending sums of the lanes in `fin`: one atomic per distinct unit
__device__ __forceinline__ void unit_cost_add(uint32_t *cost, bool fin, uint32_t unit, uint32_t c) {
    uint64_t m = __ballot(fin);
    while (m) {
        const uint32_t first = (uint32_t)__builtin_ctzll(m);
        const uint32_t u = __shfl(unit, (int)first, 64);
        const bool mine = fin && unit == u;
        const uint32_t x = wave_sum(mine ? c : 0u);
        if ((threadIdx.x & 63u) == first) unit_cost_flush(cost, u, x);
        m &= ~(uint64_t)__ballot(mine);
    }
}

template <bool COUNT, int WIDE, int RAW>
__device__ __forceinline__ void render_persistent_body(const SceneGPU &sc, const CameraGPU &cam, const OutputGPU &out,
                                                       uint32_t *queue, uint32_t threshold, unsigned long long *counters) {
    __shared__ unsigned long long lds_stack[LDS_DEPTH][BLOCK];
    __shared__ float4 lds_mat[LDS_MATERIALS];     // the scene's materials (shading reads them per hit)
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const bool mat_lds = sc.material_count <= LDS_MATERIALS;
    if (mat_lds && tid < (int)sc.material_count) lds_mat[tid] = reinterpret_cast<const float4 *>(sc.materials)[tid];
#if !RT_EXACT
    if constexpr (WIDE) lds_scene_fill(sc);
#endif
    __syncthreads();                              // once, before any wave leaves for the queue
    const TreeRoot root = uniform_root<WIDE != 0>(sc);

    Trav T;
    T.stk.lds = (LdsU2 *)&lds_stack[0][tid];
    T.tracing = false;
    T.found = false;
    alignas(16) SEnt spill[SPILL_DEPTH];
    LaneCount cnt = {0, 0, 0, 0, 0, 0, 0};
    uint32_t rays = 0, pixels = 0;

    bool has = false;                  // lane owns a pixel
    uint32_t px_steps = 0;             // traversal steps spent on the lane's pixel (COUNT cost map, reorder)
    uint32_t item = 0, sample = 0, depth = 0;
    Rng rng;
    rng.s = 0;
    f3 acc = mk(0.0f, 0.0f, 0.0f), thr = mk(1.0f, 1.0f, 1.0f);
    uint32_t pool_next = 0, pool_end = 0;     // wave-uniform
    uint32_t limit = 0, limit_part = ~0u;     // wave-uniform: claim positions in band `limit_part`
    bool exhausted = false;                   // wave-uniform
    const uint32_t S2 = cam.sqrt_s * cam.sqrt_s;
    // Work queue: the frame's units are split into `parts` bands; a wave drains the band of its own
    // XCD first (primary rays of one band share geometry in that XCD's L2), then steals from the others.
    const uint32_t parts = out.queue_parts;
    const uint32_t xcc = xcc_id();
    uint32_t part = xcc % parts, tried = 0;
    const uint32_t grab = out.grab;                 // claim size (pixels)
    const bool track = out.unit_cost != nullptr;    // record unit costs for the next launch's order
    uint32_t pend_unit = 0, pend_cost = 0;          // the lane's unflushed unit cost (flushed before a claim)
    unsigned long long t_start = 0, t_exhaust = 0;
    uint32_t n_rounds = 0, n_shades = 0, n_grabs = 0;      // wave-uniform (timeline)
    PhaseCycles pc = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (out.timeline) t_start = __builtin_amdgcn_s_memrealtime();

    for (;;) {
        // ---- refill idle lanes from the wave's pool / the global queue
        DIAG_T(t_refill);
        uint64_t need = __ballot(!has);
        while (need && !exhausted) {
            if (RT_DIAG) pc.refill_iters++;
            const uint32_t n_need = __popcll(need);
            if (pool_next >= pool_end) {
                // bands: whole unit rows in frame mode (so a band can be walked in supertiles)
                const uint32_t rows = out.tile_count == 0 ? out.units / out.units_x : out.units;
                const uint32_t upr = out.tile_count == 0 ? out.units_x : 1u;
                const uint32_t p_begin = (rows * part / parts) * upr * 64u;
                const uint32_t p_end = (rows * (part + 1) / parts) * upr * 64u;
                // ordered walk (schedule.hip): one item per claim, a whole unit or a 1/2, 1/4 of a heavy
                // one; the band's item count sits next to its head.  Screen walk: `grab` pixels per claim.
                const uint32_t step = out.order ? 1u : grab;
                if (part != limit_part) {          // the band's item count: read once per band, off the head's line
                    limit_part = part;
                    limit = out.order ? __builtin_amdgcn_readfirstlane(queue[(QUEUE_MAX_PARTS + part) * QUEUE_STRIDE])
                                      : p_end - p_begin;
                }
                if (track) {                         // completes under the claim's wait
                    unit_cost_add(out.unit_cost, pend_cost != 0, pend_unit, pend_cost);
                    pend_cost = 0;
                }
                uint32_t b = 0;
                if (lane == 0) b = atomicAdd(queue + part * QUEUE_STRIDE, step);
                b = __builtin_amdgcn_readfirstlane(__shfl(b, 0, 64));
                n_grabs++;
                if (b >= limit) {
                    // the band is dry: try the next one.  `tried` counts failures over the wave's life, so a
                    // wave retires after `parts` failed claims even if a band it left still has items: it frees
                    // its slot for the next lane's launch (a scan of every band's head instead, stealing until
                    // the last item, measured 45 % slower on C2: profiles/r02_ab_exit_scan.jsonl)
                    if (++tried >= parts) {
                        exhausted = true;
                        if (out.timeline) t_exhaust = __builtin_amdgcn_s_memrealtime();
                        break;
                    }
                    part = part + 1 == parts ? 0 : part + 1;
                    continue;
                }
                if (out.order) {
                    const uint32_t it = out.order[4u * (p_begin >> 6) + b];
                    // log2 pieces 3: two adjacent light units (schedule setting "merge"), 128 pixels
                    const uint32_t ls = it & 3u, len = ls == 3u ? 128u : 64u >> ls;
                    pool_next = (it >> 4) * 64u + (ls == 3u ? 0u : ((it >> 2) & 3u) * len);
                    pool_end = pool_next + len;
                } else {
                    b += p_begin;
                    pool_next = b;
                    pool_end = min(b + grab, p_end);
                }
                if (!out.order && out.supertile && out.tile_count == 0 && grab == 64u) {
                    // walk the band in st x st-unit supertiles (row-major supertiles, row-major units
                    // inside): the units in flight form a compact screen region, not a full-width strip
                    const uint32_t W = out.units_x, st = out.supertile;
                    const uint32_t r0 = p_begin / (64u * W), Hb = (p_end - p_begin) / (64u * W);
                    const uint32_t j = (b - p_begin) >> 6;
                    const uint32_t sr = j / (W * st);
                    const uint32_t h = min(st, Hb - sr * st);
                    const uint32_t k = j - sr * W * st;
                    const uint32_t sc = k / (st * h);
                    const uint32_t w = min(st, W - sc * st);
                    const uint32_t m = k - sc * st * h;
                    const uint32_t u = (r0 + sr * st + m / w) * W + sc * st + m % w;
                    pool_next = u * 64u;
                    pool_end = pool_next + 64u;
                }
            }
            const uint32_t take = min(n_need, pool_end - pool_next);
            const uint32_t rank = __popcll(need & ((1ull << lane) - 1ull));
            DIAG_T(t_lanes);
            if (!has && rank < take) {
                uint32_t px, py, oi;
                item = pool_next + rank;
                if (map_item(out, cam, item, px, py, oi)) {
                    has = true;
                    const uint32_t pixel = cam.pitch * py + px;                    // Kernel.cu:109
                    rng.init((uint64_t)pixel ^ cam.frame_seed, pixel);              // Kernel.cu:114
                    acc = mk(0.0f, 0.0f, 0.0f);
                    thr = mk(1.0f, 1.0f, 1.0f);
                    sample = 0; depth = 0;
                    px_steps = 0;
                    f3 o, d;
                    camera_ray(cam, px, py, 0, rng, o, d);
                    trav_init<XBOX(WIDE)>(T, root, o, d);
                    pixels++;
                }
            }
            DIAG_ADD(pc.claim, t_lanes);
            pool_next += take;
            need = __ballot(!has);          // lanes handed an out-of-frame item (edge units) retry
        }
        DIAG_ADD(pc.refill, t_refill);
        if (!__any(has)) {
            if (exhausted) break;
            continue;
        }
        // ---- traverse while enough lanes are busy
        for (;;) {
            const uint64_t tr = __ballot(T.tracing);
            if (tr == 0) break;
            const uint64_t want = __ballot(!T.tracing && (has || !exhausted));
            if ((uint32_t)__popcll(want) >= threshold) break;
            spec_round<COUNT, WIDE>(T, sc, spill, cnt, pc, px_steps, COUNT || track, out.leaf_early);
            n_rounds++;
        }
        // ---- shade lanes whose segment finished (rayColor body, Kernel.cu:64-100)
        n_shades++;
        DIAG_T(t_shade);
        bool fin = false;                    // lane wrote its pixel in this step
        if (RT_DIAG) pc.lanes_shade += (unsigned long long)__popcll(__ballot(has && !T.tracing));
        if (has && !T.tracing) {
            rays++;
            bool path_done;
            f3 no = T.wr.o, nd = T.wr.d;                                     // next segment
            if (T.found) {
                if (COUNT) cnt.hits++;
                const Surface s = finalize<WIDE != 0, RAW>(sc, T.wr.o, T.wr.d, T.hit);
                DIAG_WAIT_VM();
                DIAG_T(t_hit);
                const uint32_t mi = s.material & ~MAT_METAL_BIT;
                const float4 m = mat_lds ? lds_mat[mi] : reinterpret_cast<const float4 *>(sc.materials)[mi];
                bool absorbed = false;
                if (!(s.material & MAT_METAL_BIT)) {                         // Rough.cuh:14-29
                    // the path's last segment (depth and samples exhausted): the scattered direction and
                    // the pixel's RNG are never used again, so the draws are skipped (same image)
                    if (depth + 1 < cam.depth || sample + 1 < S2) {
                        nd = add(s.n, random_space_vector(rng));
                        if (f_eq(dot(nd, nd), FZERO * FZERO)) nd = s.n;
                    }
                } else {                                                     // Metal.cuh:15-32
                    nd = unit(sub(T.wr.d, scl(s.n, 2.0f * dot(T.wr.d, s.n))));
                    if (m.w > 0.0f) nd = add(nd, scl(random_space_vector(rng), m.w));
                    absorbed = !(dot(nd, s.n) > 0.0f);
                }
                DIAG_ADD(pc.hit, t_hit);
                if (absorbed) {
                    path_done = true;                                        // throughput (Kernel.cu:85-87)
                } else {
                    thr = mul(thr, mk(m.x, m.y, m.z));
                    no = s.p;
                    depth++;
                    path_done = depth >= cam.depth;                          // throughput on exhaustion
                }
            } else {
                thr = mul(thr, ld3(cam.background));
                path_done = true;
            }
            if (path_done) {
                acc = add(acc, thr);                                         // Kernel.cu:138
                sample++;
                uint32_t px, py, oi;
                map_item(out, cam, item, px, py, oi);
                if (sample < S2) {
                    thr = mk(1.0f, 1.0f, 1.0f);
                    depth = 0;
                    camera_ray(cam, px, py, sample, rng, no, nd);
                } else {
                    write_pixel(out, oi, scl(acc, cam.recip_sqrt * cam.recip_sqrt));   // Kernel.cu:143-146
                    if (COUNT && out.costmap) out.costmap[oi] = px_steps;
                    has = false;
                    fin = true;
                }
            }
            if (has) trav_init<XBOX(WIDE)>(T, root, no, nd);
        }
        if (track && fin) {
            const uint32_t u = item >> 6;
            if (u != pend_unit) {
                if (pend_cost) unit_cost_flush(out.unit_cost, pend_unit, pend_cost);
                pend_unit = u;
                pend_cost = 0;
            }
            pend_cost = pend_cost + px_steps + 1u;
        }
        DIAG_ADD(pc.shade, t_shade);
    }

    if (track && pend_cost) unit_cost_flush(out.unit_cost, pend_unit, pend_cost);
    const uint32_t wr = wave_sum(rays);
    const uint32_t wp = wave_sum(pixels);
    if (COUNT) {
        const uint32_t a = wave_sum(cnt.pairs), b = wave_sum(cnt.tri), c = wave_sum(cnt.sq), d = wave_sum(cnt.inst),
                       e = wave_sum(cnt.overflow), f = wave_sum(cnt.quad), g = wave_sum(cnt.hits);
        if (lane == 0) {
            atomicAdd(&counters[CNT_PAIRS], (unsigned long long)a);
            atomicAdd(&counters[CNT_TRI], (unsigned long long)b);
            atomicAdd(&counters[CNT_SPHQUAD], (unsigned long long)c);
            atomicAdd(&counters[CNT_INST], (unsigned long long)d);
            atomicAdd(&counters[CNT_OVERFLOW], (unsigned long long)e);
            atomicAdd(&counters[CNT_QUAD], (unsigned long long)f);
            atomicAdd(&counters[CNT_HITS], (unsigned long long)g);
        }
    }
    if (lane == 0) {
        atomicAdd(&counters[CNT_RAYS], (unsigned long long)wr);
        atomicAdd(&counters[CNT_PIXELS], (unsigned long long)wp);
        if (out.timeline) {
            // the wave's index from its stack window address (threadIdx.x kept live to here was spilled)
            const uint32_t wv = (uint32_t)((const unsigned long long *)T.stk.lds - &lds_stack[0][0]) >> 6;
            unsigned long long *w = out.timeline + (unsigned long long)TIMELINE_WORDS * (blockIdx.x * (BLOCK / 64) + wv);
            w[0] = t_start;
            w[1] = __builtin_amdgcn_s_memrealtime();
            w[2] = ((unsigned long long)hw_id() << 32) | xcc;
            w[3] = wp;
            w[4] = t_exhaust;
            w[5] = n_rounds;
            w[6] = n_shades;
            w[7] = n_grabs;
            w[8] = pc.refill;
            w[9] = pc.interior;
            w[10] = pc.leaf;
            w[11] = pc.shade;
            w[12] = pc.iters;
            w[13] = pc.refill_iters;
            w[14] = pc.claim;
            w[15] = pc.hit;
            w[16] = pc.lanes_interior;
            w[17] = pc.lanes_leaf_tlas;
            w[18] = pc.lanes_leaf_blas;
            w[19] = pc.lanes_shade;
        }
    }
}

// Register budget variants: WPE = minimum waves per SIMD the compiler must allow (0 = its choice).
template <bool COUNT, int WPE, int WIDE = 0, int RAW = 2>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE > 0 ? WPE : 1)))
void render_persistent_kernel(SceneGPU sc, CameraGPU cam, OutputGPU out, uint32_t *queue, uint32_t threshold,
                              unsigned long long *counters) {
    render_persistent_body<COUNT, WIDE, RAW>(sc, cam, out, queue, threshold, counters);
}

__global__ __launch_bounds__(BLOCK) void trace_rays_kernel(SceneGPU sc, const float *rays, uint32_t n, rt_hit *hits) {
    __shared__ unsigned long long lds_stack[LDS_DEPTH][BLOCK];
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    Trav T;
    T.stk.lds = (LdsU2 *)&lds_stack[0][threadIdx.x];
    alignas(16) SEnt spill[SPILL_DEPTH];
    LaneCount cnt = {0, 0, 0, 0, 0, 0, 0};
    const f3 o = mk(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
    const f3 d = mk(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
    Hit h;
    rt_hit r;
    if (trace<false, XD_ALL>(sc, o, d, h, T, spill, cnt)) {
        const Surface s = finalize(sc, o, d, h);
        r.t = h.t; r.instance = s.member ? s.member - 1u : (sc.inst_by_slot ? sc.tlas_slots[h.inst] : h.inst);
        r.primitive_type = h.ptype; r.primitive_index = s.orig;
        r.point.x = s.p.x; r.point.y = s.p.y; r.point.z = s.p.z;
        r.normal.x = s.n.x; r.normal.y = s.n.y; r.normal.z = s.n.z;
        const bool metal = (s.material & MAT_METAL_BIT) != 0;
        r.material_type = metal ? RT_MAT_METAL : RT_MAT_ROUGH;
        r.material_index = (s.material & ~MAT_METAL_BIT) - (metal ? sc.rough_count : 0u);
    } else {
        r.t = __builtin_huge_valf(); r.instance = 0xFFFFFFFFu; r.primitive_type = 0; r.primitive_index = 0;
        r.point.x = r.point.y = r.point.z = 0.0f; r.normal.x = r.normal.y = r.normal.z = 0.0f;
        r.material_type = 0; r.material_index = 0;
    }
    hits[i] = r;
}


// rt_box_test (parity tests, not a render path): the box decisions the kernels take, on caller boxes and rays, one
// thread per (box, ray, tmax) with tmin = 0.001.  Mode 0 (EXACT build): BoundingBox::hit (BoundingBox.cu:34-72).  FAST
// build: 1 the single-box conservative cull (slab<XD_CULL>: instance and root boxes of modes 1 / 2), 2 the same with
// marginal decisions re-taken exactly (slab<XD_ALL>: binary pairs, instance and root boxes of mode 3), 3 a quad slot in
// pair order with exact decisions (quad_decide<true, XD_ALL>: mode 3), 4 a quad slot's conservative cull
// (quad_decide<false, XD_CULL>: modes 1 / 2).  Modes 3 / 4 put the box in slot 0 of a quad whose slot 1 is
// its empty partner (a leaf child's) and whose slots 2 / 3 hold a box behind the ray's origin.
__global__ __launch_bounds__(BLOCK) void box_test_kernel(const float *boxes, const float *rays, const float *tmaxs, uint32_t n,
                                                         uint32_t mode, uint8_t *hit, float *te) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    float b[6];
    for (int c = 0; c < 6; c++) b[c] = boxes[6 * (size_t)i + c];
    RayP r;
    r.o = mk(rays[6 * (size_t)i], rays[6 * (size_t)i + 1], rays[6 * (size_t)i + 2]);
    r.d = mk(rays[6 * (size_t)i + 3], rays[6 * (size_t)i + 4], rays[6 * (size_t)i + 5]);
    const float tmax = tmaxs[i];
    float e = 0.0f;
    bool h = false;
#if RT_EXACT
    (void)mode;
    h = slab_ref(b, r.o, r.d, TMIN, tmax, e);
#else
    if (mode == 1 || mode == 2) {
        if (mode == 2) { prep<XD_ALL>(r); h = slab<XD_ALL>(b, r, TMIN, tmax, e); }
        else { prep<XD_CULL>(r); h = slab<XD_CULL>(b, r, TMIN, tmax, e); }
    } else {
        float4 Q[8];
        float bb[6];       // behind the origin: around o - d, half-width |d_a| / 2 per axis (exit t = -0.5 on every axis)
        const float p3[3] = {r.o.x - r.d.x, r.o.y - r.d.y, r.o.z - r.d.z}, d3[3] = {r.d.x, r.d.y, r.d.z};
        for (int a = 0; a < 3; a++) {
            const float w = 0.5f * fabsf(d3[a]);
            bb[2 * a] = p3[a] - w; bb[2 * a + 1] = p3[a] + w;
        }
        for (int c = 0; c < 6; c++) {
            float *q = reinterpret_cast<float *>(&Q[c]);
            q[0] = b[c]; q[1] = b[c]; q[2] = bb[c]; q[3] = bb[c];
        }
        uint4 R = make_uint4(0u, REF_EMPTY, 0u, REF_EMPTY);
        reinterpret_cast<uint4 *>(Q)[6] = R;
        Q[7] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        float t[4], pa, pb;
        bool hq[4];
        if (mode == 3) {
            prep<XD_ALL>(r);
            quad_decide<true, XD_ALL>(Q, Q[0], Q[1], Q[2], Q[3], Q[4], Q[5], R, r, tmax, t, hq, pa, pb);
        } else {
            prep<XD_CULL>(r);
            quad_decide<false, XD_CULL>(Q, Q[0], Q[1], Q[2], Q[3], Q[4], Q[5], R, r, tmax, t, hq, pa, pb);
        }
        h = hq[0];
        e = t[0];
    }
#endif
    hit[i] = h ? 1 : 0;
    te[i] = h ? e : __builtin_huge_valf();
}
}  // namespace dev

hipError_t RT_SUFFIX(launch_render)(const SceneGPU &sc, const CameraGPU &cam, const OutputGPU &out, bool count,
                                    unsigned long long *counters, hipStream_t stream) {
    using namespace RT_SUFFIX(dev);
    const uint32_t waves_per_block = BLOCK / 64;
    const dim3 grid((out.units + waves_per_block - 1) / waves_per_block);
    if (grid.x == 0) return hipSuccess;
    if (count) hipLaunchKernelGGL(render_kernel<true>, grid, dim3(BLOCK), 0, stream, sc, cam, out, counters);
    else hipLaunchKernelGGL(render_kernel<false>, grid, dim3(BLOCK), 0, stream, sc, cam, out, counters);
    return hipGetLastError();
}

namespace {
template <int WPE, int WIDE = 0, int RAW = 2>
hipError_t launch_persistent_wpe(const SceneGPU &sc, const CameraGPU &cam, const OutputGPU &out, bool count,
                                 unsigned long long *counters, uint32_t *queue, uint32_t blocks_per_cu_cus,
                                 uint32_t threshold, hipStream_t stream) {
    using namespace RT_SUFFIX(dev);
    const uint32_t need = (out.units + (BLOCK / 64) - 1) / (BLOCK / 64);
    const dim3 grid(blocks_per_cu_cus < need ? blocks_per_cu_cus : need);
    if (count)
        hipLaunchKernelGGL((render_persistent_kernel<true, WPE, WIDE, RAW>), grid, dim3(BLOCK), 0, stream, sc, cam, out, queue, threshold, counters);
    else
        hipLaunchKernelGGL((render_persistent_kernel<false, WPE, WIDE, RAW>), grid, dim3(BLOCK), 0, stream, sc, cam, out, queue, threshold, counters);
    return hipGetLastError();
}
template <int WPE, int WIDE = 0, int RAW = 2>
uint32_t blocks_per_cu_wpe() {
    using namespace RT_SUFFIX(dev);
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, render_persistent_kernel<false, WPE, WIDE, RAW>, BLOCK, 0) != hipSuccess) return 1;
    return n > 0 ? (uint32_t)n : 1u;
}
#if RT_EXACT
constexpr int HAS_WIDE = 0;           // EXACT keeps the reference's binary trees and visit order
#else
constexpr int HAS_WIDE = 1;
#endif
}  // namespace

// One instance per scene kind: traversal mode W (SceneGPU::wide, XBOX) and where a hit triangle's shading data lives
// (finalize's RAW: GPU-built trees without cold records).  Quad trees hold 3 waves per SIMD (WPE 3); binary pairs take
// the compiler's budget (WPE 0).  (Round 5's option "variant" 4 — at least 4 waves per SIMD — was 12 % slower: removed.)
#define RT_DISPATCH_INSTANCE(wide, raw, CALL)                                                  \
    do {                                                                                       \
        if ((wide) && HAS_WIDE) {                                                              \
            if ((raw) && (wide) == 3) return CALL(3, 3 * HAS_WIDE, 1);                         \
            if (raw) return CALL(3, 2 * HAS_WIDE, 1);                                          \
            if ((wide) == 3) return CALL(3, 3 * HAS_WIDE, 0);                                  \
            if ((wide) == 2) return CALL(3, 2 * HAS_WIDE, 0);                                  \
            return CALL(3, HAS_WIDE, 0);                                                       \
        }                                                                                      \
        return CALL(0, 0, 2);                                                                  \
    } while (0)

hipError_t RT_SUFFIX(launch_render_persistent)(const SceneGPU &sc, const CameraGPU &cam, const OutputGPU &out, bool count,
                                               unsigned long long *counters, uint32_t *queue, uint32_t blocks,
                                               uint32_t threshold, bool reset_queue, hipStream_t stream) {
    if (out.units == 0) return hipSuccess;
    if (reset_queue) {       // else the schedule kernel (schedule.hip) just reset the heads
        const hipError_t e = hipMemsetAsync(queue, 0, QUEUE_MAX_PARTS * QUEUE_STRIDE * sizeof(uint32_t), stream);
        if (e != hipSuccess) return e;
    }
#define RT_LAUNCH(WPE, W, RAW) launch_persistent_wpe<WPE, W, RAW>(sc, cam, out, count, counters, queue, blocks, threshold, stream)
    RT_DISPATCH_INSTANCE(sc.wide, sc.raw_tris != nullptr, RT_LAUNCH);
#undef RT_LAUNCH
}

// the occupancy of the instance launch_render_persistent runs for (wide, raw): the persistent grid is sized from it
uint32_t RT_SUFFIX(persistent_blocks_per_cu)(uint32_t wide, bool raw) {
#define RT_OCC(WPE, W, RAW) blocks_per_cu_wpe<WPE, W, RAW>()
    RT_DISPATCH_INSTANCE(wide, raw, RT_OCC);
#undef RT_OCC
}
hipError_t RT_SUFFIX(launch_trace_rays)(const SceneGPU &sc, const float *rays, uint32_t n, rt_hit *hits,
                                        hipStream_t stream) {
    using namespace RT_SUFFIX(dev);
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(trace_rays_kernel, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, stream, sc, rays, n, hits);
    return hipGetLastError();
}

hipError_t RT_SUFFIX(launch_box_test)(const float *boxes, const float *rays, const float *tmax, uint32_t n, uint32_t mode,
                                      uint8_t *hit, float *te, hipStream_t stream) {
    using namespace RT_SUFFIX(dev);
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(box_test_kernel, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, stream, boxes, rays, tmax, n, mode, hit, te);
    return hipGetLastError();
}

}  // namespace rtamd
