// lbvh.hip — GPU BVH builder (RT_BUILD_LBVH): BLAS forests over primitives and the per-frame TLAS
// over instances, built on the device (interface and pipeline in lbvh.hpp).
//
// Karras, "Maximizing Parallelism in the Construction of BVHs, Octrees, and k-d Trees" (HPG 2012):
// with items sorted by Morton code, interior node i of an n-leaf radix tree covers a key range with
// one end at i; its direction, far end and split follow from the longest-common-prefix function
// δ(i, j) alone, so every interior node is built by one thread with no dependencies.  Here δ is
// evaluated per segment (indices outside the segment give -1), so one launch builds a whole forest
// (9,766 particle BLASes of config C5, or one TLAS).  Equal Morton codes are ordered by sorted
// position (the sort is stable, so by item index), making builds deterministic.
//
// Compiled with -ffp-contract=off: primitive boxes, centroids and the leaf-ordered hot / cold
// records are computed with the reference's float evaluation order (host_math.hpp restates the
// same functions on the host), so a GPU-built leaf holds the same bytes a host build would.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "lbvh.hpp"

namespace rtamd {
namespace lbvh {

constexpr int BLOCK = 256;
constexpr uint32_t LEAF_BIT = 1u << 31;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr float FZERO = 1e-6f;                      // Global.cuh:147

inline uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + BLOCK - 1) / BLOCK); }

// ---- reference box / primitive arithmetic (host_math.hpp, device side) --------------------
struct V3 { float x, y, z; };
__device__ __forceinline__ V3 v3(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ V3 of(const rt_vec3 &a) { return v3(a.x, a.y, a.z); }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float comp(const V3 &a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) {        // Vec3.cuh:113-119
    float s = 0.0f; s += a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s;
}
__device__ __forceinline__ V3 cross(V3 a, V3 b) {         // Vec3.cuh:120-126
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ V3 unit(V3 a) {                // Vec3.cuh:129-137
    const float f = 1.0f / sqrtf(dot(a, a));
    return v3(a.x * f, a.y * f, a.z * f);
}

struct Box { float b[6]; };                                // {xmin,xmax,ymin,ymax,zmin,zmax}
__device__ __forceinline__ float rlength(float mn, float mx) {   // Range.cuh: length()
    return (mn >= mx || fabsf(mn - mx) < FZERO) ? 0.0f : mx - mn;
}
__device__ __forceinline__ Box from_points(V3 p1, V3 p2) {     // BoundingBox.cuh:24-28, 41-47
    Box r;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const float a = comp(p1, i), c = comp(p2, i);
        float mn = a < c ? a : c, mx = a < c ? c : a;
        if (rlength(mn, mx) < FZERO) { mn -= FZERO; mx += FZERO; }
        r.b[2 * i] = mn; r.b[2 * i + 1] = mx;
    }
    return r;
}
__device__ __forceinline__ void merge_into(float *m, const float *a) {   // BoundingBox.cuh:50-55
#pragma unroll
    for (int i = 0; i < 3; i++) {
        m[2 * i] = a[2 * i] < m[2 * i] ? a[2 * i] : m[2 * i];
        m[2 * i + 1] = a[2 * i + 1] > m[2 * i + 1] ? a[2 * i + 1] : m[2 * i + 1];
    }
}

__device__ __forceinline__ void tri_box_centroid(const float *t, Box &bx, V3 &c) {   // Triangle.cu:46-62, .cuh:53-61
    V3 mn, mx;
    float lo[3], hi[3], cc[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const float a = t[i], b = t[3 + i], d = t[6 + i];              // vertices 0, 1, 2 (9 floats)
        float l = a, h = a;
        if (b < l) l = b;
        if (d < l) l = d;
        if (h < b) h = b;
        if (h < d) h = d;
        lo[i] = l; hi[i] = h;
        float s = a + b + d;
        s /= 3.0f;
        cc[i] = s;
    }
    mn = v3(lo[0], lo[1], lo[2]); mx = v3(hi[0], hi[1], hi[2]);
    bx = from_points(mn, mx);
    c = v3(cc[0], cc[1], cc[2]);
}
__device__ __forceinline__ void sphere_box_centroid(const rt_sphere &s, Box &bx, V3 &c) {   // Sphere.cu:51-55
    const V3 ce = of(s.center), e = v3(s.radius, s.radius, s.radius);
    bx = from_points(ce - e, ce + e);
    c = ce;
}
__device__ __forceinline__ void quad_box_centroid(const rt_parallelogram &p, Box &bx, V3 &c) {   // Parallelogram.cu:48-50 (q-centred), .cuh:45-47
    const V3 h = (of(p.u) + of(p.v)) * 0.5f;
    bx = from_points(of(p.q) + h, of(p.q) - h);
    c = of(p.q) + of(p.u) * 0.5f + of(p.v) * 0.5f;
}

// a triangle's hot record as gather_item writes it without cold records (caller index and member in the pads)
__device__ __forceinline__ TriHot tri_hot_record(const float *tv, uint32_t prim, uint32_t member) {
    const V3 v0 = v3(tv[0], tv[1], tv[2]);
    const V3 e1 = v3(tv[3], tv[4], tv[5]) - v0, e2 = v3(tv[6], tv[7], tv[8]) - v0;
    TriHot H;
    H.v0[0] = v0.x; H.v0[1] = v0.y; H.v0[2] = v0.z; H.pad0 = __uint_as_float(prim);
    H.e1[0] = e1.x; H.e1[1] = e1.y; H.e1[2] = e1.z; H.pad1 = __uint_as_float(member);
    H.e2[0] = e2.x; H.e2[1] = e2.y; H.e2[2] = e2.z; H.pad2 = 0.0f;
    return H;
}

// ---- Morton / ordered-float helpers --------------------------------------------------------
__device__ __forceinline__ uint32_t f2o(float f) {          // order-preserving float -> uint
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}
__device__ __forceinline__ uint32_t expand10(uint32_t v) {  // 10 bits -> every third bit of 30
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
__device__ __forceinline__ uint32_t quant10(float c, float lo, float hi) {
    const float ext = hi - lo;
    if (!(ext > 0.0f)) return 0u;
    const float q = (c - lo) / ext * 1024.0f;
    if (!(q > 0.0f)) return 0u;
    return q >= 1023.0f ? 1023u : (uint32_t)q;
}


// ---- kernels -------------------------------------------------------------------------------
__global__ void init_bounds_kernel(uint32_t *bounds, uint32_t n_segs) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n_segs * 6) return;
    bounds[i] = (i & 1) ? 0u : 0xFFFFFFFFu;               // even: min slots, odd: max slots
}

// stage (optional, BLAS builds without cold records): each triangle item's TriHot record in item order, so the
// gather after the sort reads one 48-B record per leaf slot instead of the vertices plus the member table
__global__ void prep_blas_kernel(const LbvhSeg *segs, const uint32_t *seg_of, uint32_t n, RawPrimsGPU raw,
                                 float *box, float4 *cent, TriHot *stage, const uint32_t *item_member) {
    const uint32_t it = blockIdx.x * BLOCK + threadIdx.x;
    if (it >= n) return;
    const LbvhSeg S = segs[seg_of[it]];
    const uint32_t prim = S.prim_base + (it - S.item_base);
    Box bx;
    V3 c;
    if (S.ptype == RT_PRIM_TRIANGLE) {
        const float *tv = raw.tri_verts + 9 * (size_t)prim;
        tri_box_centroid(tv, bx, c);
        if (stage) stage[it] = tri_hot_record(tv, prim, S.member_count ? item_member[it] : 0u);
    } else if (S.ptype == RT_PRIM_SPHERE) sphere_box_centroid(raw.spheres[prim], bx, c);
    else quad_box_centroid(raw.quads[prim], bx, c);
#pragma unroll
    for (int k = 0; k < 6; k++) box[6 * (size_t)it + k] = bx.b[k];
    cent[it] = make_float4(c.x, c.y, c.z, 0.0f);
}

// Centroid bounds per segment.  Each block walks `ipt` consecutive block-wide strides of items; a wave
// whose 64 items share one segment accumulates per lane across strides and reduces only when the segment
// changes (or at the end), into the block's LDS slot when the segment is the one the block starts in, else
// with global atomics; mixed waves (segment boundaries) fall back to per-lane atomics.  One global atomic
// set per block for the common case: one segment of 10M triangles (C5's group) took 10.6 ms with a set per
// wave, all on the same six words.  Inactive TLAS items (centroid w != 0, set_items) are left out.
__device__ __forceinline__ void bounds_flush(uint32_t seg, float (&lo)[3], float (&hi)[3], uint32_t bseg, uint32_t *sb,
                                             uint32_t *bounds) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
        for (int a = 0; a < 3; a++) {
            lo[a] = fminf(lo[a], __shfl_xor(lo[a], off));
            hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off));
        }
    }
    if ((threadIdx.x & 63) == 0 && lo[0] <= hi[0]) {      // at least one live item
        uint32_t *dst = seg == bseg ? sb : bounds + 6 * seg;
#pragma unroll
        for (int a = 0; a < 3; a++) {
            atomicMin(&dst[2 * a], f2o(lo[a]));
            atomicMax(&dst[2 * a + 1], f2o(hi[a]));
        }
    }
}

__global__ __launch_bounds__(BLOCK) void bounds_kernel(const uint32_t *seg_of, const float4 *cent, uint32_t n, uint32_t ipt,
                                                       uint32_t *bounds) {
    __shared__ uint32_t sb[6];
    const uint64_t base = (uint64_t)blockIdx.x * BLOCK * ipt;
    const uint32_t bseg = base < n ? seg_of[base] : NONE;
    if (threadIdx.x < 6) sb[threadIdx.x] = (threadIdx.x & 1) ? 0u : 0xFFFFFFFFu;
    __syncthreads();
    const float inf = __builtin_huge_valf();
    uint32_t acc = NONE;                                   // wave-uniform: the segment lo/hi accumulate
    float lo[3] = {inf, inf, inf}, hi[3] = {-inf, -inf, -inf};
    for (uint32_t j = 0; j < ipt; j++) {
        const uint64_t it = base + (uint64_t)j * BLOCK + threadIdx.x;
        const bool valid = it < n;
        const uint32_t seg = valid ? seg_of[it] : NONE;
        const float4 c = valid ? cent[it] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const bool live = valid && c.w == 0.0f;
        const uint32_t seg0 = __builtin_amdgcn_readfirstlane(seg);
        if (__all(seg == seg0)) {
            if (seg0 == NONE) break;                       // past the end (uniform across the wave)
            if (seg0 != acc) {
                if (acc != NONE) bounds_flush(acc, lo, hi, bseg, sb, bounds);
                acc = seg0;
#pragma unroll
                for (int a = 0; a < 3; a++) { lo[a] = inf; hi[a] = -inf; }
            }
            if (live) {
                lo[0] = fminf(lo[0], c.x); hi[0] = fmaxf(hi[0], c.x);
                lo[1] = fminf(lo[1], c.y); hi[1] = fmaxf(hi[1], c.y);
                lo[2] = fminf(lo[2], c.z); hi[2] = fmaxf(hi[2], c.z);
            }
        } else if (live) {
            const float v[3] = {c.x, c.y, c.z};
#pragma unroll
            for (int a = 0; a < 3; a++) {
                atomicMin(&bounds[6 * seg + 2 * a], f2o(v[a]));
                atomicMax(&bounds[6 * seg + 2 * a + 1], f2o(v[a]));
            }
        }
    }
    if (acc != NONE) bounds_flush(acc, lo, hi, bseg, sb, bounds);
    __syncthreads();
    if (threadIdx.x < 6 && bseg != NONE && sb[0] != 0xFFFFFFFFu) {
        if (threadIdx.x & 1) atomicMax(&bounds[6 * bseg + threadIdx.x], sb[threadIdx.x]);
        else atomicMin(&bounds[6 * bseg + threadIdx.x], sb[threadIdx.x]);
    }
}

// 30-bit Morton codes over each segment's centroid bounds.  (Round 3's 2-bit size class above the code for the TLAS,
// option "tlas_classes", measured neutral and was removed in round 6.)
__global__ void morton_kernel(const uint32_t *seg_of, const float4 *cent, uint32_t n, const uint32_t *bounds,
                              uint32_t *keys, uint32_t *vals) {
    const uint32_t it = blockIdx.x * BLOCK + threadIdx.x;
    if (it >= n) return;
    const uint32_t seg = seg_of[it];
    const float4 c = cent[it];
    if (c.w != 0.0f) {                           // inactive item: behind every active one (no class bits reach ~0)
        keys[it] = 0xFFFFFFFFu;
        vals[it] = it;
        return;
    }
    const uint32_t *B = bounds + 6 * seg;
    const uint32_t x = quant10(c.x, o2f(B[0]), o2f(B[1]));
    const uint32_t y = quant10(c.y, o2f(B[2]), o2f(B[3]));
    const uint32_t z = quant10(c.z, o2f(B[4]), o2f(B[5]));
    keys[it] = (expand10(x) << 2) | (expand10(y) << 1) | expand10(z);
    vals[it] = it;
}

// Sorting happens per segment (items never leave their segment's range): trees of <= LOCAL_SORT_MAX items are
// sorted by one workgroup in LDS (bitonic over (code, item) pairs, which is the stable radix order), larger ones by
// one rocPRIM radix sort each over their 30- or 32-bit codes (LbvhBuilder::build).  A 64-bit (segment, code) key
// over the whole forest cost C5 five 8-bit passes over 10 M 12-byte pairs per rebuild.
constexpr uint32_t LOCAL_SORT_MAX = 2048;
__global__ __launch_bounds__(BLOCK) void local_sort_kernel(const LbvhSeg *segs, const uint32_t *keys_in, uint32_t *keys_out,
                                                           uint32_t *vals_out) {
    __shared__ unsigned long long sk[LOCAL_SORT_MAX];
    const LbvhSeg S = segs[blockIdx.x];
    if (S.count == 0 || S.count > LOCAL_SORT_MAX) return;              // block-uniform
    const uint32_t m = S.count, t = threadIdx.x;
    uint32_t np = 1;
    while (np < m) np <<= 1;
    for (uint32_t k = t; k < np; k += BLOCK)
        sk[k] = k < m ? ((unsigned long long)keys_in[S.item_base + k] << 32) | k : ~0ull;
    __syncthreads();
    for (uint32_t size = 2; size <= np; size <<= 1)
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (uint32_t k = t; k < np; k += BLOCK) {
                const uint32_t o = k ^ stride;
                if (o > k) {
                    const unsigned long long x = sk[k], y = sk[o];
                    if ((x > y) == ((k & size) == 0)) { sk[k] = y; sk[o] = x; }
                }
            }
            __syncthreads();
        }
    for (uint32_t k = t; k < m; k += BLOCK) {
        keys_out[S.item_base + k] = (uint32_t)(sk[k] >> 32);
        vals_out[S.item_base + k] = S.item_base + (uint32_t)sk[k];
    }
}

// Leaf-ordered BLAS records (rt_api.cpp builds the same records on the host: Triangle.cuh:26-46,
// Parallelogram.cuh:26-39).
__device__ __forceinline__ uint32_t material_slot(uint32_t type, uint32_t index, uint32_t rough_count) {
    return type == RT_MAT_ROUGH ? index : ((rough_count + index) | MAT_METAL_BIT);
}

__device__ __forceinline__ void gather_item(const LbvhSeg &S, uint32_t p, const uint32_t *vals, const RawPrimsGPU &raw,
                                            const PrimOutGPU &out, const uint32_t *item_member, const TriHot *stage) {
    const uint32_t slot = S.slot_base + (p - S.item_base);
    if (stage && S.ptype == RT_PRIM_TRIANGLE && !out.tri_cold) {     // prep staged the record in item order
        out.tri_hot[slot] = stage[vals[p]];
        return;
    }
    const uint32_t prim = S.prim_base + (vals[p] - S.item_base);
    if (S.ptype == RT_PRIM_TRIANGLE) {
        const float *tv = raw.tri_verts + 9 * (size_t)prim;
        const V3 v0 = v3(tv[0], tv[1], tv[2]);
        const V3 e1 = v3(tv[3], tv[4], tv[5]) - v0, e2 = v3(tv[6], tv[7], tv[8]) - v0;
        const uint32_t member = S.member_count ? item_member[vals[p]] : 0u;   // a group's BLAS: member instance + 1
        TriHot H;
        H.v0[0] = v0.x; H.v0[1] = v0.y; H.v0[2] = v0.z; H.pad0 = 0.0f;
        H.e1[0] = e1.x; H.e1[1] = e1.y; H.e1[2] = e1.z; H.pad1 = 0.0f;
        H.e2[0] = e2.x; H.e2[1] = e2.y; H.e2[2] = e2.z; H.pad2 = 0.0f;
        if (!out.tri_cold) {                          // no cold records: the index and member ride in the pads
            H.pad0 = __uint_as_float(prim);
            H.pad1 = __uint_as_float(member);
            out.tri_hot[slot] = H;
            return;
        }
        const rt_triangle &t = raw.tris[prim];
        V3 nn[3];
        if (t.has_normals) { nn[0] = of(t.normal[0]); nn[1] = of(t.normal[1]); nn[2] = of(t.normal[2]); }
        else { const V3 u = unit(cross(e1, e2)); nn[0] = u; nn[1] = u; nn[2] = u; }
        TriCold C;
        C.n0[0] = nn[0].x; C.n0[1] = nn[0].y; C.n0[2] = nn[0].z;
        C.n1[0] = nn[1].x; C.n1[1] = nn[1].y; C.n1[2] = nn[1].z;
        C.n2[0] = nn[2].x; C.n2[1] = nn[2].y; C.n2[2] = nn[2].z;
        C.material = material_slot(t.material_type, t.material_index, raw.rough_count);
        C.orig_index = prim;
        C.pad = member;
        out.tri_hot[slot] = H;
        out.tri_cold[slot] = C;
    } else if (S.ptype == RT_PRIM_SPHERE) {
        const rt_sphere sp = raw.spheres[prim];
        SphereHot H;
        H.center[0] = sp.center.x; H.center[1] = sp.center.y; H.center[2] = sp.center.z; H.radius = sp.radius;
        PrimCold C;
        C.material = material_slot(sp.material_type, sp.material_index, raw.rough_count);
        C.orig_index = prim; C.pad0 = 0; C.pad1 = 0;
        out.sph_hot[slot] = H;
        out.sph_cold[slot] = C;
    } else {
        const rt_parallelogram q = raw.quads[prim];
        const V3 nx = cross(of(q.u), of(q.v));
        const V3 nn = unit(nx);
        float d = 0.0f;
        d += nn.x * q.q.x; d += nn.y * q.q.y; d += nn.z * q.q.z;
        QuadHot H;
        H.n[0] = nn.x; H.n[1] = nn.y; H.n[2] = nn.z; H.d = d;
        H.q[0] = q.q.x; H.q[1] = q.q.y; H.q[2] = q.q.z; H.den = dot(nx, nx);
        H.u[0] = q.u.x; H.u[1] = q.u.y; H.u[2] = q.u.z; H.pad0 = 0.0f;
        H.v[0] = q.v.x; H.v[1] = q.v.y; H.v[2] = q.v.z; H.pad1 = 0.0f;
        H.nx[0] = nx.x; H.nx[1] = nx.y; H.nx[2] = nx.z; H.pad2 = 0.0f;
        PrimCold C;
        C.material = material_slot(q.material_type, q.material_index, raw.rough_count);
        C.orig_index = prim; C.pad0 = 0; C.pad1 = 0;
        out.quad_hot[slot] = H;
        out.quad_cold[slot] = C;
    }
}

// Karras 2012, one thread per interior node.  Local indices are positions inside the segment.  The sorted codes
// within KWIN positions of the workgroup's own are staged in LDS first: nearly every node's searches stay inside
// that window (a range of <= KWIN / 2 items), so a search step is an LDS read, not a dependent global load.
constexpr int KWIN = 256;
__global__ __launch_bounds__(BLOCK) void karras_kernel(const LbvhSeg *segs, const uint32_t *seg_of, const uint32_t *keys,
                                                       uint32_t n, uint32_t *child, uint32_t *parent, uint32_t *parent_leaf,
                                                       uint32_t *range, uint32_t *flag, const uint32_t *vals, RawPrimsGPU raw,
                                                       PrimOutGPU out, const uint32_t *item_member, const TriHot *stage,
                                                       uint32_t gather) {
    __shared__ uint32_t skey[BLOCK + 2 * KWIN];
    const int64_t w0 = (int64_t)blockIdx.x * BLOCK - KWIN;       // position of skey[0]
    for (int k = threadIdx.x; k < BLOCK + 2 * KWIN; k += BLOCK) {
        const int64_t q = w0 + k;
        skey[k] = (q >= 0 && q < (int64_t)n) ? keys[q] : 0u;
    }
    __syncthreads();
    const uint32_t p = blockIdx.x * BLOCK + threadIdx.x;
    if (p >= n) return;
    const LbvhSeg S = segs[seg_of[p]];
    // fused BLAS gather (build() with raw / out): item p's leaf-ordered record; its loads overlap the searches below
    if (gather) gather_item(S, p, vals, raw, out, item_member, stage);
    const int m = (int)S.count;
    const int i = (int)(p - S.item_base);
    if (m == 1) { parent_leaf[p] = NONE; return; }
    if (i >= m - 1) return;
    const auto key = [&](int a) -> uint32_t {                    // code at segment position a (0 <= a < m)
        const int64_t pos = (int64_t)S.item_base + a, o = pos - w0;
        return (o >= 0 && o < BLOCK + 2 * KWIN) ? skey[o] : keys[pos];
    };
    const uint32_t ki = key(i);
    auto delta = [&](int a, int b) -> int {                      // a == i throughout
        if (b < 0 || b >= m) return -1;
        const uint32_t ka = ki, kb = key(b);
        if (ka != kb) return __clz(ka ^ kb);
        return 32 + __clz((uint32_t)a ^ (uint32_t)b);
    };
    const int d = (delta(i, i + 1) - delta(i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(i, i - d);
    int lmax = 2;
    while (delta(i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (delta(i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int gamma = i + s * d + (d < 0 ? -1 : 0);
    const int lo = i < j ? i : j, hi = i < j ? j : i;
    const uint32_t g = S.node_base + (uint32_t)i;
    uint32_t c0, c1;
    if (lo == gamma) { c0 = LEAF_BIT | (S.item_base + (uint32_t)gamma); parent_leaf[S.item_base + gamma] = g; }
    else { c0 = S.node_base + (uint32_t)gamma; parent[c0] = g; }
    if (hi == gamma + 1) { c1 = LEAF_BIT | (S.item_base + (uint32_t)gamma + 1); parent_leaf[S.item_base + gamma + 1] = g; }
    else { c1 = S.node_base + (uint32_t)gamma + 1; parent[c1] = g; }
    child[2 * g] = c0;
    child[2 * g + 1] = c1;
    range[2 * g] = S.item_base + (uint32_t)lo;
    range[2 * g + 1] = S.item_base + (uint32_t)hi;
    flag[g] = 0;
    if (i == 0) parent[g] = NONE;
}

// ---- bottom-up box union -------------------------------------------------------------------------
// Each leaf climbs; the second thread to reach a node finishes it (union of the two child boxes,
// height) and climbs on.  Trees of <= LOCAL_MAX items (every particle BLAS, small TLASes) are
// finished by one workgroup with node boxes and arrival counters in LDS, so the hand-off between
// the two arriving threads is a workgroup-scope one.  Larger trees use the device-wide kernel, where
// the two threads may sit on different XCDs (per-XCD L2s are not coherent): the finished node is
// published with write-through (sc1) stores, drained (s_waitcnt vmcnt(0)) before the arrival
// counter's agent-scope add, and the second arriver reads it with sc1 loads — no __threadfence()
// (an L2 writeback + invalidate per step, MI355X_MICROARCH.md § visibility).
constexpr uint32_t LOCAL_MAX = 2048;

__device__ __forceinline__ void union_children(const uint32_t *child, uint32_t g, const uint32_t *vals, const float *item_box,
                                               float *b, uint32_t &h, const float *node_box_lds, const uint32_t *height_lds,
                                               uint32_t node_base, bool sc1) {
    h = 0;
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const uint32_t ch = child[2 * g + c];
        float cb[6];
        uint32_t chh = 0;
        if (ch & LEAF_BIT) {
            const float2 *src = reinterpret_cast<const float2 *>(item_box + 6 * (size_t)vals[ch & ~LEAF_BIT]);
#pragma unroll
            for (int k = 0; k < 3; k++) { const float2 v = src[k]; cb[2 * k] = v.x; cb[2 * k + 1] = v.y; }
        } else if (!sc1) {
            const uint32_t l = ch - node_base;
#pragma unroll
            for (int k = 0; k < 6; k++) cb[k] = node_box_lds[6 * l + k];
            chh = height_lds[l];
        } else {
            const unsigned long long *src = reinterpret_cast<const unsigned long long *>(node_box_lds + 6 * (size_t)ch);
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const unsigned long long v = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                cb[2 * k] = __uint_as_float((uint32_t)v);
                cb[2 * k + 1] = __uint_as_float((uint32_t)(v >> 32));
            }
            chh = __hip_atomic_load(height_lds + ch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (c == 0) {
#pragma unroll
            for (int k = 0; k < 6; k++) b[k] = cb[k];
        } else {
            merge_into(b, cb);
        }
        h = chh > h ? chh : h;
    }
}

__global__ __launch_bounds__(BLOCK) void bottom_up_local_kernel(const LbvhSeg *segs, const uint32_t *vals, const float *item_box,
                                                                const uint32_t *child, const uint32_t *parent,
                                                                const uint32_t *parent_leaf, const uint32_t *range,
                                                                float *nbox, uint32_t *height, uint32_t *kept) {
    __shared__ float sbox[(LOCAL_MAX - 1) * 6];
    __shared__ uint32_t sheight[LOCAL_MAX - 1];
    __shared__ uint32_t sflag[LOCAL_MAX - 1];
    const LbvhSeg S = segs[blockIdx.x];
    if (S.count < 2 || S.count > LOCAL_MAX) return;                    // block-uniform
    const uint32_t m = S.count, ni = m - 1;
    for (uint32_t k = threadIdx.x; k < ni; k += BLOCK) sflag[k] = 0;
    __syncthreads();
    for (uint32_t li = threadIdx.x; li < m; li += BLOCK) {
        uint32_t g = parent_leaf[S.item_base + li];
        while (g != NONE) {
            const uint32_t l = g - S.node_base;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (atomicAdd(&sflag[l], 1u) == 0u) break;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            float b[6];
            uint32_t h;
            union_children(child, g, vals, item_box, b, h, sbox, sheight, S.node_base, false);
            const uint32_t size = range[2 * g + 1] - range[2 * g] + 1u;
#pragma unroll
            for (int k = 0; k < 6; k++) sbox[6 * l + k] = b[k];
            sheight[l] = size > S.leaf_cap ? h + 1u : 0u;
            g = parent[g];
        }
    }
    __syncthreads();
    for (uint32_t l = threadIdx.x; l < ni; l += BLOCK) {
        const uint32_t g = S.node_base + l;
#pragma unroll
        for (int k = 0; k < 6; k++) nbox[6 * (size_t)g + k] = sbox[6 * l + k];
        height[g] = sheight[l];
        kept[g] = (range[2 * g + 1] - range[2 * g] + 1u) > S.leaf_cap ? 1u : 0u;
    }
}

// Large trees (> LOCAL_MAX items, e.g. C5's 10 M-triangle group BLAS): one workgroup per CHUNK consecutive sorted
// items finishes, through LDS, every node whose item range lies inside its chunk (a node's range holds its own
// index, so it has an LDS slot there) — nearly all nodes; a thread whose climb reaches a node crossing a chunk
// edge records that arrival, and a second kernel climbs from each recorded arrival with the device-wide hand-off
// described above (kernel boundary: the chunk-finished boxes are visible to it).
// (One device-wide pass over all 10 M nodes took 1.7 ms per C5 rebuild: every level an agent-scope round trip.)
#ifndef LBVH_CHUNK
#define LBVH_CHUNK 1024                         // round 6: 2048-item chunks (two items per thread, ~153 KB of LDS, one
#endif                                          // workgroup per CU) made the C5 rebuild slower: 2.33 against 2.17 ms
constexpr uint32_t CHUNK = LBVH_CHUNK;         // sorted items per workgroup
constexpr uint32_t CHUNK_THREADS = 1024;       // the chunk kernel's workgroup: CHUNK / CHUNK_THREADS items per thread
constexpr uint32_t CHUNK_PER = CHUNK / CHUNK_THREADS;
static_assert(CHUNK % CHUNK_THREADS == 0, "whole items per thread");
__device__ __forceinline__ bool chunk_local(const uint32_t *range, uint32_t g) {
    return range[2 * g] / CHUNK == range[2 * g + 1] / CHUNK;
}

// device-wide climb from node g (its range crosses a chunk edge): the hand-off described above
__device__ __forceinline__ void climb_top(const LbvhSeg &S, uint32_t g, const uint32_t *vals, const float *item_box,
                                          const uint32_t *child, const uint32_t *parent, const uint32_t *range,
                                          uint32_t *flag, float *nbox, uint32_t *height, uint32_t *kept) {
    while (g != NONE) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");              // this lane's sc1 stores have landed
        if (atomicAdd(&flag[g], 1u) == 0u) return;
        float b[6];
        uint32_t h;
        union_children(child, g, vals, item_box, b, h, nbox, height, 0, true);
        unsigned long long *dst = reinterpret_cast<unsigned long long *>(nbox + 6 * (size_t)g);
#pragma unroll
        for (int k = 0; k < 3; k++)
            __hip_atomic_store(dst + k, (unsigned long long)__float_as_uint(b[2 * k]) |
                                            ((unsigned long long)__float_as_uint(b[2 * k + 1]) << 32),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t size = range[2 * g + 1] - range[2 * g] + 1u;
        const bool keep = size > S.leaf_cap;
        __hip_atomic_store(height + g, keep ? h + 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        kept[g] = keep ? 1u : 0u;
        g = parent[g];
    }
}

// The chunk's own nodes (the interior node at each of its positions: child refs, item range, parent) are staged
// in LDS with coalesced loads before the climbs, so a climb step waits on LDS only (reading them from HBM / L2 per
// step made every level a dependent global round trip: 0.64 ms per C5 rebuild).  LBVH_CHUNK = 2048 (two items per
// thread) halves the chunk edges and the top pass's device-wide climbs, but was measured slower (above).
__global__ __launch_bounds__(CHUNK_THREADS) void bottom_up_chunk_kernel(const LbvhSeg *segs, const uint32_t *seg_of,
                                                                        const uint32_t *vals, const float *item_box,
                                                                        uint32_t n, const uint32_t *child,
                                                                        const uint32_t *parent, const uint32_t *parent_leaf,
                                                                        const uint32_t *range, float *nbox, uint32_t *height,
                                                                        uint32_t *kept, uint32_t *frontier) {
    __shared__ float sleaf[CHUNK * 6];          // the chunk's item boxes, in sorted order
    __shared__ float sbox[CHUNK * 6];           // node boxes, at the node's own position
    __shared__ uint32_t sheight[CHUNK];
    __shared__ uint32_t sflag[CHUNK];
    __shared__ uint2 schild[CHUNK], srange[CHUNK];   // the interior node at each position (segment's last: unused)
    __shared__ uint32_t sparent[CHUNK];
    constexpr uint32_t FRONT_LDS = 256;         // this chunk's arrivals for the top pass (~20 typical; more go direct)
    __shared__ uint32_t sfront[FRONT_LDS];
    __shared__ uint32_t sfront_n, sfront_at;
    const uint32_t lo = blockIdx.x * CHUNK;
    for (uint32_t j = 0; j < CHUNK_PER; j++) sflag[threadIdx.x + j * CHUNK_THREADS] = 0;
    if (threadIdx.x == 0) sfront_n = 0;
    uint32_t seg[CHUNK_PER];
    bool big[CHUNK_PER];
    LbvhSeg S[CHUNK_PER];
#pragma unroll
    for (uint32_t j = 0; j < CHUNK_PER; j++) {
        const uint32_t l = threadIdx.x + j * CHUNK_THREADS, p = lo + l;
        seg[j] = p < n ? seg_of[p] : NONE;
        big[j] = seg[j] != NONE && segs[seg[j]].count > LOCAL_MAX;   // else bottom_up_local_kernel
        if (big[j]) {
            S[j] = segs[seg[j]];
            const float2 *src = reinterpret_cast<const float2 *>(item_box + 6 * (size_t)vals[p]);
#pragma unroll
            for (int k = 0; k < 3; k++) { const float2 v = src[k]; sleaf[6 * l + 2 * k] = v.x; sleaf[6 * l + 2 * k + 1] = v.y; }
            if (p - S[j].item_base + 1u < S[j].count) {
                const uint32_t g = S[j].node_base + (p - S[j].item_base);
                schild[l] = reinterpret_cast<const uint2 *>(child)[g];
                srange[l] = reinterpret_cast<const uint2 *>(range)[g];
                sparent[l] = parent[g];
            }
        }
    }
    __syncthreads();
    for (uint32_t j = 0; j < CHUNK_PER; j++) {
        if (!big[j]) continue;
        const uint32_t p = lo + threadIdx.x + j * CHUNK_THREADS;
        const LbvhSeg &Sj = S[j];
        uint32_t g = parent_leaf[p];
        bool first = false;                             // stopped as a node's first arrival
        while (g != NONE) {
            const uint32_t l = Sj.item_base + (g - Sj.node_base) - lo;   // the node's own position, if in this chunk
            if (l >= CHUNK) break;                                       // its range leaves the chunk
            const uint2 rg = srange[l];
            if (rg.x / CHUNK != rg.y / CHUNK) break;                     // the same
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (atomicAdd(&sflag[l], 1u) == 0u) { first = true; break; }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            float b[6];
            uint32_t h = 0;
            const uint2 cc = schild[l];
#pragma unroll
            for (int c = 0; c < 2; c++) {                                // union_children's order
                const uint32_t ch = c == 0 ? cc.x : cc.y;
                const float *cb;
                uint32_t chh = 0;
                if (ch & LEAF_BIT) {                                     // sorted position = the leaf's item index
                    cb = sleaf + 6 * ((ch & ~LEAF_BIT) - lo);
                } else {                                                 // inside the parent's range: this chunk
                    const uint32_t lc = Sj.item_base + (ch - Sj.node_base) - lo;
                    cb = sbox + 6 * lc;
                    chh = sheight[lc];
                }
                if (c == 0) {
#pragma unroll
                    for (int k = 0; k < 6; k++) b[k] = cb[k];
                } else {
                    float t[6];
#pragma unroll
                    for (int k = 0; k < 6; k++) t[k] = cb[k];
                    merge_into(b, t);
                }
                h = chh > h ? chh : h;
            }
            const uint32_t size = rg.y - rg.x + 1u;
#pragma unroll
            for (int k = 0; k < 6; k++) sbox[6 * l + k] = b[k];
            sheight[l] = size > Sj.leaf_cap ? h + 1u : 0u;
            g = sparent[l];
        }
        if (!first && g != NONE) {                      // g's range crosses a chunk edge: an arrival for the top pass
            const uint32_t k = atomicAdd(&sfront_n, 1u);
            if (k < FRONT_LDS) sfront[k] = g;
            else frontier[1 + atomicAdd(frontier, 1u)] = g;
        }
    }
    __syncthreads();
    // one global reservation per chunk (~20 arrivals each): a per-arrival atomic on the one frontier counter
    // serialised ~200 k same-address atomics per C5 rebuild at the L2 (0.64 ms for the whole kernel)
    const uint32_t nf = sfront_n < FRONT_LDS ? sfront_n : FRONT_LDS;
    if (threadIdx.x == 0 && nf) sfront_at = atomicAdd(frontier, nf);
    __syncthreads();
    if (threadIdx.x < nf) frontier[1 + sfront_at + threadIdx.x] = sfront[threadIdx.x];
#pragma unroll
    for (uint32_t j = 0; j < CHUNK_PER; j++) {
        const uint32_t l = threadIdx.x + j * CHUNK_THREADS, p = lo + l;
        if (sflag[l] == 2u) {                                            // the node at this position finished here
            const uint32_t g = S[j].node_base + (p - S[j].item_base);
            const uint2 rg = srange[l];
#pragma unroll
            for (int k = 0; k < 6; k++) nbox[6 * (size_t)g + k] = sbox[6 * l + k];
            height[g] = sheight[l];
            kept[g] = (rg.y - rg.x + 1u) > S[j].leaf_cap ? 1u : 0u;
        }
    }
}

// the top pass: one climb per arrival the chunk pass recorded (frontier[0] = count, then crossing-node ids)
__global__ void bottom_up_top_kernel(const LbvhSeg *segs, const uint32_t *seg_of, const uint32_t *vals,
                                     const float *item_box, const uint32_t *child, const uint32_t *parent,
                                     const uint32_t *range, uint32_t *flag, float *nbox, uint32_t *height, uint32_t *kept,
                                     const uint32_t *frontier) {
    const uint32_t count = frontier[0];
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < count; i += gridDim.x * BLOCK) {
        const uint32_t g = frontier[1 + i];
        climb_top(segs[seg_of[range[2 * g]]], g, vals, item_box, child, parent, range, flag, nbox, height, kept);
    }
}

struct ChildInfo { uint32_t ref; const float *box; };

__device__ __forceinline__ uint32_t child_ref(const LbvhSeg &S, uint32_t ch, const uint32_t *range, const uint32_t *pidx) {
    if (ch & LEAF_BIT)
        return make_leaf_ref(S.slot_base + ((ch & ~LEAF_BIT) - S.item_base), 1u, S.ptype, S.blas != 0);
    const uint32_t first = range[2 * ch], size = range[2 * ch + 1] - first + 1u;
    if (size <= S.leaf_cap) return make_leaf_ref(S.slot_base + (first - S.item_base), size, S.ptype, S.blas != 0);
    return make_interior_ref(pidx[ch], S.blas != 0);
}
__device__ __forceinline__ const float *child_box(uint32_t ch, const uint32_t *vals, const float *item_box, const float *nbox) {
    return (ch & LEAF_BIT) ? item_box + 6 * (size_t)vals[ch & ~LEAF_BIT] : nbox + 6 * (size_t)ch;
}

__global__ void emit_kernel(const LbvhSeg *segs, const uint32_t *seg_of, const uint32_t *vals, const float *item_box,
                            uint32_t n_int, const uint32_t *child, const uint32_t *range, const float *nbox,
                            const uint32_t *kept, const uint32_t *pidx, NodePair *pairs, uint32_t *pair_count) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= n_int) return;
    if (g == n_int - 1 && pair_count) *pair_count = pidx[g] + kept[g];
    if (!kept[g]) return;
    const LbvhSeg S = segs[seg_of[range[2 * g]]];
    const uint32_t c0 = child[2 * g], c1 = child[2 * g + 1];
    const float *b0 = child_box(c0, vals, item_box, nbox), *b1 = child_box(c1, vals, item_box, nbox);
    NodePair P;
#pragma unroll
    for (int k = 0; k < 6; k++) { P.c0[k] = b0[k]; P.c1[k] = b1[k]; }
    P.ref0 = child_ref(S, c0, range, pidx);
    P.ref1 = child_ref(S, c1, range, pidx);
    P.pad0 = 0; P.pad1 = 0;
    float4 *dst = reinterpret_cast<float4 *>(pairs + pidx[g]);
    const float4 *src = reinterpret_cast<const float4 *>(&P);
#pragma unroll
    for (int k = 0; k < 4; k++) dst[k] = src[k];
}

__global__ void roots_kernel(const LbvhSeg *segs, uint32_t n_segs, const uint32_t *vals, const float *item_box,
                             const float *nbox, const uint32_t *height, const uint32_t *pidx, TreeRoot *roots) {
    const uint32_t s = blockIdx.x * BLOCK + threadIdx.x;
    if (s >= n_segs) return;
    const LbvhSeg S = segs[s];
    TreeRoot R;
    const float *b;
    if (S.count == 0) {
        for (int k = 0; k < 6; k++) R.box[k] = 0.0f;
        R.ref = NONE; R.height = 0;
        roots[s] = R;
        return;
    }
    if (S.count == 1) {
        b = item_box + 6 * (size_t)vals[S.item_base];
        R.ref = make_leaf_ref(S.slot_base, 1u, S.ptype, S.blas != 0);
        R.height = 0;
    } else {
        b = nbox + 6 * (size_t)S.node_base;
        R.ref = S.count <= S.leaf_cap ? make_leaf_ref(S.slot_base, S.count, S.ptype, S.blas != 0)
                                      : make_interior_ref(pidx[S.node_base], S.blas != 0);
        R.height = height[S.node_base];
    }
    for (int k = 0; k < 6; k++) R.box[k] = b[k];
    roots[s] = R;
}



__global__ void gather_items_kernel(const LbvhSeg *segs, const uint32_t *seg_of, const uint32_t *vals, uint32_t n,
                                    uint32_t *slots) {
    const uint32_t p = blockIdx.x * BLOCK + threadIdx.x;
    if (p >= n) return;
    const LbvhSeg S = segs[seg_of[p]];
    slots[S.slot_base + (p - S.item_base)] = vals[p];
}

// ---- 4-wide collapse of a built forest (the quad form the FAST persistent kernel traverses) -------
// Restates flatten_tree_wide (bvh_build.hpp) on the GPU: the quad of node pair q holds q's two binary
// levels as two halves (layout.hpp NodeQuad) — slots 0, 1 = the left child's children, slots 2, 3 = the
// right child's, a leaf child in its half's first slot and an empty slot with a copy of its box — so a ray
// descends half as many dependent levels and the kernel still visits the binary tree's order; leaves and
// boxes are the binary tree's.  Quad q is the quad rooted at node pair q (pair indices are unique across
// the forest, so the interior refs the pairs hold are also the quads' refs, and a tree's quad root ref
// equals its pair root ref).  One workgroup per tree walks it level by level: a frontier of quad roots in
// LDS (global scratch, this tree's pair range, for trees of more than LDS_FRONT pairs).
constexpr uint32_t LDS_FRONT = 1024;

__device__ __forceinline__ NodeQuad collapse_pair(const NodePair *pairs, uint32_t q) {
    const NodePair P = pairs[q];
    NodeQuad Q;
    for (uint32_t h = 0; h < 2; h++) {
        const float *b = h ? P.c1 : P.c0;
        const uint32_t r = h ? P.ref1 : P.ref0;
        if (r & REF_LEAF) {
            quad_set_slot(Q, 2 * h, b, r);
            quad_set_slot(Q, 2 * h + 1, b, REF_EMPTY);
        } else {
            const NodePair C = pairs[r & REF_INDEX_MASK];
            quad_set_slot(Q, 2 * h, C.c0, C.ref0);
            quad_set_slot(Q, 2 * h + 1, C.c1, C.ref1);
        }
    }
    return Q;
}

__global__ __launch_bounds__(BLOCK) void collapse_wide_kernel(const LbvhSeg *segs, const TreeRoot *roots, const NodePair *pairs,
                                                              NodeQuad *quads, uint32_t *scratch, uint32_t scratch_half,
                                                              TreeRoot *roots_wide) {
    __shared__ uint32_t lds_front[2][LDS_FRONT];
    __shared__ uint32_t n_cur, n_next;
    const uint32_t s = blockIdx.x, t = threadIdx.x;
    const TreeRoot R = roots[s];
    if (roots_wide && t == 0) roots_wide[s] = R;              // quad root ref == pair root ref
    if ((R.ref & REF_LEAF) || R.ref == NONE) return;          // a leaf (or empty) tree has no quads
    const uint32_t root = R.ref & REF_INDEX_MASK;
    const uint32_t max_pairs = segs[s].count > 1 ? segs[s].count - 1 : 1;
    uint32_t *front[2];
    if (max_pairs <= LDS_FRONT) { front[0] = lds_front[0]; front[1] = lds_front[1]; }
    else {          // this tree's own pair range [root, root + its pairs): a frontier never holds more
        front[0] = scratch + root;
        front[1] = scratch + scratch_half + root;
    }
    if (t == 0) { front[0][0] = root; n_cur = 1; n_next = 0; }
    __syncthreads();
    uint32_t cur = 0;
    while (n_cur > 0) {
        const uint32_t nc_level = n_cur;
        for (uint32_t i = t; i < nc_level; i += BLOCK) {
            const uint32_t q = front[cur][i];
            const NodeQuad Q = collapse_pair(pairs, q);
            for (uint32_t k = 0; k < 4; k++)
                if (Q.ref[k] != REF_EMPTY && !(Q.ref[k] & REF_LEAF))
                    front[cur ^ 1][atomicAdd(&n_next, 1u)] = Q.ref[k] & REF_INDEX_MASK;
            float4 *dst = reinterpret_cast<float4 *>(quads + q);
            const float4 *src = reinterpret_cast<const float4 *>(&Q);
#pragma unroll
            for (int k = 0; k < 8; k++) dst[k] = src[k];
        }
        __syncthreads();
        if (t == 0) { n_cur = n_next; n_next = 0; }
        cur ^= 1;
        __syncthreads();
    }
}

// The same quads for forests with a large tree (an instance group's merged BLAS: C5's 10 M triangles in one
// tree would keep the per-tree kernel's single workgroup walking level by level for ~60 ms): quad q is a pure
// function of node pair q (its children's children, collapse_pair), so every pair gets
// its quad, one thread each; the quads of pairs absorbed into a parent's quad are written but never reached.
__global__ void collapse_all_kernel(const NodePair *pairs, const uint32_t *n_pairs, NodeQuad *quads) {
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    if (q >= *n_pairs) return;
    const NodeQuad Q = collapse_pair(pairs, q);
    float4 *dst = reinterpret_cast<float4 *>(quads + q);
    const float4 *src = reinterpret_cast<const float4 *>(&Q);
#pragma unroll
    for (int k = 0; k < 8; k++) dst[k] = src[k];
}

__global__ void copy_roots_kernel(const TreeRoot *roots, uint32_t n, TreeRoot *roots_wide) {
    const uint32_t s = blockIdx.x * BLOCK + threadIdx.x;
    if (s < n) roots_wide[s] = roots[s];                        // quad root ref == pair root ref
}

// ---- the whole per-frame GPU TLAS in one workgroup (GPU-built frames with few TLAS items) ---------------
// The multi-kernel chain (instance deltas -> records -> bounds -> Morton -> radix sort -> Karras -> boxes ->
// scan -> pairs -> roots -> quads -> slots -> slot-ordered records) is ~17 launches on one stream per frame:
// ~100 us of launch gaps for a C2-size TLAS, which bounded GPU-built C2 frames.  With option "group" a GPU-built
// scene's TLAS holds a handful of items (C2: 6, C5: 6 of 9,772 records), so one workgroup runs the same build
// in LDS: the same Morton codes, the stable (key, item) order, Karras' hierarchy, exact box unions, leaf
// collapse, node pairs, quads and slots — over the active records only (inactive ones are left out instead of
// being sorted behind them).
constexpr uint32_t SMALL_BLOCK = 1024;

__global__ __launch_bounds__(SMALL_BLOCK) void tlas_small_kernel(SmallTlasArgs a) {
    __shared__ unsigned long long skey[SMALL_TLAS_MAX];        // (Morton << 32 | live index), sorted
    __shared__ float snbox[(SMALL_TLAS_MAX - 1) * 6];
    __shared__ float sibox[SMALL_TLAS_MAX * 6];               // live item boxes
    __shared__ uint32_t schild[2 * (SMALL_TLAS_MAX - 1)], sparent[SMALL_TLAS_MAX - 1], srange[2 * (SMALL_TLAS_MAX - 1)];
    __shared__ uint32_t sparent_leaf[SMALL_TLAS_MAX], sflag[SMALL_TLAS_MAX - 1], sheight[SMALL_TLAS_MAX - 1];
    __shared__ uint32_t spidx[SMALL_TLAS_MAX], slive[SMALL_TLAS_MAX];
    __shared__ uint32_t scount[SMALL_BLOCK];
    __shared__ uint32_t sbound[6];
    const uint32_t t = threadIdx.x, n = a.n;
    if (t < 6) sbound[t] = (t & 1) ? 0u : 0xFFFFFFFFu;
    // 1. the live records (instance_update_kernel computed every record; centroid w != 0 marks an inactive one),
    // in record order: contiguous chunks per thread
    const uint32_t chunk = (n + SMALL_BLOCK - 1) / SMALL_BLOCK, i0 = t * chunk, i1 = min(n, i0 + chunk);
    uint32_t live = 0;
    for (uint32_t i = i0; i < i1; i++) live += a.tcent[i].w == 0.0f ? 1u : 0u;
    scount[t] = live;
    __syncthreads();
    if (t == 0) {                                            // exclusive scan of the per-thread live counts
        uint32_t acc = 0;
        for (uint32_t k = 0; k < SMALL_BLOCK; k++) { const uint32_t v = scount[k]; scount[k] = acc; acc += v; }
        sflag[0] = acc;                                      // (reused below) m
    }
    __syncthreads();
    const uint32_t m = sflag[0];
    uint32_t pos = scount[t];
    for (uint32_t i = i0; i < i1; i++)
        if (a.tcent[i].w == 0.0f && pos < SMALL_TLAS_MAX) slive[pos++] = i;
    __syncthreads();
    if (m == 0 || m > SMALL_TLAS_MAX) {                      // the host checked; nothing to build
        if (t == 0) { *a.pair_count = 0; }
        return;
    }
    // 2. item boxes / centroid bounds over the live items (bounds_kernel), Morton keys (morton_kernel)
    for (uint32_t k = t; k < m; k += SMALL_BLOCK) {
        const uint32_t i = slive[k];
#pragma unroll
        for (int q = 0; q < 6; q++) sibox[6 * k + q] = a.tbox[6 * (size_t)i + q];
        const float4 c = a.tcent[i];
        atomicMin(&sbound[0], f2o(c.x)); atomicMax(&sbound[1], f2o(c.x));
        atomicMin(&sbound[2], f2o(c.y)); atomicMax(&sbound[3], f2o(c.y));
        atomicMin(&sbound[4], f2o(c.z)); atomicMax(&sbound[5], f2o(c.z));
    }
    __syncthreads();
    uint32_t np = 1;
    while (np < m) np <<= 1;
    for (uint32_t k = t; k < np; k += SMALL_BLOCK) {
        unsigned long long key = ~0ull;
        if (k < m) {
            const float4 c = a.tcent[slive[k]];
            const uint32_t x = quant10(c.x, o2f(sbound[0]), o2f(sbound[1]));
            const uint32_t y = quant10(c.y, o2f(sbound[2]), o2f(sbound[3]));
            const uint32_t z = quant10(c.z, o2f(sbound[4]), o2f(sbound[5]));
            key = ((unsigned long long)((expand10(x) << 2) | (expand10(y) << 1) | expand10(z)) << 32) | k;
        }
        skey[k] = key;
    }
    __syncthreads();
    // bitonic sort of (code, item): the radix sort's stable order
    for (uint32_t size = 2; size <= np; size <<= 1)
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (uint32_t k = t; k < np; k += SMALL_BLOCK) {
                const uint32_t o = k ^ stride;
                if (o > k) {
                    const unsigned long long x = skey[k], y = skey[o];
                    const bool up = (k & size) == 0;
                    if ((x > y) == up) { skey[k] = y; skey[o] = x; }
                }
            }
            __syncthreads();
        }
    // 3. Karras hierarchy over the sorted codes (karras_kernel, one segment)
    const int mi = (int)m;
    auto code = [&](int i) { return (uint32_t)(skey[i] >> 32); };
    auto delta = [&](int x, int y) -> int {
        if (y < 0 || y >= mi) return -1;
        const uint32_t kx = code(x), ky = code(y);
        if (kx != ky) return __clz(kx ^ ky);
        return 32 + __clz((uint32_t)x ^ (uint32_t)y);
    };
    for (int i = (int)t; i < mi - 1; i += SMALL_BLOCK) {
        const int d = (delta(i, i + 1) - delta(i, i - 1)) >= 0 ? 1 : -1;
        const int dmin = delta(i, i - d);
        int lmax = 2;
        while (delta(i, i + lmax * d) > dmin) lmax <<= 1;
        int l = 0;
        for (int q = lmax >> 1; q >= 1; q >>= 1)
            if (delta(i, i + (l + q) * d) > dmin) l += q;
        const int j = i + l * d;
        const int dnode = delta(i, j);
        int sp = 0, q = l;
        do {
            q = (q + 1) >> 1;
            if (delta(i, i + (sp + q) * d) > dnode) sp += q;
        } while (q > 1);
        const int gamma = i + sp * d + (d < 0 ? -1 : 0);
        const int lo = i < j ? i : j, hi = i < j ? j : i;
        uint32_t c0, c1;
        if (lo == gamma) { c0 = LEAF_BIT | (uint32_t)gamma; sparent_leaf[gamma] = (uint32_t)i; }
        else { c0 = (uint32_t)gamma; sparent[gamma] = (uint32_t)i; }
        if (hi == gamma + 1) { c1 = LEAF_BIT | (uint32_t)(gamma + 1); sparent_leaf[gamma + 1] = (uint32_t)i; }
        else { c1 = (uint32_t)gamma + 1; sparent[gamma + 1] = (uint32_t)i; }
        schild[2 * i] = c0; schild[2 * i + 1] = c1;
        srange[2 * i] = (uint32_t)lo; srange[2 * i + 1] = (uint32_t)hi;
        sflag[i] = 0;
        if (i == 0) sparent[0] = NONE;
    }
    if (m == 1 && t == 0) sparent_leaf[0] = NONE;
    __syncthreads();
    // 4. exact box unions bottom-up (bottom_up_local_kernel)
    const uint32_t cap = a.leaf_cap;
    for (uint32_t li = t; li < m && m > 1; li += SMALL_BLOCK) {
        uint32_t g = sparent_leaf[li];
        while (g != NONE) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (atomicAdd(&sflag[g], 1u) == 0u) break;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            float b[6];
            uint32_t h = 0;
            for (int c = 0; c < 2; c++) {
                const uint32_t ch = schild[2 * g + c];
                const float *cb = (ch & LEAF_BIT) ? sibox + 6 * (skey[ch & ~LEAF_BIT] & 0xFFFFFFFFu) : snbox + 6 * ch;
                const uint32_t chh = (ch & LEAF_BIT) ? 0u : sheight[ch];
                if (c == 0) {
                    for (int k = 0; k < 6; k++) b[k] = cb[k];
                } else {
                    merge_into(b, cb);
                }
                h = chh > h ? chh : h;
            }
            const uint32_t size = srange[2 * g + 1] - srange[2 * g] + 1u;
#pragma unroll
            for (int k = 0; k < 6; k++) snbox[6 * g + k] = b[k];
            sheight[g] = size > cap ? h + 1u : 0u;
            g = sparent[g];
        }
    }
    __syncthreads();
    // 5. kept interior nodes -> pair index (exclusive scan), pairs, root, slots
    if (t == 0) {
        uint32_t acc = 0;
        for (uint32_t g = 0; g + 1 < m; g++) {
            spidx[g] = acc;
            acc += (srange[2 * g + 1] - srange[2 * g] + 1u) > cap ? 1u : 0u;
        }
        *a.pair_count = acc;
    }
    __syncthreads();
    auto ref_of = [&](uint32_t ch) -> uint32_t {
        if (ch & LEAF_BIT) return make_leaf_ref(ch & ~LEAF_BIT, 1u, 0u, false);
        const uint32_t first = srange[2 * ch], size = srange[2 * ch + 1] - first + 1u;
        if (size <= cap) return make_leaf_ref(first, size, 0u, false);
        return make_interior_ref(spidx[ch], false);
    };
    for (uint32_t g = t; g + 1 < m; g += SMALL_BLOCK) {
        if ((srange[2 * g + 1] - srange[2 * g] + 1u) <= cap) continue;
        const uint32_t c0 = schild[2 * g], c1 = schild[2 * g + 1];
        const float *b0 = (c0 & LEAF_BIT) ? sibox + 6 * (skey[c0 & ~LEAF_BIT] & 0xFFFFFFFFu) : snbox + 6 * c0;
        const float *b1 = (c1 & LEAF_BIT) ? sibox + 6 * (skey[c1 & ~LEAF_BIT] & 0xFFFFFFFFu) : snbox + 6 * c1;
        NodePair P;
#pragma unroll
        for (int k = 0; k < 6; k++) { P.c0[k] = b0[k]; P.c1[k] = b1[k]; }
        P.ref0 = ref_of(c0);
        P.ref1 = ref_of(c1);
        P.pad0 = 0; P.pad1 = 0;
        a.pairs[spidx[g]] = P;
    }
    for (uint32_t k = t; k < m; k += SMALL_BLOCK) a.slots[k] = slive[skey[k] & 0xFFFFFFFFu];
    if (t == 0) {
        TreeRoot R;
        const float *b = m == 1 ? sibox : snbox;
        for (int k = 0; k < 6; k++) R.box[k] = b[k];
        R.ref = m == 1 ? make_leaf_ref(0, 1u, 0u, false)
                       : (m <= cap ? make_leaf_ref(0, m, 0u, false) : make_interior_ref(spidx[0], false));
        R.height = m == 1 ? 0u : sheight[0];
        *a.root = R;
        *a.root_wide = R;                                    // quad root ref == pair root ref
    }
    __syncthreads();                                         // pairs and records (global, this workgroup) complete
    // 6. quads (collapse_all_kernel) and the records in leaf-slot order (slot_order_kernel)
    const uint32_t npairs = *a.pair_count;
    for (uint32_t q = t; q < npairs; q += SMALL_BLOCK) {
        const NodeQuad Q = collapse_pair(a.pairs, q);
        a.quads[q] = Q;
    }
    for (uint32_t k = t; k < m; k += SMALL_BLOCK) {
        const uint32_t i = slive[skey[k] & 0xFFFFFFFFu];
        a.hot_s[k] = a.hot[i];
        a.cold_s[k] = a.cold[i];
    }
}

}  // namespace lbvh

__global__ void extract_tri_verts_kernel(const rt_triangle *tris, float *verts, size_t first, size_t count) {
    const size_t k = (size_t)blockIdx.x * lbvh::BLOCK + threadIdx.x;
    if (k >= count) return;
    const rt_triangle &t = tris[first + k];
    float *v = verts + 9 * (first + k);
#pragma unroll
    for (int i = 0; i < 3; i++) { v[3 * i] = t.vertex[i].x; v[3 * i + 1] = t.vertex[i].y; v[3 * i + 2] = t.vertex[i].z; }
}

hipError_t extract_tri_verts(const rt_triangle *tris, float *verts, size_t first, size_t count, hipStream_t stream) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(extract_tri_verts_kernel, dim3((uint32_t)((count + lbvh::BLOCK - 1) / lbvh::BLOCK)), dim3(lbvh::BLOCK), 0, stream, tris,
                       verts, first, count);
    return hipGetLastError();
}

hipError_t launch_tlas_small(const SmallTlasArgs &a, hipStream_t stream) {
    hipLaunchKernelGGL(lbvh::tlas_small_kernel, dim3(1), dim3(lbvh::SMALL_BLOCK), 0, stream, a);
    return hipGetLastError();
}

// ---- host --------------------------------------------------------------------------------------
using namespace lbvh;

#define LB_TRY(x)                               \
    do {                                        \
        hipError_t e_ = (x);                    \
        if (e_ != hipSuccess) return e_;        \
    } while (0)

template <typename T>
static hipError_t dalloc(T *&p, size_t n) {
    return hipMalloc(reinterpret_cast<void **>(&p), (n ? n : 1) * sizeof(T));
}
template <typename T>
static void dfree(T *&p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

void LbvhBuilder::release() {
    for (hipEvent_t &e : stage_ev_)
        if (e) { (void)hipEventDestroy(e); e = nullptr; }
    timing_ = false;
    last_timed_ = false;
    dfree(segs_); dfree(seg_of_); dfree(members_); dfree(item_member_); dfree(own_box_); dfree(own_cent_); dfree(stage_); dfree(bounds_);
    dfree(k0_); dfree(k1_); dfree(v0_); dfree(v1_); dfree(child_); dfree(parent_); dfree(parent_leaf_);
    dfree(range_); dfree(flag_); dfree(height_); dfree(nbox_); dfree(kept_); dfree(pidx_); dfree(front_); dfree(count_); dfree(frontier_);
    last_count_ = nullptr;
    if (tmp_) (void)hipFree(tmp_);
    tmp_ = nullptr; tmp_bytes_ = 0;
    box_ = nullptr; cent_ = nullptr;
    n_items_ = n_segs_ = 0;
    big_segs_.clear();
}

hipError_t LbvhBuilder::init(const std::vector<LbvhSeg> &segs, hipStream_t stream) {
    release();
    uint64_t n = 0;
    for (const LbvhSeg &s : segs) {
        if (s.item_base != n || s.leaf_cap < 1 || s.leaf_cap > 4) return hipErrorInvalidValue;
        n += s.count;
    }
    if (n >= (1ull << 31) || segs.empty()) return hipErrorInvalidValue;
    n_items_ = (uint32_t)n;
    n_segs_ = (uint32_t)segs.size();
    max_count_ = 0;
    for (const LbvhSeg &sg : segs) max_count_ = sg.count > max_count_ ? sg.count : max_count_;
    big_segs_.clear();
    uint32_t big_max = 0;
    for (const LbvhSeg &sg : segs)
        if (sg.count > LOCAL_SORT_MAX) { big_segs_.push_back({sg.item_base, sg.count}); big_max = std::max(big_max, sg.count); }
    const size_t N = n_items_, NI = max_pairs();
    LB_TRY(dalloc(segs_, n_segs_));
    LB_TRY(hipMemcpyAsync(segs_, segs.data(), n_segs_ * sizeof(LbvhSeg), hipMemcpyHostToDevice, stream));
    std::vector<uint32_t> seg_of(N);
    for (uint32_t s = 0; s < n_segs_; s++)
        for (uint32_t k = 0; k < segs[s].count; k++) seg_of[segs[s].item_base + k] = s;
    LB_TRY(dalloc(seg_of_, N));
    LB_TRY(hipMemcpyAsync(seg_of_, seg_of.data(), N * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
    LB_TRY(dalloc(bounds_, 6 * (size_t)n_segs_));
    LB_TRY(dalloc(k0_, N)); LB_TRY(dalloc(k1_, N)); LB_TRY(dalloc(v0_, N)); LB_TRY(dalloc(v1_, N));
    LB_TRY(dalloc(child_, 2 * NI)); LB_TRY(dalloc(parent_, NI)); LB_TRY(dalloc(parent_leaf_, N));
    LB_TRY(dalloc(range_, 2 * NI)); LB_TRY(dalloc(flag_, NI)); LB_TRY(dalloc(height_, NI));
    LB_TRY(dalloc(nbox_, 6 * NI)); LB_TRY(dalloc(kept_, NI)); LB_TRY(dalloc(pidx_, NI));
    size_t sort_bytes = 0, scan_bytes = 0;
    if (big_max) LB_TRY(rocprim::radix_sort_pairs(nullptr, sort_bytes, k0_, k1_, v0_, v1_, big_max, 0, 32, stream));
    LB_TRY(rocprim::exclusive_scan(nullptr, scan_bytes, kept_, pidx_, 0u, NI, rocprim::plus<uint32_t>(), stream));
    tmp_bytes_ = sort_bytes > scan_bytes ? sort_bytes : scan_bytes;
    LB_TRY(hipMalloc(&tmp_, tmp_bytes_ ? tmp_bytes_ : 1));
    // kept/pidx of nodes that no thread visits (none in a valid forest) start defined
    LB_TRY(hipMemsetAsync(kept_, 0, NI * sizeof(uint32_t), stream));
    // synchronous: seg_of (host vector) must outlive the copy
    return hipStreamSynchronize(stream);
}

const char *const LbvhBuilder::STAGE_NAMES[LbvhBuilder::STAGES] = {
    "prep", "bounds", "morton", "sort", "karras_gather", "bottom_up", "scan", "emit_roots", "collapse"};

hipError_t LbvhBuilder::set_timing(bool on) {
    if (on)
        for (hipEvent_t &e : stage_ev_)
            if (!e) LB_TRY(hipEventCreate(&e));
    timing_ = on;
    return hipSuccess;
}

hipError_t LbvhBuilder::stage_ms(float (&ms)[STAGES]) const {
    if (!last_timed_) return hipErrorNotReady;          // the last build ran without timing: no stale figures
    for (int k = 0; k < STAGES; k++) {
        ms[k] = 0.0f;
        if (!stage_ev_[k] || !stage_ev_[k + 1]) return hipErrorInvalidValue;
        LB_TRY(hipEventSynchronize(stage_ev_[k + 1]));
        LB_TRY(hipEventElapsedTime(&ms[k], stage_ev_[k], stage_ev_[k + 1]));
    }
    return hipSuccess;
}

hipError_t LbvhBuilder::prep_blas_items(const RawPrimsGPU &raw, hipStream_t stream, bool stage_hot) {
    last_timed_ = timing_;
    LB_TRY(mark(0, stream));
    if (!own_box_) {
        LB_TRY(dalloc(own_box_, 6 * (size_t)n_items_));
        LB_TRY(dalloc(own_cent_, n_items_));
    }
    if (stage_hot && !stage_) LB_TRY(dalloc(stage_, n_items_));
    box_ = own_box_;
    cent_ = own_cent_;
    stage_ready_ = stage_hot;
    hipLaunchKernelGGL(prep_blas_kernel, dim3(blocks_for(n_items_)), dim3(BLOCK), 0, stream, segs_, seg_of_, n_items_, raw,
                       box_, cent_, stage_hot ? stage_ : nullptr, item_member_);
    LB_TRY(hipGetLastError());
    return mark(1, stream);
}

// item -> its member instance + 1 (group segments; 0 elsewhere), found once here instead of by every rebuild's gather
__global__ void member_map_kernel(const LbvhSeg *segs, const uint32_t *seg_of, uint32_t n, const uint32_t *members,
                                  uint32_t *item_member) {
    const uint32_t it = blockIdx.x * BLOCK + threadIdx.x;
    if (it >= n) return;
    const LbvhSeg S = segs[seg_of[it]];
    uint32_t v = 0;
    if (S.member_count) {
        const uint32_t prim = S.prim_base + (it - S.item_base);
        const uint32_t *M = members + 2 * (size_t)S.member_base;
        uint32_t lo = 0, hi = S.member_count;          // last member whose first primitive <= prim
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) / 2;
            if (M[2 * mid] <= prim) lo = mid; else hi = mid;
        }
        v = M[2 * lo + 1] + 1u;
    }
    item_member[it] = v;
}

hipError_t LbvhBuilder::set_members(const std::vector<uint32_t> &pairs, hipStream_t stream) {
    dfree(members_);
    dfree(item_member_);
    members_n_ = 0;
    if (pairs.empty()) return hipSuccess;
    LB_TRY(dalloc(members_, pairs.size()));
    members_n_ = pairs.size();
    LB_TRY(dalloc(item_member_, (size_t)n_items_));
    LB_TRY(hipMemcpyAsync(members_, pairs.data(), pairs.size() * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(member_map_kernel, dim3(blocks_for(n_items_)), dim3(BLOCK), 0, stream, segs_, seg_of_, n_items_,
                       members_, item_member_);
    LB_TRY(hipGetLastError());
    return hipStreamSynchronize(stream);            // `pairs` (host) must outlive the copy
}

size_t LbvhBuilder::workspace_bytes() const {
    if (!segs_) return 0;
    const size_t N = n_items_, NI = max_pairs(), u = sizeof(uint32_t);
    size_t b = n_segs_ * sizeof(LbvhSeg) + N * u /*seg_of*/ + 6 * (size_t)n_segs_ * u /*bounds*/ + 4 * N * u /*keys, values*/ +
               N * u /*parent_leaf*/ + NI * (2 + 1 + 2 + 1 + 1 + 6 + 1 + 1) * u /*child parent range flag height nbox kept pidx*/ +
               tmp_bytes_;
    if (own_box_) b += 6 * N * sizeof(float) + N * sizeof(float4);
    if (stage_) b += N * sizeof(TriHot);
    if (members_) b += members_n_ * u;
    if (item_member_) b += N * u;
    if (frontier_) b += (1 + 2 * NI) * u;
    if (front_) b += 2 * (size_t)max_pairs() * u;
    if (count_) b += u;
    return b;
}

hipError_t LbvhBuilder::set_items(const float *boxes, const float4 *centroids) {
    box_ = const_cast<float *>(boxes);
    cent_ = const_cast<float4 *>(centroids);
    return hipSuccess;
}

hipError_t LbvhBuilder::build(NodePair *pairs, TreeRoot *roots, uint32_t *pair_count, hipStream_t stream,
                              const RawPrimsGPU *raw, const PrimOutGPU *out) {
    if (!box_ || !cent_ || n_items_ == 0) return hipErrorInvalidValue;
    const uint32_t N = n_items_, NI = n_items_ - n_segs_;
    hipLaunchKernelGGL(init_bounds_kernel, dim3(blocks_for(6ull * n_segs_)), dim3(BLOCK), 0, stream, bounds_, n_segs_);
    {   // ~1024 blocks at most: one LDS-combined atomic set per block (bounds_kernel)
        const uint32_t ipt = std::max<uint32_t>(1u, (uint32_t)((N + (uint64_t)BLOCK * 1024 - 1) / ((uint64_t)BLOCK * 1024)));
        const uint32_t nb = (uint32_t)((N + (uint64_t)BLOCK * ipt - 1) / ((uint64_t)BLOCK * ipt));
        hipLaunchKernelGGL(bounds_kernel, dim3(nb), dim3(BLOCK), 0, stream, seg_of_, cent_, N, ipt, bounds_);
    }
    if (box_ == own_box_) LB_TRY(mark(2, stream));           // BLAS builds: stage timing (TLAS builds record nothing)
    const bool tm = box_ == own_box_;
    hipLaunchKernelGGL(morton_kernel, dim3(blocks_for(N)), dim3(BLOCK), 0, stream, seg_of_, cent_, N, bounds_, k0_, v0_);
    LB_TRY(hipGetLastError());
    if (tm) LB_TRY(mark(3, stream));
    size_t bytes = tmp_bytes_;
    if (big_segs_.size() < n_segs_)
        hipLaunchKernelGGL(local_sort_kernel, dim3(n_segs_), dim3(BLOCK), 0, stream, segs_, k0_, k1_, v1_);
    // BLAS codes are 30-bit Morton codes; TLAS items may be inactive (0xFFFFFFFF)
    const int end_bit = box_ == own_box_ ? 30 : 32;
    for (const auto &b : big_segs_) {
        bytes = tmp_bytes_;
        LB_TRY(rocprim::radix_sort_pairs(tmp_, bytes, k0_ + b.first, k1_ + b.first, v0_ + b.first, v1_ + b.first, b.second, 0,
                                         end_bit, stream));
    }
    if (tm) LB_TRY(mark(4, stream));
    hipLaunchKernelGGL(karras_kernel, dim3(blocks_for(N)), dim3(BLOCK), 0, stream, segs_, seg_of_, k1_, N, child_, parent_,
                       parent_leaf_, range_, flag_, v1_, raw ? *raw : RawPrimsGPU{}, out ? *out : PrimOutGPU{}, item_member_,
                       stage_ready_ ? stage_ : nullptr, (uint32_t)(raw && out));
    stage_ready_ = false;
    if (tm) LB_TRY(mark(5, stream));
    hipLaunchKernelGGL(bottom_up_local_kernel, dim3(n_segs_), dim3(BLOCK), 0, stream, segs_, v1_, box_, child_, parent_,
                       parent_leaf_, range_, nbox_, height_, kept_);
    if (max_count_ > LOCAL_MAX) {
        if (!frontier_) LB_TRY(dalloc(frontier_, 1 + 2 * (size_t)NI));   // <= 2 arrivals per internal node
        LB_TRY(hipMemsetAsync(frontier_, 0, sizeof(uint32_t), stream));
        hipLaunchKernelGGL(bottom_up_chunk_kernel, dim3((N + CHUNK - 1) / CHUNK), dim3(CHUNK_THREADS), 0, stream, segs_, seg_of_, v1_,
                           box_, N, child_, parent_, parent_leaf_, range_, nbox_, height_, kept_, frontier_);
        hipLaunchKernelGGL(bottom_up_top_kernel, dim3(256), dim3(BLOCK), 0, stream, segs_, seg_of_, v1_, box_, child_, parent_,
                           range_, flag_, nbox_, height_, kept_, frontier_);
    }
    LB_TRY(hipGetLastError());
    if (tm) LB_TRY(mark(6, stream));
    if (!pair_count) {                                // collapse_wide needs the count of this build's pairs
        if (!count_) LB_TRY(dalloc(count_, 1));
        pair_count = count_;
    }
    last_count_ = pair_count;
    if (NI > 0) {
        bytes = tmp_bytes_;
        LB_TRY(rocprim::exclusive_scan(tmp_, bytes, kept_, pidx_, 0u, NI, rocprim::plus<uint32_t>(), stream));
        if (tm) LB_TRY(mark(7, stream));
        hipLaunchKernelGGL(emit_kernel, dim3(blocks_for(NI)), dim3(BLOCK), 0, stream, segs_, seg_of_, v1_, box_, NI, child_,
                           range_, nbox_, kept_, pidx_, pairs, pair_count);
    } else {
        if (pair_count) LB_TRY(hipMemsetAsync(pair_count, 0, sizeof(uint32_t), stream));
        if (tm) LB_TRY(mark(7, stream));
    }
    hipLaunchKernelGGL(roots_kernel, dim3(blocks_for(n_segs_)), dim3(BLOCK), 0, stream, segs_, n_segs_, v1_, box_, nbox_,
                       height_, pidx_, roots);
    LB_TRY(hipGetLastError());
    return tm ? mark(8, stream) : hipSuccess;
}

hipError_t LbvhBuilder::collapse_wide(const NodePair *pairs, const TreeRoot *roots, NodeQuad *quads, TreeRoot *roots_wide,
                                      hipStream_t stream) {
    const bool tm = box_ == own_box_;
    if (max_count_ > COLLAPSE_ALL_MIN && last_count_) {
        hipLaunchKernelGGL(collapse_all_kernel, dim3(blocks_for(max_pairs())), dim3(BLOCK), 0, stream, pairs, last_count_, quads);
        if (roots_wide)
            hipLaunchKernelGGL(copy_roots_kernel, dim3(blocks_for(n_segs_)), dim3(BLOCK), 0, stream, roots, n_segs_, roots_wide);
        LB_TRY(hipGetLastError());
        return tm ? mark(9, stream) : hipSuccess;
    }
    if (max_count_ - 1 > LDS_FRONT && !front_) LB_TRY(dalloc(front_, 2 * (size_t)max_pairs()));
    hipLaunchKernelGGL(collapse_wide_kernel, dim3(n_segs_), dim3(BLOCK), 0, stream, segs_, roots, pairs, quads, front_,
                       max_pairs(), roots_wide);
    LB_TRY(hipGetLastError());
    return tm ? mark(9, stream) : hipSuccess;
}

hipError_t LbvhBuilder::gather_items(uint32_t *slots, hipStream_t stream) {
    hipLaunchKernelGGL(gather_items_kernel, dim3(blocks_for(n_items_)), dim3(BLOCK), 0, stream, segs_, seg_of_, v1_, n_items_,
                       slots);
    return hipGetLastError();
}

}  // namespace rtamd

