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
// The large trees' rocPRIM sort: onesweep over 10-bit digits (3 passes over a 30-bit code) instead of rocPRIM's gfx950
// default of 8 (4 passes).  Measured on 10 M clustered Morton pairs (scripts/sort_bench.hip, profiles/r06/sort/):
// 0.404 -> 0.279 ms per sort; 9 bits 0.401, 11 bits 0.376, 10 bits over 512 x 16 or 1024 x 24 items 0.33 / 0.35.
#ifndef LBVH_SORT_BITS
#define LBVH_SORT_BITS 10
#endif
using BigSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 16>, rocprim::kernel_config<1024, 16>, LBVH_SORT_BITS,
                                        rocprim::block_radix_rank_algorithm::match>>;
// the pair-index scan over every interior node's kept flag: 256 x 32 items per block, 0.051 -> 0.036 ms over 10 M flags
// against rocPRIM's default (scripts/scan_bench.hip, profiles/r06/sort/)
using PairScanConfig = rocprim::scan_config<256, 32, rocprim::block_load_method::block_load_transpose,
                                            rocprim::block_store_method::block_store_transpose,
                                            rocprim::block_scan_algorithm::using_warp_scan>;
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
constexpr uint32_t LOCAL_MAX = 2048;    // trees of <= LOCAL_MAX items: bottom_up_local_kernel (one workgroup, LDS)
__global__ __launch_bounds__(BLOCK) void karras_kernel(const LbvhSeg *segs, const uint32_t *seg_of, const uint32_t *keys,
                                                       uint32_t n, uint32_t *child, uint32_t *parent, uint32_t *parent_leaf,
                                                       uint32_t *range, uint32_t *flag, const uint32_t *vals, RawPrimsGPU raw,
                                                       PrimOutGPU out, const uint32_t *item_member, const TriHot *stage,
                                                       uint32_t gather, uint32_t small_only) {
    __shared__ uint32_t skey[BLOCK + 2 * KWIN];
    if (small_only) {               // trees of > LOCAL_MAX items: hierarchy_chunk_kernel (block-uniform exit)
        const uint32_t p0 = blockIdx.x * BLOCK, p1 = min(p0 + BLOCK, n) - 1u;
        const uint32_t s0 = seg_of[p0];
        if (s0 == seg_of[p1] && segs[s0].count > LOCAL_MAX) return;
    }
    const int64_t w0 = (int64_t)blockIdx.x * BLOCK - KWIN;       // position of skey[0]
    for (int k = threadIdx.x; k < BLOCK + 2 * KWIN; k += BLOCK) {
        const int64_t q = w0 + k;
        skey[k] = (q >= 0 && q < (int64_t)n) ? keys[q] : 0u;
    }
    __syncthreads();
    const uint32_t p = blockIdx.x * BLOCK + threadIdx.x;
    if (p >= n) return;
    const LbvhSeg S = segs[seg_of[p]];
    if (small_only && S.count > LOCAL_MAX) return;
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
// the two arriving threads is a workgroup-scope one.  Larger trees end in a device-wide pass
// (hierarchy_top_kernel), where the two threads may sit on different XCDs (per-XCD L2s are not
// coherent): the finished node is published with write-through (sc1) stores, drained (s_waitcnt
// vmcnt(0)) before the arrival's agent-scope atomic, and the second arriver reads it with sc1
// loads — no __threadfence() (an L2 writeback + invalidate per step, MI355X_MICROARCH.md § visibility).
__device__ __forceinline__ void union_children(const uint32_t *child, uint32_t g, const uint32_t *vals, const float *item_box,
                                               float *b, uint32_t &h, const float *node_box_lds, const uint32_t *height_lds,
                                               uint32_t node_base) {
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
        } else {
            const uint32_t l = ch - node_base;
#pragma unroll
            for (int k = 0; k < 6; k++) cb[k] = node_box_lds[6 * l + k];
            chh = height_lds[l];
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
            union_children(child, g, vals, item_box, b, h, sbox, sheight, S.node_base);
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

// Large trees (> LOCAL_MAX items, e.g. C5's 10 M-triangle group BLAS): hierarchy_chunk_kernel / hierarchy_top_kernel
// below.  (One device-wide pass over all 10 M nodes took 1.7 ms per C5 rebuild: every level an agent-scope round trip;
// rounds 3-5 ran karras_kernel over them and then a chunk climb over its parent arrays: 0.42 + 0.47 ms per C5 rebuild
// against 0.78 for the two kernels below, gather included, profiles/r06/hierarchy/.)
#ifndef LBVH_CHUNK
#define LBVH_CHUNK 1024                         // 2048-item chunks (~150 KB of LDS, one workgroup per CU): 2.33 against
#endif                                          // 2.17 ms per C5 rebuild (round 6, Karras chunks); 512: equal, 256: +0.27 ms
#ifndef LBVH_TOP_BLOCKS
#define LBVH_TOP_BLOCKS 4096                    // hierarchy_top_kernel's grid (its gather wants the waves; 256: +0.2 ms)
#endif
constexpr uint32_t CHUNK = LBVH_CHUNK;         // sorted items per workgroup
constexpr uint32_t CHUNK_THREADS = CHUNK < 1024 ? CHUNK : 1024;   // the chunk kernel's workgroup: CHUNK / CHUNK_THREADS items per thread
constexpr uint32_t CHUNK_PER = CHUNK / CHUNK_THREADS;
static_assert(CHUNK % CHUNK_THREADS == 0, "whole items per thread");

// ---- large trees without the Karras pass: hierarchy and boxes in one bottom-up climb ------------------------------
// Apetrei, "Fast and Simple Agglomerative LBVH Construction" (CGVC 2014): over the sorted codes, a finished node
// [l, r] is its parent's LEFT child iff l == 0 or (r != m - 1 and δ(r, r + 1) > δ(l - 1, l)) — the parent takes the
// neighbour sharing the longer prefix (δ as karras_kernel's: code prefix, then the position's, so no two adjacent δ
// are equal) — and the parent's split lies at r (left child) or l - 1 (right child).  That is the same binary radix
// tree Karras' per-node searches build, and the Karras index of every node follows from it locally: a left child's
// index is its last position, a right child's its first (the root's is 0), and the children of the node split at γ
// are Karras nodes / leaves γ and γ + 1.  So each leaf climbs, the second arrival at a split finishes the parent
// (range, children, box, height) and writes it at its Karras index: the arrays karras_kernel + a climb over its parent
// arrays produce, bit for bit, without the searches, the parent arrays or a second pass over the chunk (tests/test_gpu_lbvh.py
// compares every node with the restatement).  Arrival bits per split: 1 / 2 = the left / right child arrived, 4 / 8 =
// that child is a leaf.
struct SegKeys {                // the top pass's view of one tree's sorted codes (the chunk pass stages δ in LDS)
    const uint32_t *keys;       // sorted codes (global)
    uint32_t base;              // the segment's first sorted position
    int m;                      // the segment's items
};
__device__ __forceinline__ uint32_t seg_key(const SegKeys &K, int a) { return K.keys[(size_t)K.base + a]; }
__device__ __forceinline__ int seg_delta(const SegKeys &K, int a, int b) {      // 0 <= a < m
    if (b < 0 || b >= K.m) return -1;
    const uint32_t ka = seg_key(K, a), kb = seg_key(K, b);
    if (ka != kb) return __clz(ka ^ kb);
    return 32 + __clz((uint32_t)a ^ (uint32_t)b);
}
__device__ __forceinline__ bool left_child(const SegKeys &K, int l, int r) {
    return l == 0 || (r != K.m - 1 && seg_delta(K, r, r + 1) > seg_delta(K, l - 1, l));
}

// Chunk pass: one workgroup per CHUNK sorted positions finishes every node whose range lies inside the chunk (LDS
// arrivals, node records at their Karras index in LDS), and also writes the chunk's leaf-ordered primitive records
// (karras_kernel's fused gather).  A climb whose parent split has a child outside the chunk, and every split that got
// only one of its arrivals here, go to the top pass as (split, bits) arrivals.
__global__ __launch_bounds__(CHUNK_THREADS) void hierarchy_chunk_kernel(const LbvhSeg *segs, const uint32_t *seg_of,
                                                                        const uint32_t *keys, const uint32_t *vals,
                                                                        const float *item_box, uint32_t n, uint32_t *child,
                                                                        uint32_t *range, float *nbox, uint32_t *height,
                                                                        uint32_t *kept, uint32_t *frontier) {
    __shared__ int sdel[CHUNK + 1];             // δ(q, q + 1) for positions q = lo - 1 .. lo + CHUNK - 1 (-1 across trees)
    __shared__ float sleaf[CHUNK * 6];          // the chunk's item boxes, in sorted order
    __shared__ float sbox[CHUNK * 6];           // node boxes, at the node's Karras index
    __shared__ uint32_t sheight[CHUNK];
    __shared__ uint2 srl[CHUNK];                // node range (segment-local first, last); x = NONE: not finished here
    __shared__ uint32_t ssplit[CHUNK];          // node split (segment-local)
    __shared__ uint32_t sarr[CHUNK];            // arrival bits per split position
    constexpr uint32_t FRONT_LDS = 256;         // this chunk's arrivals for the top pass (more go direct)
    __shared__ uint2 sfront[FRONT_LDS];
    __shared__ uint32_t sfront_n, sfront_at;
    const uint32_t lo = blockIdx.x * CHUNK;
    if (threadIdx.x == 0) sfront_n = 0;
    // the parent rule compares only adjacent δ's: each is computed once here (seg_delta's value) instead of from four
    // staged codes per climb step
    for (uint32_t k = threadIdx.x; k < CHUNK + 1; k += CHUNK_THREADS) {
        const int64_t q = (int64_t)lo - 1 + k;
        int d = -1;
        if (q >= 0 && q + 1 < (int64_t)n) {
            const uint32_t s0 = seg_of[q];
            if (s0 == seg_of[q + 1]) {
                const uint32_t ka = keys[q], kb = keys[q + 1], a = (uint32_t)q - segs[s0].item_base;
                d = ka != kb ? __clz(ka ^ kb) : 32 + __clz(a ^ (a + 1u));
            }
        }
        sdel[k] = d;
    }
    bool big[CHUNK_PER];
    LbvhSeg S[CHUNK_PER];
#pragma unroll
    for (uint32_t j = 0; j < CHUNK_PER; j++) {
        const uint32_t l = threadIdx.x + j * CHUNK_THREADS, p = lo + l;
        sarr[l] = 0;
        srl[l].x = NONE;
        const uint32_t seg = p < n ? seg_of[p] : NONE;
        big[j] = seg != NONE && segs[seg].count > LOCAL_MAX;   // else karras_kernel + bottom_up_local_kernel
        if (big[j]) {
            S[j] = segs[seg];
            const float2 *src = reinterpret_cast<const float2 *>(item_box + 6 * (size_t)vals[p]);
#pragma unroll
            for (int k = 0; k < 3; k++) { const float2 v = src[k]; sleaf[6 * l + 2 * k] = v.x; sleaf[6 * l + 2 * k + 1] = v.y; }
        }
    }
    __syncthreads();
    for (uint32_t j = 0; j < CHUNK_PER; j++) {
        if (!big[j]) continue;
        const uint32_t p = lo + threadIdx.x + j * CHUNK_THREADS;
        const LbvhSeg &Sj = S[j];
        const int m = (int)Sj.count;
        const int off = (int)((int64_t)Sj.item_base - (int64_t)lo + 1);   // sdel[off + i] = δ(i, i + 1), segment-local i
        const auto left_child_local = [&](int l, int r) {
            return l == 0 || (r != m - 1 && sdel[off + r] > sdel[off + l - 1]);
        };
        int l = (int)(p - Sj.item_base), r = l;
        bool leaf = true, left = left_child_local(l, r);
        for (;;) {
            const int gam = left ? r : l - 1;
            const uint32_t P = Sj.item_base + (uint32_t)gam;       // the split: children at positions P, P + 1
            const uint32_t bits = (left ? 1u : 2u) | (leaf ? (left ? 4u : 8u) : 0u);
            if (P < lo || P + 1 >= lo + CHUNK) {                 // a child outside the chunk: the top pass's
                const uint32_t k = atomicAdd(&sfront_n, 1u);
                if (k < FRONT_LDS) sfront[k] = make_uint2(P, bits);
                else {
                    const uint32_t at = atomicAdd(frontier, 1u);
                    frontier[1 + 2 * at] = P;
                    frontier[2 + 2 * at] = bits;
                }
                break;
            }
            const uint32_t sl = P - lo, sr = sl + 1;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            const uint32_t old = atomicOr(&sarr[sl], bits);
            if (old == 0u) break;                                 // first arrival: the sibling finishes the parent
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            const uint32_t a = old | bits;
            const int lL = (a & 4u) ? gam : (int)srl[sl].x;
            const int rR = (a & 8u) ? gam + 1 : (int)srl[sr].y;
            const float *c0 = (a & 4u) ? sleaf + 6 * sl : sbox + 6 * sl;
            const float *c1 = (a & 8u) ? sleaf + 6 * sr : sbox + 6 * sr;
            float b[6], t[6];
#pragma unroll
            for (int k = 0; k < 6; k++) { b[k] = c0[k]; t[k] = c1[k]; }
            merge_into(b, t);                                     // union_children's order
            const uint32_t h0 = (a & 4u) ? 0u : sheight[sl], h1 = (a & 8u) ? 0u : sheight[sr];
            const uint32_t h = h0 > h1 ? h0 : h1;
            const bool root = lL == 0 && rR == m - 1;
            const bool nleft = !root && left_child_local(lL, rR);
            const uint32_t slot = Sj.item_base + (uint32_t)(root ? 0 : (nleft ? rR : lL)) - lo;
            const uint32_t size = (uint32_t)(rR - lL) + 1u;
#pragma unroll
            for (int k = 0; k < 6; k++) sbox[6 * slot + k] = b[k];
            sheight[slot] = size > Sj.leaf_cap ? h + 1u : 0u;
            ssplit[slot] = (uint32_t)gam;
            srl[slot] = make_uint2((uint32_t)lL, (uint32_t)rR);
            if (root) break;
            l = lL; r = rR; leaf = false; left = nleft;
        }
    }
    __syncthreads();
    // splits that got one arrival here: the other child finishes in the top pass
#pragma unroll
    for (uint32_t j = 0; j < CHUNK_PER; j++) {
        const uint32_t l = threadIdx.x + j * CHUNK_THREADS;
        const uint32_t a = sarr[l];
        if (a != 0u && (a & 3u) != 3u) {
            const uint32_t k = atomicAdd(&sfront_n, 1u);
            if (k < FRONT_LDS) sfront[k] = make_uint2(lo + l, a);
            else {
                const uint32_t at = atomicAdd(frontier, 1u);
                frontier[1 + 2 * at] = lo + l;
                frontier[2 + 2 * at] = a;
            }
        }
    }
    __syncthreads();
    const uint32_t nf = sfront_n < FRONT_LDS ? sfront_n : FRONT_LDS;   // one global reservation per chunk
    if (threadIdx.x == 0 && nf) sfront_at = atomicAdd(frontier, nf);
    __syncthreads();
    if (threadIdx.x < nf) {
        frontier[1 + 2 * (sfront_at + threadIdx.x)] = sfront[threadIdx.x].x;
        frontier[2 + 2 * (sfront_at + threadIdx.x)] = sfront[threadIdx.x].y;
    }
#pragma unroll
    for (uint32_t j = 0; j < CHUNK_PER; j++) {
        const uint32_t l = threadIdx.x + j * CHUNK_THREADS, p = lo + l;
        const uint2 rl = srl[l];
        if (big[j] && rl.x != NONE) {                         // the node at this Karras position finished here
            const LbvhSeg &Sj = S[j];
            const uint32_t g = Sj.node_base + (p - Sj.item_base), gam = ssplit[l];
            child[2 * g] = rl.x == gam ? (LEAF_BIT | (Sj.item_base + gam)) : Sj.node_base + gam;
            child[2 * g + 1] = rl.y == gam + 1 ? (LEAF_BIT | (Sj.item_base + gam + 1)) : Sj.node_base + gam + 1;
            range[2 * g] = Sj.item_base + rl.x;
            range[2 * g + 1] = Sj.item_base + rl.y;
#pragma unroll
            for (int k = 0; k < 6; k++) nbox[6 * (size_t)g + k] = sbox[6 * l + k];
            height[g] = sheight[l];
            kept[g] = (rl.y - rl.x + 1u) > Sj.leaf_cap ? 1u : 0u;
        }
    }
}

// Top pass: one climb per recorded arrival, device-wide, with the hand-off described above bottom_up_local_kernel (node records published
// with write-through stores, drained before the arrival's agent-scope atomic, read with sc1 loads).  Arrival bits per
// split in `flag` (indexed by split position); the second arrival clears them for the next build.
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void hierarchy_top_kernel(const LbvhSeg *segs, const uint32_t *seg_of, const uint32_t *keys, const uint32_t *vals,
                                     const float *item_box, uint32_t *child, uint32_t *range, float *nbox, uint32_t *height,
                                     uint32_t *kept, uint32_t *flag, const uint32_t *frontier, uint32_t n, RawPrimsGPU raw,
                                     PrimOutGPU out, const uint32_t *item_member, const TriHot *stage, uint32_t gather) {
    const uint32_t count = frontier[0];
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < count; i += gridDim.x * BLOCK) {
        uint32_t P = frontier[1 + 2 * i], bits = frontier[2 + 2 * i];
        const LbvhSeg S = segs[seg_of[P]];
        const SegKeys K = {keys, S.item_base, (int)S.count};
        for (;;) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // this lane's sc1 stores have landed
            const uint32_t old = atomicOr(&flag[P], bits);
            if (old == 0u) break;
            flag[P] = 0u;                                              // no other arrival at P in this build
            const uint32_t a = old | bits;
            const int gam = (int)(P - S.item_base);
            const uint32_t g0 = S.node_base + (uint32_t)gam, g1 = g0 + 1u;
            float b[6], t[6];
            uint32_t h = 0;
            int lL, rR;
            if (a & 4u) {
                lL = gam;
                const float *src = item_box + 6 * (size_t)vals[P];
#pragma unroll
                for (int k = 0; k < 6; k++) b[k] = src[k];
            } else {
                lL = (int)(ld_sc1(range + 2 * (size_t)g0) - S.item_base);
                const unsigned long long *src = reinterpret_cast<const unsigned long long *>(nbox + 6 * (size_t)g0);
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    const unsigned long long v = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    b[2 * k] = __uint_as_float((uint32_t)v);
                    b[2 * k + 1] = __uint_as_float((uint32_t)(v >> 32));
                }
                h = ld_sc1(height + g0);
            }
            if (a & 8u) {
                rR = gam + 1;
                const float *src = item_box + 6 * (size_t)vals[P + 1];
#pragma unroll
                for (int k = 0; k < 6; k++) t[k] = src[k];
            } else {
                rR = (int)(ld_sc1(range + 2 * (size_t)g1 + 1) - S.item_base);
                const unsigned long long *src = reinterpret_cast<const unsigned long long *>(nbox + 6 * (size_t)g1);
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    const unsigned long long v = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    t[2 * k] = __uint_as_float((uint32_t)v);
                    t[2 * k + 1] = __uint_as_float((uint32_t)(v >> 32));
                }
                const uint32_t h1 = ld_sc1(height + g1);
                h = h1 > h ? h1 : h;
            }
            merge_into(b, t);
            const bool root = lL == 0 && rR == (int)S.count - 1;
            const bool nleft = !root && left_child(K, lL, rR);
            const uint32_t g = S.node_base + (uint32_t)(root ? 0 : (nleft ? rR : lL));
            const uint32_t size = (uint32_t)(rR - lL) + 1u;
            const bool keep = size > S.leaf_cap;
            unsigned long long *dst = reinterpret_cast<unsigned long long *>(nbox + 6 * (size_t)g);
#pragma unroll
            for (int k = 0; k < 3; k++)
                __hip_atomic_store(dst + k, (unsigned long long)__float_as_uint(b[2 * k]) |
                                                ((unsigned long long)__float_as_uint(b[2 * k + 1]) << 32),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            st_sc1(height + g, keep ? h + 1u : 0u);
            st_sc1(range + 2 * (size_t)g, S.item_base + (uint32_t)lL);
            st_sc1(range + 2 * (size_t)g + 1, S.item_base + (uint32_t)rR);
            child[2 * (size_t)g] = (a & 4u) ? (LEAF_BIT | P) : g0;
            child[2 * (size_t)g + 1] = (a & 8u) ? (LEAF_BIT | (P + 1u)) : g1;
            kept[g] = keep ? 1u : 0u;
            if (root) break;
            P = S.item_base + (uint32_t)(nleft ? rR : lL - 1);
            bits = nleft ? 1u : 2u;
        }
    }
    // the large trees' leaf-ordered primitive records (karras_kernel's fused gather for the small ones): bandwidth
    // work that fills the issue slots the climbs above leave idle while they wait on their hand-offs (on a side stream
    // beside the chunk and top kernels instead: rebuild 1.97 -> 2.06 ms, C5 frame 8.3 ms; profiles/r06/hierarchy/)
    if (gather)
        for (uint32_t p = blockIdx.x * BLOCK + threadIdx.x; p < n; p += gridDim.x * BLOCK) {
            const LbvhSeg S = segs[seg_of[p]];
            if (S.count > LOCAL_MAX) gather_item(S, p, vals, raw, out, item_member, stage);
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
    LB_TRY(dalloc(range_, 2 * NI)); LB_TRY(dalloc(flag_, N)); LB_TRY(dalloc(height_, NI));
    LB_TRY(dalloc(nbox_, 6 * NI)); LB_TRY(dalloc(kept_, NI)); LB_TRY(dalloc(pidx_, NI));
    size_t sort_bytes = 0, scan_bytes = 0;
    if (big_max) LB_TRY(rocprim::radix_sort_pairs<BigSortConfig>(nullptr, sort_bytes, k0_, k1_, v0_, v1_, big_max, 0, 32, stream));
    LB_TRY(rocprim::exclusive_scan<PairScanConfig>(nullptr, scan_bytes, kept_, pidx_, 0u, NI, rocprim::plus<uint32_t>(), stream));
    tmp_bytes_ = sort_bytes > scan_bytes ? sort_bytes : scan_bytes;
    LB_TRY(hipMalloc(&tmp_, tmp_bytes_ ? tmp_bytes_ : 1));
    // kept/pidx of nodes that no thread visits (none in a valid forest) start defined
    LB_TRY(hipMemsetAsync(kept_, 0, NI * sizeof(uint32_t), stream));
    // arrival bits of the top pass (hierarchy_top_kernel clears what it sets)
    LB_TRY(hipMemsetAsync(flag_, 0, N * sizeof(uint32_t), stream));
    // synchronous: seg_of (host vector) must outlive the copy
    return hipStreamSynchronize(stream);
}

const char *const LbvhBuilder::STAGE_NAMES[LbvhBuilder::STAGES] = {
    "prep", "bounds", "morton", "sort", "hierarchy_small", "hierarchy_large", "scan", "emit_roots", "collapse"};

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
               N * u /*parent_leaf*/ + N * u /*flag*/ + NI * (2 + 1 + 2 + 1 + 6 + 1 + 1) * u /*child parent range height nbox kept pidx*/ +
               tmp_bytes_;
    if (own_box_) b += 6 * N * sizeof(float) + N * sizeof(float4);
    if (stage_) b += N * sizeof(TriHot);
    if (members_) b += members_n_ * u;
    if (item_member_) b += N * u;
    if (frontier_) b += (1 + 2 * N) * u;
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
        LB_TRY(rocprim::radix_sort_pairs<BigSortConfig>(tmp_, bytes, k0_ + b.first, k1_ + b.first, v0_ + b.first, v1_ + b.first, b.second, 0,
                                         end_bit, stream));
    }
    if (tm) LB_TRY(mark(4, stream));
    // trees of > LOCAL_MAX items: hierarchy_chunk_kernel / hierarchy_top_kernel build them (and gather their records)
    const bool fused = max_count_ > LOCAL_MAX;
    const RawPrimsGPU graw = raw ? *raw : RawPrimsGPU{};
    const PrimOutGPU gout = out ? *out : PrimOutGPU{};
    const TriHot *gstage = stage_ready_ ? stage_ : nullptr;
    hipLaunchKernelGGL(karras_kernel, dim3(blocks_for(N)), dim3(BLOCK), 0, stream, segs_, seg_of_, k1_, N, child_, parent_,
                       parent_leaf_, range_, flag_, v1_, graw, gout, item_member_, gstage, (uint32_t)(raw && out),
                       (uint32_t)fused);
    hipLaunchKernelGGL(bottom_up_local_kernel, dim3(n_segs_), dim3(BLOCK), 0, stream, segs_, v1_, box_, child_, parent_,
                       parent_leaf_, range_, nbox_, height_, kept_);
    if (tm) LB_TRY(mark(5, stream));
    if (fused) {
        if (!frontier_) LB_TRY(dalloc(frontier_, 1 + 2 * (size_t)N));    // <= 1 (split, bits) arrival per item
        LB_TRY(hipMemsetAsync(frontier_, 0, sizeof(uint32_t), stream));
        hipLaunchKernelGGL(hierarchy_chunk_kernel, dim3((N + CHUNK - 1) / CHUNK), dim3(CHUNK_THREADS), 0, stream, segs_, seg_of_,
                           k1_, v1_, box_, N, child_, range_, nbox_, height_, kept_, frontier_);
        hipLaunchKernelGGL(hierarchy_top_kernel, dim3(LBVH_TOP_BLOCKS), dim3(BLOCK), 0, stream, segs_, seg_of_, k1_, v1_, box_, child_,
                           range_, nbox_, height_, kept_, flag_, frontier_, N, graw, gout, item_member_, gstage,
                           (uint32_t)(raw && out));
    }
    stage_ready_ = false;
    LB_TRY(hipGetLastError());
    if (tm) LB_TRY(mark(6, stream));
    if (!pair_count) {                                // collapse_wide needs the count of this build's pairs
        if (!count_) LB_TRY(dalloc(count_, 1));
        pair_count = count_;
    }
    last_count_ = pair_count;
    if (NI > 0) {
        bytes = tmp_bytes_;
        LB_TRY(rocprim::exclusive_scan<PairScanConfig>(tmp_, bytes, kept_, pidx_, 0u, NI, rocprim::plus<uint32_t>(), stream));
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

