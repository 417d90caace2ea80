// layout.hpp — HBM data layout of a scene, shared by the host builder and the HIP kernels.
//
// The reference stores AoS BLASNode/TLASNode records of 40 B (24 B box + two size_t,
// include/AS/BLAS.cuh:20-34), 16 B {type,size_t} index pairs, 112 B triangles and 464 B
// instances, and fetches them node by node with a re-test of every popped node.  This layout
// keeps exactly the same trees (same topology, same leaf order) but stores them as
//   * node PAIRS: the two child boxes of one interior node in one 64 B record (4 x dwordx4),
//     so visiting a node = one 64 B fetch that tests both children (BLAS.cu:180-202);
//   * leaf-ordered primitive arrays: a leaf's primitives are contiguous, so the per-slot index
//     array (BLAS.cu:72-77) disappears; hot intersection data (v0,e1,e2) is split from cold
//     shading data (vertex normals, material) that is only read for the final hit;
//   * instance hot records (inverse 3x4 + BLAS root box/ref, 80 B) split from cold records
//     (forward 3x4 + inverse-transpose 3x4, 96 B) used once per closest hit.
#pragma once
#include <stdint.h>

#include "../../include/rt.h"

namespace rtamd {

// ---- node references (32 bit) --------------------------------------------------------
// interior:            [31]=0 [30]=level [29:0]  node-pair index
// leaf:                [31]=1 [30]=level [29:28] primitive type (BLAS) [27:26] count-1
//                      [25:0] first slot (BLAS: slot in the type's leaf-ordered array;
//                      TLAS: slot in tlas_slots)
// level: 0 = TLAS (world-space ray), 1 = BLAS (instance-space ray)
constexpr uint32_t REF_LEAF = 1u << 31;
constexpr uint32_t REF_BLAS = 1u << 30;
constexpr uint32_t REF_INDEX_MASK = (1u << 30) - 1u;
constexpr uint32_t REF_START_MASK = (1u << 26) - 1u;
constexpr uint32_t REF_EMPTY = 0xFFFFFFFFu;       // empty NodeQuad slot (= the kernel's REF_NONE)
constexpr uint32_t MAX_LEAF_SLOTS = 1u << 26;

__host__ __device__ inline uint32_t make_interior_ref(uint32_t pair, bool blas) {
    return (blas ? REF_BLAS : 0u) | (pair & REF_INDEX_MASK);
}
__host__ __device__ inline uint32_t make_leaf_ref(uint32_t start, uint32_t count, uint32_t ptype, bool blas) {
    return REF_LEAF | (blas ? REF_BLAS : 0u) | ((ptype & 3u) << 28) | (((count - 1u) & 3u) << 26) |
           (start & REF_START_MASK);
}
__host__ __device__ inline uint32_t ref_leaf_start(uint32_t r) { return r & REF_START_MASK; }
__host__ __device__ inline uint32_t ref_leaf_count(uint32_t r) { return ((r >> 26) & 3u) + 1u; }
__host__ __device__ inline uint32_t ref_leaf_type(uint32_t r) { return (r >> 28) & 3u; }

// ---- screen-tile sharding (multi-GPU frames) ------------------------------------
// Tiles of tw x th pixels cover the frame in row-major tile order; rank r of n owns tiles t = r, r + n,
// r + 2n, ...  Its slab holds its tiles back to back, row-major inside a tile, padded to the largest
// rank's tile count.  Slab pixel i of rank r -> frame pixel (x, y); false for a pixel outside the frame
// (the right / bottom edge tiles, the padding of a short slab).  The assemble kernel, the host ABI
// (rt_tile_pixels) and the CPU protocol tests share this one definition.
__host__ __device__ inline uint32_t tiles_total(uint32_t W, uint32_t H, uint32_t tw, uint32_t th) {
    return ((W + tw - 1) / tw) * ((H + th - 1) / th);
}
__host__ __device__ inline uint32_t slab_tile_count(uint32_t W, uint32_t H, uint32_t tw, uint32_t th, uint32_t count) {
    return (tiles_total(W, H, tw, th) + count - 1) / count;      // rank 0 owns the most tiles
}
__host__ __device__ inline bool tile_pixel(uint32_t W, uint32_t H, uint32_t tw, uint32_t th, uint32_t rank, uint32_t count,
                                           uint64_t i, uint32_t &x, uint32_t &y) {
    const uint32_t tiles_x = (W + tw - 1) / tw;
    const uint64_t tile_px = (uint64_t)tw * th;
    const uint64_t t = rank + (i / tile_px) * count;
    const uint32_t p = (uint32_t)(i % tile_px);
    if (t >= tiles_total(W, H, tw, th)) return false;
    x = (uint32_t)(t % tiles_x) * tw + p % tw;
    y = (uint32_t)(t / tiles_x) * th + p / tw;
    return x < W && y < H;
}

// ---- records -------------------------------------------------------------------------
struct alignas(16) NodePair {       // 64 B
    float c0[6];                    // child 0 box {xmin,xmax,ymin,ymax,zmin,zmax}
    float c1[6];                    // child 1 box
    uint32_t ref0, ref1;            // child refs (child 0 = `left`, child 1 = `left+1`)
    uint32_t pad0, pad1;
};
static_assert(sizeof(NodePair) == 64, "NodePair must be 64 B");

// FAST kernel, option "wide": the same trees collapsed to 4 children per interior node, so a ray
// descends half as many dependent levels.  The quad of binary node N holds N's two binary levels below
// it as two halves: slots 0, 1 = the left child's two children, slots 2, 3 = the right child's (a child
// that is a leaf takes its half's first slot, and the second slot is empty).  The kernel orders the hit
// slots exactly as the reference's stack would visit them — the halves by their boxes' entry t, then the
// slots inside a half (push far / visit near per node pair, left on ties: BLAS.cu:186-202,
// TLAS.cu:182-197) — and a half's box is the union of its two slots' boxes (a node's box is the union of
// its children's, BLAS.cu:4-117), so its entry t comes from the slots' own slab planes.  Child boxes
// are SoA (one dwordx4 per bound) so the 4 slab tests share each load; an empty slot carries a copy of
// its sibling's box (the half's union stays exact) and ref REF_EMPTY, which the kernel never accepts.
struct alignas(16) NodeQuad {       // 128 B
    float lo_x[4], hi_x[4], lo_y[4], hi_y[4], lo_z[4], hi_z[4];
    uint32_t ref[4];                // child refs (interior refs index the quad array), REF_EMPTY = empty
    uint32_t pad[4];
};
static_assert(sizeof(NodeQuad) == 128, "NodeQuad must be 128 B");

// slot k of a quad: box b = {xmin, xmax, ymin, ymax, zmin, zmax}
__host__ __device__ inline void quad_set_slot(NodeQuad &q, uint32_t k, const float *b, uint32_t ref) {
    q.lo_x[k] = b[0]; q.hi_x[k] = b[1]; q.lo_y[k] = b[2]; q.hi_y[k] = b[3]; q.lo_z[k] = b[4]; q.hi_z[k] = b[5];
    q.ref[k] = ref;
    q.pad[k] = 0;
}

struct alignas(16) TriHot {         // 48 B: Moller-Trumbore operands (Triangle.cu:4-44)
    float v0[3]; float pad0;            // GPU-built BLASes without cold records (SceneGPU::raw_tris): the caller's
    float e1[3]; float pad1;            // triangle index (pad0) and the group member instance + 1 (pad1), as bits
    float e2[3]; float pad2;
};
struct alignas(16) TriCold {        // 48 B: vertex normals + material + caller index
    float n0[3]; uint32_t material;     // material = slot | (type << 31)
    float n1[3]; uint32_t orig_index;
    float n2[3]; uint32_t pad;          // a group's merged BLAS (option "group"): caller instance + 1, else 0
};
struct alignas(16) SphereHot {      // 16 B (Sphere.cu:4-49)
    float center[3]; float radius;
};
struct alignas(16) QuadHot {        // 80 B: every value Parallelogram::hit reads or recomputes
    float n[3]; float d;            // unit plane normal, plane constant (Parallelogram.cuh:31-38)
    float q[3]; float den;          // origin, |u x v|^2 (Parallelogram.cu:23-24)
    float u[3]; float pad0;
    float v[3]; float pad1;
    float nx[3]; float pad2;        // u x v, unnormalised (Parallelogram.cu:23)
};
struct alignas(16) PrimCold {       // 16 B: sphere / quad material and caller index
    uint32_t material; uint32_t orig_index; uint32_t pad0, pad1;
};

struct alignas(16) InstHot {        // 80 B: what Instance::hit needs before BLAS traversal
    float inv[12];                  // rows 1..3 of transformInverse (4 cols)  (Instance.cu:26-27)
    float root_box[6];              // BLAS root node box (local space)
    uint32_t root_ref;              // BLAS root ref (leaf or interior, level = BLAS)
    uint32_t root_ref_wide;         // the same root in the quad (option "wide") tree
};
static_assert(sizeof(InstHot) == 80, "InstHot must be 80 B");
struct alignas(16) InstCold {       // 96 B: hit finalisation (Instance.cu:41-45)
    float fwd[12];                  // rows 1..3 of transformMatrix
    float nrm[12];                  // rows 1..3 of normalTransformMatrix
};

// GPU instance update (instances.hip, GPU-built frames): per-instance inputs kept resident in HBM, and the
// delta record the host uploads for an instance whose transform or local box changed.
struct alignas(16) InstParams {     // 96 B
    float shift[3], cos[3], sin[3], scale[3];   // Instance::updateTransformArguments arguments (cos / sin: host libm)
    float box[6];                   // local box {xmin,xmax,ymin,ymax,zmin,zmax} (volume-expanded, as the host holds it)
    float centroid[3];              // local centroid
    float pad[3];                   // pad[0] != 0: inactive record (kept out of the GPU TLAS, option "group")
};
static_assert(sizeof(InstParams) == 96, "InstParams must be 96 B");
struct alignas(16) InstDelta {      // 112 B
    uint32_t index, pad0, pad1, pad2;
    InstParams p;
};
static_assert(sizeof(InstDelta) == 112, "InstDelta must be 112 B");

constexpr uint32_t MAT_METAL_BIT = 1u << 31;

struct alignas(16) TreeRoot {       // 32 B: root of one tree (GPU-built trees keep it in HBM)
    float box[6];
    uint32_t ref;
    uint32_t height;                // interior levels on the longest root-to-leaf path
};
static_assert(sizeof(TreeRoot) == 32, "TreeRoot must be 32 B");

// ---- kernel arguments ----------------------------------------------------------------
struct SceneGPU {
    const NodePair *blas_pairs;
    const NodePair *tlas_pairs;
    const uint32_t *tlas_slots;     // TLAS leaf slot -> instance index
    const InstHot *inst_hot;
    const InstCold *inst_cold;
    const TriHot *tri_hot;
    const TriCold *tri_cold;
    // GPU-built BLASes (option "cold_records" 0): no TriCold records; a hit triangle's normals and material come from
    // the caller's triangle (index in TriHot::pad0), so a per-frame rebuild writes and reads half the bytes
    const rt_triangle *raw_tris;
    const SphereHot *sph_hot;
    const PrimCold *sph_cold;
    const QuadHot *quad_hot;
    const PrimCold *quad_cold;
    const float *materials;         // 4 floats per slot: albedo.xyz, fuzz (roughs then metals)
    const TreeRoot *tlas_root;      // this frame's TLAS root, in the per-frame block (host- or GPU-built)
    const NodeQuad *blas_quads;     // option "wide" (host-built trees): quad forms of the BLASes / TLAS
    const NodeQuad *tlas_quads;
    const TreeRoot *tlas_root_wide;
    uint32_t wide;                  // FAST persistent kernel: 0 binary node pairs, 1..3 quad trees (trace_kernel.hip XBOX)
    uint32_t inst_by_slot;          // 1 (host-built TLAS): inst_hot / inst_cold are stored in TLAS leaf-slot
                                    // order, so entering an instance needs no tlas_slots load (the slot
                                    // is the record index; tlas_slots maps it back to the instance id)
    uint32_t instance_count;
    uint32_t rough_count;           // material slot of metal m = rough_count + m
    uint32_t material_count;        // slots in `materials` (roughs + metals)
    // setting "lds_scene" (FAST persistent kernel, quad trees): the frame's TLAS quads (7 dwordx4 each, the
    // pad dropped) and then, if they fit as well, the instance hot records (5 dwordx4 each) are copied into
    // LDS_SCENE_F4 dwordx4 of LDS at the start of every workgroup; 0 = read from HBM
    uint32_t lds_quads;             // TLAS quads in LDS (every TLAS interior ref indexes below it)
    uint32_t lds_insts;             // instance hot records in LDS (0 or instance_count)
    // further records in LDS when they fit as well (dwordx4 offsets into the region, LDS_NONE = in HBM):
    // instance cold records (6 dwordx4 each), sphere hot / cold (1 each), parallelogram hot (5) / cold (1)
    uint32_t lds_icold, lds_sph_hot, lds_sph_cold, lds_q_hot, lds_q_cold;
    // then the first lds_bqn quads of one BLAS (a group's, option "group", numbered level by level so they
    // are its top levels): BLAS quad q in [lds_bq0, lds_bq0 + lds_bqn) is read at lds_bq_at + (q - lds_bq0) * 7
    uint32_t lds_bq0, lds_bqn, lds_bq_at;
};
constexpr uint32_t LDS_NONE = 0xFFFFFFFFu;
#ifndef RT_LDS_SCENE_F4
#define RT_LDS_SCENE_F4 1216
#endif
constexpr uint32_t LDS_SCENE_F4 = RT_LDS_SCENE_F4;   // 19 KB per workgroup: 32 KB stack + 1 KB materials + 19 KB
                                                     // keeps 3 workgroups per CU (160 KB)
constexpr uint32_t LDS_QUAD_F4 = 7, LDS_INST_F4 = 5, LDS_ICOLD_F4 = 6, LDS_QPRIM_F4 = 5;

struct CameraGPU {                  // Camera (RendererImpl.cuh:32-61), precomputed on host
    float pixel_origin[3];
    float dx[3], dy[3];
    float center[3];
    float cu[3], cv[3];
    float background[3];
    float focus_radius;
    float recip_sqrt;
    uint32_t sqrt_s;
    uint32_t depth;
    uint32_t width, height;
    uint32_t pitch;                 // ceil(W/16)*16: the padded width of Kernel.cu:109
    uint64_t frame_seed;
};

// n / d by multiply-shift, exact for every n < 2^27 (round-up method: with l = ceil(log2 d),
// s = 27 + l and m = ceil(2^s / d), the error m d - 2^s < d <= 2^l keeps n (m d - 2^s) < 2^s).
// Work-item indices stay below 2^27 (rt_render checks units * 64); m < 2^28 + 1 fits 32 bits.
constexpr uint32_t FASTDIV_BITS = 27;
struct FastDiv {
    uint32_t d, m, s;
    __host__ __device__ uint32_t div(uint32_t n) const { return (uint32_t)(((uint64_t)n * m) >> s); }
};
inline FastDiv make_fastdiv(uint32_t d) {
    uint32_t l = 0;
    while (l < 31 && (1u << l) < d) l++;
    const uint32_t s = FASTDIV_BITS + l;
    return FastDiv{d, (uint32_t)(((1ull << s) + d - 1) / d), s};
}

struct OutputGPU {
    uint8_t *rgba;                  // uchar4 per pixel
    float *rgb;                     // optional
    uint32_t units;                 // number of 8x8 work units
    uint32_t units_x;               // frame layout: units per row
    // tile layout (tile_count > 0)
    uint32_t tile_w, tile_h, tile_rank, tile_count, tiles_x;
    // the work-item -> pixel map's divisors: units_x (frame), units per tile, units per tile row, tiles_x
    FastDiv div_units_x, div_upt, div_upr, div_tiles_x;
    // persistent kernel: work queue split into `queue_parts` bands of units (one per XCD), each with
    // its own head counter QUEUE_STRIDE words apart; optional per-wave timeline (debug)
    uint32_t queue_parts;
    uint32_t grab;                  // pixels claimed per queue atomic
    uint32_t supertile;             // frame mode, grab 64: walk bands in supertile x supertile units (0 = rows)
    unsigned long long *timeline;   // TIMELINE_WORDS per wave (rt.h, rt_scene_debug_read)
    uint32_t *costmap;              // COUNT launches: traversal rounds per output pixel (debug)
    // option "reorder" (schedule.hip): claim position j of a band takes unit order[j] (heaviest-first
    // permutation inside the band; null = natural / supertile walk), and unit_cost[u] receives the
    // largest cost (traversal rounds + 1) of unit u's pixels for the next launch's order
    const uint32_t *order;
    uint32_t *unit_cost;
    uint32_t leaf_early;            // setting "leaf_early": interior loop ends with <= this many lanes still descending
};
constexpr uint32_t QUEUE_STRIDE = 32;         // u32 words between partition heads (128 B lines)
constexpr uint32_t QUEUE_MAX_PARTS = 8;
// queue block of a lane: band heads (lines 0..7), band item counts (lines 8..15)
constexpr uint32_t QUEUE_WORDS = 2 * QUEUE_MAX_PARTS * QUEUE_STRIDE;
constexpr uint32_t SCHED_CLASSES = 16;       // cost classes of the claim order (half-octaves of steps per pixel)

// class 0 = heaviest: half-octaves of a unit's mean traversal steps per pixel, floor(2 log2(c/64 + 1))
// (a sky unit averages ~5 steps per pixel, a unit over the particle cluster ~100; classes saturate at ~180);
// in integers: 2 log2(x/64) = log2(x^2) - 12 with x = c + 64
__host__ __device__ inline uint32_t cost_class(uint32_t c) {
    const uint64_t x = (uint64_t)c + 64u;
    const int k = (63 - __builtin_clzll(x * x)) - 12;
    return (SCHED_CLASSES - 1) - (uint32_t)(k < 0 ? 0 : (k > (int)SCHED_CLASSES - 1 ? (int)SCHED_CLASSES - 1 : k));
}
// heavy units may be claimed in pieces so that several waves share them: 1/4 of a unit (16 pixels)
// from class level k_quarter up, 1/2 from k_half up (levels k = 15 - class; > 15 = never)
__host__ __device__ inline uint32_t split_log2(uint32_t cls, uint32_t k_half, uint32_t k_quarter) {
    const uint32_t k = (SCHED_CLASSES - 1) - cls;
    return k >= k_quarter ? 2u : (k >= k_half ? 1u : 0u);
}
constexpr uint32_t TIMELINE_WORDS = 20;

// Counter slots (device uint64 array)
enum CounterSlot : uint32_t {
    CNT_RAYS = 0, CNT_PIXELS, CNT_PAIRS, CNT_TRI, CNT_SPHQUAD, CNT_QUAD, CNT_INST, CNT_HITS, CNT_OVERFLOW, CNT_NUM
};

}  // namespace rtamd
