// lbvh.hpp — host interface of the GPU BVH builder (RT_BUILD_LBVH, lbvh.hip).
//
// The reference builds every BLAS once and the TLAS every frame on the host with a random-axis
// median split (src/AS/BLAS.cu:4-117, src/AS/TLAS.cu:4-129, driven from Renderer.cu:123-155 and
// :269-293).  SURVEY §8f rows 1-2 move both builds onto the GPU so that a frame never waits on a
// host build, and so that a 10 M-triangle scene (config C5) can rebuild its BLASes every frame.
//
// One builder instance owns the device workspace of one forest: a set of independent trees
// ("segments") over disjoint, contiguous item ranges.  A build is a fixed sequence of kernels on
// one stream, no host synchronisation:
//   centroid bounds per segment -> 30-bit Morton key per item -> sort within each segment (LDS bitonic for
//   small trees, rocPRIM radix sort for large ones) -> Karras radix-tree hierarchy per segment -> bottom-up box union
//   (arrival counters; one workgroup per tree of <= 2048 items, LDS hand-offs) -> subtrees of <= leaf_cap items collapse into leaves, the surviving
//   interior nodes are compacted (exclusive scan) into the node-pair layout of layout.hpp ->
//   per-segment root {box, ref}.
// Item boxes are exact unions (min/max) of the ε-expanded primitive boxes the reference builds
// (BoundingBox.cuh:24-55), so every node box equals the one a host build over the same leaf sets
// would produce, bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>
#include <vector>

#include "layout.hpp"
#include "../../include/rt.h"

namespace rtamd {

struct LbvhSeg {            // one tree of the forest
    uint32_t item_base;     // first item (= first sorted position) of the segment
    uint32_t count;         // items
    uint32_t slot_base;     // first leaf slot of the tree in its (leaf-ordered) output array
    uint32_t prim_base;     // BLAS: caller primitive index of item item_base
    uint32_t ptype;         // BLAS: rt_primitive_type
    uint32_t node_base;     // first Karras interior node = item_base - segment index
    uint32_t leaf_cap;      // subtrees of <= leaf_cap items become one leaf (<= 4)
    uint32_t blas;          // 1: BLAS-level refs
    // an instance group's merged BLAS (option "group"): its members' entries in the builder's member table
    // ({first caller primitive, caller instance}, ascending), so a leaf slot records the instance it came from
    uint32_t member_base, member_count;
};

// Raw caller primitives in HBM (the builder recomputes boxes, centroids and the leaf-ordered hot /
// cold records from them on every BLAS build).
struct RawPrimsGPU {
    const rt_triangle *tris;
    const float *tri_verts; // the triangles' vertices alone, 9 floats each (extract_tri_verts): what the box / Morton
                            // pass and the leaf-ordered gather read, 36 of the 88 B of an rt_triangle
    const rt_sphere *spheres;
    const rt_parallelogram *quads;
    uint32_t rough_count;   // material slot of metal m = rough_count + m
};

struct PrimOutGPU {         // leaf-ordered arrays written by the BLAS gather
    TriHot *tri_hot; TriCold *tri_cold;
    SphereHot *sph_hot; PrimCold *sph_cold;
    QuadHot *quad_hot; PrimCold *quad_cold;
};

// The per-frame GPU TLAS of a frame with at most SMALL_TLAS_MAX active records, built by one workgroup
// (tlas_small_kernel) after instance_update_kernel computed the records: the LBVH over the active records,
// pairs, quads, slots and the slot-ordered records — one launch instead of ~14.
constexpr uint32_t SMALL_TLAS_MAX = 512;
struct SmallTlasArgs {
    uint32_t n;                                     // records (instances, then groups)
    const InstHot *hot; const InstCold *cold; const float *tbox; const float4 *tcent;   // record order
    NodePair *pairs; TreeRoot *root; TreeRoot *root_wide; NodeQuad *quads; uint32_t *slots;
    InstHot *hot_s; InstCold *cold_s;               // leaf-slot order
    uint32_t *pair_count;
    uint32_t leaf_cap;
};
hipError_t launch_tlas_small(const SmallTlasArgs &a, hipStream_t stream);
// verts[9 k ..] = the vertices of tris[k] for k in [first, first + count)
hipError_t extract_tri_verts(const rt_triangle *tris, float *verts, size_t first, size_t count, hipStream_t stream);

class LbvhBuilder {
public:
    LbvhBuilder() = default;
    LbvhBuilder(const LbvhBuilder &) = delete;
    LbvhBuilder &operator=(const LbvhBuilder &) = delete;
    ~LbvhBuilder() { release(); }

    // Allocates the workspace for `segs` (item ranges must tile [0, n_items) in order).
    hipError_t init(const std::vector<LbvhSeg> &segs, hipStream_t stream);
    void release();

    uint32_t items() const { return n_items_; }
    uint32_t segments() const { return n_segs_; }
    uint32_t max_pairs() const { return n_items_ > n_segs_ ? n_items_ - n_segs_ : 1u; }
    // items in trees of more than 2048 items (the rocPRIM sort, hierarchy_chunk_kernel / hierarchy_top_kernel) and
    // those trees' count: the stage byte model of bench.py's rebuild roofline
    uint32_t large_items() const { uint32_t c = 0; for (const auto &b : big_segs_) c += b.second; return c; }
    uint32_t large_trees() const { return (uint32_t)big_segs_.size(); }
    // device bytes the builder's workspace holds now (sort keys, hierarchy, staged records, rocPRIM scratch, ...):
    // part of rt_scene_info::device_bytes
    size_t workspace_bytes() const;

    // BLAS items: boxes / centroids of the segments' primitives (reference box semantics).
    // stage_hot (BLAS builds without cold records): triangle records staged in item order for the next build()
    hipError_t prep_blas_items(const RawPrimsGPU &raw, hipStream_t stream, bool stage_hot = false);
    // TLAS items: caller-provided boxes (6 floats per item) and centroids (4 floats per item).  An item whose
    // centroid has w != 0 is inactive (an instance group's member while the group is one item, or a broken
    // group): it is kept out of the centroid bounds and sorted behind every active item (its box must be all
    // +inf, which no slab test accepts), so the active items form the tree's first subtree.
    hipError_t set_items(const float *boxes, const float4 *centroids);
    // Member tables of group segments (LbvhSeg::member_base / member_count): {first primitive, instance} pairs.
    hipError_t set_members(const std::vector<uint32_t> &pairs, hipStream_t stream);

    // Builds every segment: pairs written from index 0 of `pairs` (capacity max_pairs()),
    // roots[s] receives segment s's root; `pair_count` (device, may be null) the pairs written.
    // With `raw` / `out` (BLAS builds), the leaf-ordered primitive records are written by the Karras kernel as well
    // (one launch and one pass over the sorted items fewer than a separate gather).
    hipError_t build(NodePair *pairs, TreeRoot *roots, uint32_t *pair_count, hipStream_t stream,
                     const RawPrimsGPU *raw = nullptr, const PrimOutGPU *out = nullptr);

    // After build(): the 4-wide form of every tree (quads[q] = the quad rooted at node pair q, capacity
    // max_pairs()); roots_wide (may be null) receives each tree's root for the quad traversal.
    hipError_t collapse_wide(const NodePair *pairs, const TreeRoot *roots, NodeQuad *quads, TreeRoot *roots_wide,
                             hipStream_t stream);
    // After build(): item index per leaf slot (TLAS: instance index per slot).
    hipError_t gather_items(uint32_t *slots, hipStream_t stream);

    // Stage timing of a BLAS build (rt_api: option "timeline"): with timing on, prep_blas_items / build /
    // collapse_wide record an event at the start and after each stage (STAGES: prep, bounds, morton, sort,
    // hierarchy of the small trees (Karras + gather, bottom-up), hierarchy of the large trees (chunk + top pass +
    // gather), scan, emit + roots, collapse); stage_ms() reads the last build's durations
    // (after the stream has passed them).  Each record between two kernels idles the GPU ~5 us.
    static constexpr int STAGES = 9;
    static const char *const STAGE_NAMES[STAGES];
    hipError_t set_timing(bool on);
    hipError_t stage_ms(float (&ms)[STAGES]) const;

private:
    uint32_t n_items_ = 0, n_segs_ = 0, max_count_ = 0;
    std::vector<std::pair<uint32_t, uint32_t>> big_segs_;   // {item_base, count} of trees sorted by rocPRIM
    LbvhSeg *segs_ = nullptr;
    uint32_t *seg_of_ = nullptr;          // item -> segment
    uint32_t *members_ = nullptr;         // group segments: {first primitive, instance} pairs
    size_t members_n_ = 0;
    uint32_t *item_member_ = nullptr;     // per item: its member instance + 1 (group segments), from members_
    float *box_ = nullptr;                // 6 floats per item (owned or caller's)
    float4 *cent_ = nullptr;
    float *own_box_ = nullptr;
    float4 *own_cent_ = nullptr;
    TriHot *stage_ = nullptr;             // prep_blas_items(stage_hot): TriHot per item, item order
    bool stage_ready_ = false;
    uint32_t *bounds_ = nullptr;          // 6 ordered-uint per segment (centroid bounds)
    uint32_t *k0_ = nullptr, *k1_ = nullptr;           // Morton codes (per item, then sorted within each segment)
    uint32_t *v0_ = nullptr, *v1_ = nullptr;
    uint32_t *child_ = nullptr;           // 2 per interior node: LEAF_BIT | sorted position, or node
    uint32_t *parent_ = nullptr;          // per interior node
    uint32_t *parent_leaf_ = nullptr;     // per sorted position
    uint32_t *range_ = nullptr;           // 2 per interior node: first, last sorted position
    uint32_t *flag_ = nullptr;            // arrival counters
    uint32_t *frontier_ = nullptr;        // trees > LOCAL_MAX items: [count, arrivals at chunk-crossing nodes]
    uint32_t *height_ = nullptr;          // per interior node
    float *nbox_ = nullptr;               // 6 per interior node
    uint32_t *kept_ = nullptr, *pidx_ = nullptr;
    uint32_t *front_ = nullptr;           // collapse_wide frontier of trees too large for LDS
    uint32_t *count_ = nullptr;           // pairs written by the last build (when the caller passed no counter)
    uint32_t *last_count_ = nullptr;      // the counter the last build wrote
    // a forest with a tree of more than this many items is collapsed one pair per thread (collapse_all_kernel)
    static constexpr uint32_t COLLAPSE_ALL_MIN = 65536;
    void *tmp_ = nullptr;
    size_t tmp_bytes_ = 0;
    hipEvent_t stage_ev_[STAGES + 1] = {};
    bool timing_ = false;
    bool last_timed_ = false;             // the last BLAS build recorded its stage events (stage_ms reads them)
    hipError_t mark(int k, hipStream_t stream) { return timing_ ? hipEventRecord(stage_ev_[k], stream) : hipSuccess; }
};

}  // namespace rtamd
