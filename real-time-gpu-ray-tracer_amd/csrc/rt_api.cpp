// rt_api.cpp — the C ABI (include/rt.h): scene lifecycle, BLAS/TLAS builds, HBM upload,
// per-frame instance update with double-buffered TLAS upload, and kernel launches.
//
// Mirrors the reference's host orchestration (src/Global/Renderer.cu, RenderPin.cu,
// RenderGlob.cu) without windowing: commit geometry/materials, configure instances, build the
// acceleration structures, configure the camera, then per frame update instances, rebuild the
// TLAS on the host, upload it on a stream that is ordered against the previous frame's kernel
// through events (Renderer.cu:236-317), and launch the trace kernel.  Errors return rt_status
// with a thread-local message instead of exit() (Global.cu:34-41).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/rt.h"
#include "bvh_build.hpp"
#include "comm.hpp"
#include "comm_wait.hpp"
#include "host_math.hpp"
#include "layout.hpp"
#include "lbvh.hpp"

namespace rtamd {
hipError_t launch_render_exact(const SceneGPU &, const CameraGPU &, const OutputGPU &, bool, unsigned long long *, hipStream_t);
hipError_t launch_render_fast(const SceneGPU &, const CameraGPU &, const OutputGPU &, bool, unsigned long long *, hipStream_t);
hipError_t launch_trace_rays_exact(const SceneGPU &, const float *, uint32_t, rt_hit *, hipStream_t);
hipError_t launch_trace_rays_fast(const SceneGPU &, const float *, uint32_t, rt_hit *, hipStream_t);
hipError_t launch_assemble(const void *, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, void *, hipStream_t);
hipError_t launch_render_persistent_exact(const SceneGPU &, const CameraGPU &, const OutputGPU &, bool, unsigned long long *,
                                          uint32_t *, uint32_t, uint32_t, bool, hipStream_t);
hipError_t launch_render_persistent_fast(const SceneGPU &, const CameraGPU &, const OutputGPU &, bool, unsigned long long *,
                                         uint32_t *, uint32_t, uint32_t, bool, hipStream_t);
hipError_t launch_frame_copy(void *, const void *, size_t, unsigned long long *, uint32_t *, hipStream_t);
hipError_t launch_schedule(uint32_t *, uint32_t *, uint32_t *, uint32_t *, uint32_t, uint32_t, uint32_t, bool, uint32_t,
                           uint32_t, uint32_t, void *, const void *, size_t, unsigned long long *, hipStream_t);
uint32_t persistent_blocks_per_cu_exact(uint32_t wide, bool raw);
hipError_t launch_instance_slot_order(const uint32_t *, const InstHot *, const InstCold *, uint32_t, InstHot *, InstCold *,
                                      hipStream_t);
hipError_t launch_instance_update(const InstDelta *, uint32_t, InstParams *, uint32_t, InstHot *, InstCold *, float *, float4 *,
                                  const uint32_t *, const TreeRoot *, const uint32_t *, bool, hipStream_t);
uint32_t persistent_blocks_per_cu_fast(uint32_t wide, bool raw);
// option "fast_math": the FAST kernels compiled with hardware reciprocals and FMA contraction (trace_fastmath.o)
hipError_t launch_render_fastmath(const SceneGPU &, const CameraGPU &, const OutputGPU &, bool, unsigned long long *, hipStream_t);
hipError_t launch_trace_rays_fastmath(const SceneGPU &, const float *, uint32_t, rt_hit *, hipStream_t);
hipError_t launch_render_persistent_fastmath(const SceneGPU &, const CameraGPU &, const OutputGPU &, bool, unsigned long long *,
                                             uint32_t *, uint32_t, uint32_t, bool, hipStream_t);
uint32_t persistent_blocks_per_cu_fastmath(uint32_t wide, bool raw);
hipError_t launch_box_test_exact(const float *, const float *, const float *, uint32_t, uint32_t, uint8_t *, float *, hipStream_t);
hipError_t launch_box_test_fast(const float *, const float *, const float *, uint32_t, uint32_t, uint8_t *, float *, hipStream_t);
}  // namespace rtamd

using namespace rtamd;

namespace {
thread_local std::string g_error;
}  // namespace

void rtamd_set_error(const std::string &msg) { g_error = msg; }   // shared with vtk_reader.cpp

namespace {

rt_status fail(rt_status s, const std::string &msg) {
    g_error = msg;
    return s;
}

#define RT_TRY(expr)                                                                               \
    do {                                                                                           \
        const rt_status st_ = (expr);                                                              \
        if (st_ != RT_OK) return st_;                                                              \
    } while (0)

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return fail(e_ == hipErrorOutOfMemory ? RT_ERR_OUT_OF_MEMORY : RT_ERR_DEVICE,          \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                       \
    } while (0)

constexpr uint32_t BLAS_LEAF_CAP = 4;   // BLAS.cuh:17
constexpr uint32_t TLAS_LEAF_CAP = 2;   // TLAS.cuh:22
constexpr uint32_t SAH_LEAF_CAP = 4;    // RT_BUILD_SAH: <= 4 items per leaf (2-bit count in a leaf ref)
constexpr uint32_t LBVH_BLAS_LEAF_CAP = 4;
// GPU TLAS leaves hold up to fixed setting "tlas_leaf" (an option until round 5) instances (default 1, as the SAH TLAS: a leaf's
// instances are entered without their own box test; 2 = the reference's TLAS leaf size, TLAS.cuh:22)

struct InstState {
    uint32_t ptype, pindex, pcount, blas;
    hm::Box box;
    hm::V3 centroid;
    hm::Mat fwd, inv, nrm;
    hm::Box tbox;
    hm::V3 tcentroid;
    rt_xform x;
};

struct BlasHost {
    uint32_t type;
    Tree tree;
    FlatTree flat;
    FlatWide wide;                 // quad form (option "wide"; host-built modes)
    uint32_t pair_base, slot_base;
    // a group's merged BLAS (option "group"): the members' triangle ranges {first, count, instance}
    std::vector<std::array<uint32_t, 3>> members;
};

// Option "group" (RT_BUILD_SAH, host-built TLAS): triangle instances whose transforms are bit-identical
// (the reference's VTK particles all carry one fixed transform, VTKReader.cu:204-215) share one instance
// space, so one SAH BLAS over all their triangles replaces their overlapping instance boxes in the TLAS.
// A frame uses the group while every member still has the group's transform (and its triangles and
// bounds were not replaced since the build); otherwise that frame's TLAS takes the members one by one.
struct InstGroup {
    InstState st;                  // the group as one instance: the shared transform, the union of the boxes
    std::vector<uint32_t> members;
    bool valid = true;
};

template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    void release() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
};

// rt_scene_attach_comm: this scene is rank `rank` of a `world`-rank frame.  One communicator
// per overlap lane at attach time (split from the first), so the lanes' gathers on different streams do not
// share one; lane q uses comm[q % ncomm] if "overlap" is raised after the attach (every rank issues the same
// lane sequence, so a shared communicator still sees its operations in one order on every rank).
struct CommState {
    static constexpr int NLANE = 8;        // = rt_scene::NLANE
    int rank = 0, world = 1;
    int ncomm = 1;
    uint32_t timeout_ms = 0;               // rt_comm_set_timeout: 0 = no deadline (async errors still polled)
    uint32_t tile_w = 64, tile_h = 64;
    ncclComm_t comm[NLANE] = {};
    size_t slab_bytes = 0;                 // one rank's slab (largest tile count), RGBA8
    DevBuf<uint8_t> slab[NLANE];           // ranks > 0: this rank's traced tiles
    DevBuf<uint8_t> gathered[NLANE];       // rank 0: world slabs; its own tiles are traced into slab 0
};

size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

}  // namespace

struct rt_scene {
    int device = 0;
    // caller data (copied, Renderer.cu:31-39)
    std::vector<rt_sphere> spheres;
    std::vector<rt_parallelogram> quads;
    std::vector<rt_triangle> tris;
    std::vector<rt_rough> roughs;
    std::vector<rt_metal> metals;
    std::vector<rt_instance_desc> inst_desc;
    rt_update_fn update = nullptr;
    void *update_user = nullptr;

    std::vector<InstState> inst;
    std::vector<BlasHost> blas;
    size_t blas_own = 0;            // per-instance BLASes; the groups' merged BLASes follow them in `blas`
    std::vector<InstGroup> groups;  // option "group": TLAS item n + g is group g
    std::vector<uint32_t> group_of; // per instance: its group + 1 (0: none)
    bool group_inst = true;         // option "group" (set before the build)
    bool lds_blas = true;           // fixed setting "lds_blas" (an option until round 5): with "lds_scene" 2, a group BLAS's top levels in LDS
    // frame blocks (= NLANE, below).  Round 6 measured 12 and 16 lanes: 1/8 shares equal or slower (C2 0.0384-0.0388
    // ms/frame at 8, 0.0394-0.0420 at 12, 0.0385-0.0392 at 16; C4 0.0465-0.0472 at 8, 0.0483-0.0499 at 16), the whole
    // frame equal at 6 and 8 (profiles/r06/lanes/)
    static constexpr int NBLOCK = 8;
    uint32_t frame_items[NBLOCK] = {};   // per frame block: TLAS items (= instance records when staged by slot)
    Tree tlas;
    FlatTree tlas_flat;
    FlatWide tlas_wide;
    uint64_t build_seed = 0;
    rt_build_mode build_mode = RT_BUILD_COMPAT_MEDIAN;
    bool built = false;
    uint64_t frame = 0;

    // HBM: static scene data
    DevBuf<NodePair> blas_pairs;
    DevBuf<NodeQuad> blas_quads;    // option "wide"
    bool wide = true;               // FAST persistent kernel traverses the quad trees (host-built modes)
    bool exact_decisions = false;   // option "exact_decisions": GPU-built trees take the exact-decision traversal (mode 3)
    uint32_t lds_scene = 2;         // quad-tree kernel: 1 = TLAS quads (+ instance hot records) in LDS when they
                                    // fit, 2 = also sphere / parallelogram records and instance cold records
    // option "grid_pct": the persistent grid as a percentage of the resident capacity; 0 = auto: 50 when
    // another lane's launch is still in flight ("overlap"), so two lanes' launches are resident side by
    // side instead of the next one filling only the slots the previous one's tail frees (C2, 3 lanes:
    // 0.252 -> 0.229 ms/frame; a C2 1/8 share 0.115 -> 0.084; C3 1.64 -> 1.59,
    // profiles/r02_sweep_grid2.jsonl), else 100 (a frame alone on the GPU takes all of it)
    uint32_t grid_pct = 0;
    static constexpr uint64_t BIG_LAUNCH_PATHS = 16ull << 20;
    // option "cold_records" (RT_BUILD_LBVH, set before rt_scene_build; default 0): 1 = the BLAS builds write TriCold
    // records (normals, material, caller index) as the host builders do; 0 = they write TriHot only, with the caller's
    // triangle index and group member in its pads, and a hit reads normals and material from the caller's triangle
    // (SceneGPU::raw_tris) — a C5 rebuild's leaf-ordered gather then moves about half the bytes
    // -1 (auto, default): 1 when the BLASes are built once (option "rebuild" 0 at rt_scene_build: a hit's normals and
    // material are then one dependent HBM round trip nearer — C5 static 4.97 -> 4.80 ms/frame, C2-LBVH -1 %), 0 when
    // they are rebuilt every frame (the rebuild's gather moves half the bytes: C5 8.36 against 8.52;
    // profiles/r05/cold_records/)
    int cold_records = -1;
    bool cold_eff = false;          // the build's choice (rt_scene_build)
    bool raw_shading() const { return build_mode == RT_BUILD_LBVH && !cold_eff; }
    DevBuf<TriHot> tri_hot;
    DevBuf<TriCold> tri_cold;
    DevBuf<SphereHot> sph_hot;
    DevBuf<PrimCold> sph_cold;
    DevBuf<QuadHot> quad_hot;
    DevBuf<PrimCold> quad_cold;
    DevBuf<float> materials;
    uint64_t blas_pair_count = 0, blas_leaf_count = 0;

    // per-frame data, double-buffered:
    //   [tlas root | tlas pairs | tlas slots | inst hot | inst cold | tlas item boxes | tlas item centroids]
    // (the root and the item arrays are used by GPU-built TLASes only)
    size_t frame_block = 0, off_root = 0, off_pairs = 0, off_slots = 0, off_hot = 0, off_cold = 0, off_tbox = 0,
           off_tcent = 0, off_root_wide = 0, off_quads = 0, off_delta = 0, off_hot_s = 0, off_cold_s = 0;
    // frame blocks cycle through NLANE buffers, so "overlap" lanes never wait on each other's block
    static constexpr int NLANE = 8;
    static_assert(NLANE == NBLOCK, "one frame block per lane");
    // GPU-built frames: per-instance parameters resident in HBM (instances.hip), one copy per frame block
    // (block b's at inst_params.p + b * records), so frames of different lanes update their records
    // concurrently; the host stages a delta (InstDelta at off_delta) only for the records whose transform
    // or local box changed since block b was last written: inst_dirty bit b (ALL_BLOCKS: every block)
    DevBuf<InstParams> inst_params;
    std::vector<uint16_t> inst_dirty;
    static constexpr uint16_t ALL_BLOCKS = 0xFFFF;
    static_assert(NLANE <= 16, "inst_dirty holds one bit per frame block");
    hipStream_t chain_stream[NLANE] = {};         // GPU-built frame b's records / TLAS were built on this stream
    hipEvent_t ev_blas_built = nullptr;           // the last GPU BLAS build on the scene stream finished
    hipEvent_t ev_caller = nullptr;               // rt_render with device outputs and no stream: the null stream's
                                                  // work before the call (the trace writes the caller's buffers after it)
    uint64_t blas_build_seq = 0;                  // BLAS builds recorded on ev_blas_built so far
    uint64_t blas_build_done = 0;                 // ... of which the host has seen the last one complete
    // pinned host staging, cycled independently of the frame blocks and twice as deep: a frame's staging is
    // reusable once its upload ran, which rt_render can only tell by the trace's completion event (a record
    // right after the copy kernel would idle the GPU ~5 us) — with one staging per block, the host waited for
    // frame k-8's whole trace before it could stage frame k (8 lanes of 1/8-frame shares: 0.12 ms lane gaps)
    // option "stage_depth" (default 2 x NLANE): buffers in the cycle, allocated on first use
    static constexpr int NSTAGE = 64;
    int stage_depth = 16;
    uint8_t *staging[NSTAGE] = {};
    uint8_t *staging_dev[NSTAGE] = {};            // the same, as device-visible pointers
    hipEvent_t r_staged[NSTAGE] = {};             // staging[i] no longer read (null: never used)
    int stage_next = 0;
    int pending_copy = -1, pending_stage = -1;    // rt_render: block (and its staging) whose upload the next launch performs
    uint8_t *frame_dev[NLANE] = {};               // HBM
    hipEvent_t ev_copied[NLANE] = {};             // frame block b uploaded / built
    hipEvent_t ev_used[NLANE] = {};               // last kernel reading frame_dev[b] finished
    // What the waits below use: the event last recorded for each purpose.  A trace launch records one event
    // after it (its ring_stop timing event, or one event after a multi-GPU gather) and points every purpose
    // it completes at that event — each event record between two kernels of a stream costs ~5 us of GPU
    // idle time (profiles/r02_gaps.txt), and a launch completed four purposes with four records.
    hipEvent_t r_copied[NLANE] = {}, r_used[NLANE] = {}, r_lane[NLANE] = {};
    hipEvent_t r_done = nullptr;
    int active = -1;

    hipStream_t stream = nullptr;
    // per-frame kernel timing ring for pipelined frames (rt_scene_collect)
    static constexpr uint32_t RING = 256;
    hipEvent_t ring_start[RING] = {}, ring_stop[RING] = {};
    hipEvent_t ring_post[RING] = {};     // multi-GPU frames: the launch's completion event after its gather
    uint32_t ring_head = 0, ring_pending = 0;
    hipStream_t last_stream = nullptr;
    // persistent megakernel: work-queue head, grid size (#CUs x resident blocks), refill threshold
    // option "overlap" = L lanes: consecutive frames cycle through L lanes (queue heads, unit costs,
    // schedule), so frame k+1's persistent launch fills the CUs frame k's tail leaves idle when the caller
    // cycles L streams; with L <= 1 every frame uses lane 0 and launches of one scene are serialised.
    uint32_t *queue[NLANE] = {};
    bool overlap = false;
    uint32_t blas_leaf = SAH_LEAF_CAP;   // fixed setting "blas_leaf" (an option until round 5): RT_BUILD_SAH BLAS leaf size (1..4), next rt_scene_build
    uint32_t tlas_leaf = 1;   // fixed setting "tlas_leaf" (an option until round 5): RT_BUILD_SAH per-frame SAH TLAS leaf size (1..4; 1 measured best)
    uint32_t tlas_median_leaf = 0;   // fixed setting "tlas_median_leaf" (an option until round 5): RT_BUILD_SAH median TLAS leaf size (0 = the reference's 2)
    bool tlas_sah = true;     // option "tlas_sah": RT_BUILD_SAH builds its per-frame TLAS with SAH (0: the median split)
    bool inst_by_slot = true;       // fixed setting "inst_by_slot" (an option until round 5): host-built TLAS stages instance records in slot order
    bool block_by_slot[NLANE] = {};  // per frame block: staged in slot order
    uint32_t lanes = 1;
    // fixed setting "reserve" (an option until round 5): with overlapped lanes the persistent grid leaves this many workgroup slots free (two
    // per XCD at 16), so the next lanes' schedule / upload kernels and GPU TLAS builds run beside a launch
    // that holds the rest of the GPU instead of waiting for its drain (C2, 3 lanes: 16 -> 0.260-0.261,
    // 8 -> 0.261-0.265, 0 -> 0.268-0.272 ms/frame; profiles/r02_sweep_lanes.jsonl)
    uint32_t reserve = 16;
    uint32_t lane = 0;              // lane of the next rt_render (overlap)
    int last_lane = 0;              // lane of the last rt_render
    // "overlap" frames rendered without a caller stream (opts.stream NULL) run on lane streams the scene owns; with
    // option "overlap" -1 (overlap_auto) the scene also picks the lane count and the staging depth per frame kind
    // (auto_lanes: the settings bench.py measured best), so a drop-in caller passes no streams at all
    hipStream_t lane_st[NLANE] = {};
    bool overlap_auto = false;
    // fixed setting "leaf_early" (an option until round 5) (OutputGPU::leaf_early): -1 = auto, 0 for paths of <= 2 segments (depth x samples; C2, C4),
    // else LEAF_EARLY_AUTO (C3 1.54 -> 1.25, C5 5.79 -> 4.97 ms/frame; C2 0.181 -> 0.185 with it,
    // profiles/r05/leaf_early/)
    int leaf_early = -1;
    static constexpr uint32_t LEAF_EARLY_AUTO = 12;
    // option "lane_priority": the scene's own lane streams at the device's highest priority (default 1): HIP gives them
    // hardware queues of their own, so 4 lanes run side by side at the default GPU_MAX_HW_QUEUES (4) — C2 0.256 ->
    // 0.180 ms/frame, C3 2.15 -> 1.54, a 1/8 share 0.064 -> 0.046 — as at 12 queues (profiles/r05/lanes/)
    bool lane_priority = true;
    bool stage_depth_set = false;   // option "stage_depth" given explicitly (auto lanes leave it alone)
    hipEvent_t ev_lane_done[NLANE] = {};   // last trace launch of each lane finished
    uint32_t cus = 0;
    // fixed setting "threshold" (an option until round 5) (lanes waiting before a wave leaves traversal to shade and refill); 0 = auto: 64 when
    // a pixel's path has at most two segments (depth x samples <= 2: the wave then shades and refills all its
    // lanes at once), else 40 (C2 0.194 -> 0.184 ms/frame, serialised 0.35 -> 0.33 ms; C3 at 64 would lose
    // 23 %, 40 ties 32; profiles/r02_sweep_thr2.jsonl)
    uint32_t threshold = 0;
    // option "fast_math": FAST frames with hardware reciprocal / rsq and FMA contraction instead of the reference's
    // correctly rounded arithmetic (C2 -7 %, C3 -9 % per pipelined frame; 0.008-0.09 % of pixels then differ from the
    // oracle even on its own trees); default 0: bit-identical to the oracle on the reference's trees
    bool fast_math = false;
    double update_wait_ms = 0.0;    // last frame_update: time blocked on ev_copied (GPU progress)
    bool use_persistent = true;
    uint32_t queue_parts = 8;       // one band per XCD (measured with "reorder": 8 beat 4, 2 and 1 on C2)
    uint32_t grab = 64;             // pixels per queue claim
    // fixed setting "merge" (an option until round 5): two adjacent units below this cost level share one claim item (128 pixels): 6 (sky, about
    // 4 steps per pixel) measured C2 0.203 -> 0.199 ms/frame; 8 or 10 (also the ground) put 128-pixel items at
    // the end of the order and lengthen the tail (profiles/r02_sweep_merge.jsonl)
    uint32_t merge = 6;
    uint32_t supertile = 16;        // band walk order: st x st-unit supertiles (measured: 16 beats rows, 8 and 32)
    uint32_t max_blas_height = 0;
    bool timeline_on = false;
    bool costmap_on = false;
    // option "reorder" (schedule.hip): longest-first claim order from the previous launch's unit costs
    bool reorder = true;
    // heavy-unit pieces: class level for halves | quarters << 8 (0xFF = never); measured (C2 / C3 / C4
    // shares, profiles/r02_sweep_period*.jsonl): quarters from level 12 and no halves
    uint32_t split = 12u | 12u << 8;
    DevBuf<uint32_t> unit_cost[NLANE], unit_order[NLANE];
    uint32_t sched_sig[NLANE][7] = {};  // launch layout the recorded costs belong to
    // fixed setting "reorder_period" (an option until round 5) K: a lane records unit costs on one launch in K and rebuilds its order on
    // the next; the launches between reuse the order (the heaviest regions move little between frames)
    uint32_t reorder_period = 8;        // measured: 8 (C2 0.242 ms/step) beats 1 (0.265) with 3 lanes
    uint32_t sched_phase[NLANE] = {};
    bool order_ok[NLANE] = {};
    bool sched_valid[NLANE] = {};
    DevBuf<uint32_t> costmap;
    size_t costmap_pixels = 0;
    DevBuf<unsigned long long> timeline;
    uint32_t timeline_waves = 0;    // waves of the last launch that recorded a timeline
    // device counters, one CNT_NUM block per lane: a launch only adds to its own lane's block, so resetting
    // or reading it never races with another lane's launch still in flight (rt_scene_collect sums the lanes)
    unsigned long long *counters = nullptr;       // HBM NLANE x CNT_NUM
    unsigned long long *counters_host = nullptr;  // pinned NLANE x CNT_NUM
    // a frame without RT_RENDER_KEEP_COUNTERS starts a new epoch; a lane's block is cleared by the first launch
    // of that lane in the epoch (no waiting on the other lanes), and rt_scene_collect sums only blocks of the
    // current epoch
    uint64_t cnt_epoch = 0;
    uint64_t lane_epoch[NLANE] = {};

    // camera
    bool cam_ok = false;
    CameraGPU cam{};
    uint32_t width = 0, height = 0;

    // scene-owned outputs
    DevBuf<uint8_t> out_rgba;
    DevBuf<float> out_rgb;

    // RT_BUILD_LBVH: GPU builders and the raw caller primitives they read
    LbvhBuilder *blas_builder = nullptr, *tlas_builder = nullptr;
    DevBuf<rt_triangle> raw_tris;
    DevBuf<float> raw_verts;            // 9 floats per triangle (extract_tri_verts): the builder's reads
    // rt_scene_update_triangles: the new triangles are staged in pinned memory and copied on the scene stream,
    // behind the BLAS builds that read raw_tris (the only readers) and without waiting for any trace
    rt_triangle *raw_stage = nullptr;
    size_t raw_stage_cap = 0;
    hipEvent_t ev_raw_staged = nullptr;            // the last staged copy finished (raw_stage reusable)
    DevBuf<rt_sphere> raw_sph;
    DevBuf<rt_parallelogram> raw_quad;
    DevBuf<TreeRoot> blas_roots;        // per segment the builder holds (seg_of_blas)
    DevBuf<uint32_t> inst_blas;         // instance record (instances, then groups) -> segment
    // RT_BUILD_LBVH + option "group": every unique BLAS's segment (index = BLAS index; the groups' merged BLASes
    // follow the own ones), BLAS -> segment the builder currently holds (NONE: not built), and per group whether
    // it was intact at that setup.  A group's BLAS and its members' BLASes share one leaf-slot range, and only
    // one of them is built: the group's while it is intact, the members' once it breaks (lbvh_segments)
    std::vector<LbvhSeg> lbvh_segs;
    std::vector<uint32_t> seg_of_blas;
    std::vector<uint8_t> lbvh_intact;
    DevBuf<uint32_t> gpu_counts;        // [0] BLAS pairs written, [1] unused, [2 + b] TLAS pairs of frame block b
    bool rebuild_blas = false;          // option "rebuild": rebuild every BLAS each frame
    bool blas_dirty = false;            // rt_scene_update_triangles since the last BLAS build
    // RT_BUILD_LBVH rebuilds (option "blas_double", default on): a rebuild writes a spare BLAS set and swaps it
    // in, so frame k+1's rebuild runs while frame k's trace still reads the other set (C5: the rebuild no
    // longer waits for every lane's trace).  ev_blas_lane[q]: lane q's last trace of the current set.
    // Option "blas_sets" = 3 (default; 2 = one spare): two spare sets in rotation, so frame k+1's rebuild waits only
    // for frame k-2's trace and three traces stay in flight beside it (spare[0] = the set read longest ago, the next
    // one written; C5 with the rebuild 11.18 -> 10.85 ms/frame, profiles/r04/c5_rebuild/).
    struct BlasSet {
        DevBuf<NodePair> pairs; DevBuf<NodeQuad> quads; DevBuf<TreeRoot> roots;
        DevBuf<TriHot> tri_hot; DevBuf<TriCold> tri_cold; DevBuf<SphereHot> sph_hot; DevBuf<PrimCold> sph_cold;
        DevBuf<QuadHot> quad_hot; DevBuf<PrimCold> quad_cold;
        hipEvent_t ev_lane[NLANE] = {};
        void release() {
            pairs.release(); quads.release(); roots.release(); tri_hot.release(); tri_cold.release();
            sph_hot.release(); sph_cold.release(); quad_hot.release(); quad_cold.release();
        }
    };
    static constexpr uint32_t MAX_BLAS_SETS = 8;
    BlasSet spare[MAX_BLAS_SETS - 1];   // spare[0]: the set read longest ago (written next) .. spare[sets - 2]: the newest
    uint32_t blas_sets = 3;
    hipEvent_t ev_blas_lane[NLANE] = {};
    bool blas_double = true;
    uint64_t blas_builds = 0;
    hipEvent_t ev_render_done = nullptr;   // last trace launch finished (BLAS rebuilds wait on it)
    bool gpu_tlas_sah = false;          // option "gpu_tlas" (set before the build): RT_BUILD_SAH BLASes, per-frame TLAS on the GPU
    // option "tlas_small": GPU-built frames with at most SMALL_TLAS_MAX records in the TLAS build it in one workgroup
    // (lbvh.hip tlas_small_kernel) instead of the ~17-launch chain
    bool tlas_small = true;
    DevBuf<uint32_t> blas_wide_refs;    // host-built BLASes under a GPU TLAS: quad root ref per BLAS
    // instance records + TLAS built by kernels each frame: RT_BUILD_LBVH, or RT_BUILD_SAH with "gpu_tlas"
    bool gpu_tlas() const { return build_mode == RT_BUILD_LBVH || (gpu_tlas_sah && build_mode == RT_BUILD_SAH); }
    // quads of two binary levels visited in the reference's order (layout.hpp NodeQuad): the reference's own trees and
    // GPU-built ones; host SAH trees keep the greedy collapse visited by entry t
    bool quad_halves() const { return build_mode != RT_BUILD_SAH; }

    CommState *comm = nullptr;             // multi-GPU frame (rt_scene_attach_comm)
    uint32_t comm_timeout_ms = 0;          // rt_comm_set_timeout (kept across attach / detach)
    void release_comm() {
        if (!comm) return;
        for (int q = 0; q < CommState::NLANE; q++) {
            if (comm->comm[q]) (void)rccl().CommDestroy(comm->comm[q]);
            comm->slab[q].release();
            comm->gathered[q].release();
        }
        delete comm;
        comm = nullptr;
    }
    // A failed frame (peer error or deadline): abort every communicator so the gather kernels in flight
    // return, and drop the communicator state.  The slabs are not freed: kernels of the aborted frames may
    // still reference them, and hipFree would wait for those (a bounded leak instead of a hang).
    void abort_comm() {
        if (!comm) return;
        for (int q = 0; q < CommState::NLANE; q++)
            if (comm->comm[q]) (void)rccl().CommAbort(comm->comm[q]);
        delete comm;
        comm = nullptr;
        for (int q = 0; q < NLANE; q++) r_lane[q] = ev_lane_done[q];
        r_done = ev_render_done;                   // never recorded after the build's drain: waits on it are no-ops
        for (int b = 0; b < NLANE; b++) { r_copied[b] = ev_copied[b]; r_used[b] = ev_used[b]; }
        for (hipEvent_t &e : r_staged) e = nullptr;     // drained: every staging buffer is free
    }

    ~rt_scene() {
        (void)hipSetDevice(device);
        if (comm) {                            // a peer may be gone: bounded waits, abort instead of hanging
            bool ok = true;
            const auto q_ev = [](hipEvent_t e) { const hipError_t r = hipEventQuery(e); return r == hipSuccess ? 1 : (r == hipErrorNotReady ? 0 : -1); };
            for (int q = 0; q < NLANE && ok; q++)
                if (r_lane[q]) ok = poll_wait([&] { return q_ev(r_lane[q]); }, [] { return 0; },
                                              comm->timeout_ms ? comm->timeout_ms : 10000u) == WaitResult::done;
            if (!ok) abort_comm();
        }
        if (stream) (void)hipStreamSynchronize(stream);
        for (int q = 0; q < NLANE; q++)          // launches still running on caller streams
            if (r_lane[q]) (void)hipEventSynchronize(r_lane[q]);
        if (r_done) (void)hipEventSynchronize(r_done);
        release_comm();
        blas_pairs.release(); blas_quads.release(); tri_hot.release(); tri_cold.release(); sph_hot.release(); sph_cold.release();
        quad_hot.release(); quad_cold.release(); materials.release(); out_rgba.release(); out_rgb.release();
        timeline.release(); costmap.release();
        for (int q = 0; q < NLANE; q++) { unit_cost[q].release(); unit_order[q].release(); }
        delete blas_builder; delete tlas_builder;
        raw_tris.release(); raw_verts.release(); raw_sph.release(); raw_quad.release(); blas_roots.release(); inst_blas.release();
        blas_wide_refs.release();
        gpu_counts.release(); inst_params.release();
        for (BlasSet &sp : spare) sp.release();
        for (int q = 0; q < NLANE; q++) {
            if (ev_blas_lane[q]) (void)hipEventDestroy(ev_blas_lane[q]);
            for (BlasSet &sp : spare)
                if (sp.ev_lane[q]) (void)hipEventDestroy(sp.ev_lane[q]);
        }
        if (ev_render_done) (void)hipEventDestroy(ev_render_done);
        if (ev_caller) (void)hipEventDestroy(ev_caller);
        if (ev_blas_built) (void)hipEventDestroy(ev_blas_built);
        if (ev_raw_staged) (void)hipEventDestroy(ev_raw_staged);
        if (raw_stage) (void)hipHostFree(raw_stage);
        for (int i = 0; i < NSTAGE; i++)
            if (staging[i]) (void)hipHostFree(staging[i]);
        for (int b = 0; b < NLANE; b++) {
            if (frame_dev[b]) (void)hipFree(frame_dev[b]);
            if (ev_copied[b]) (void)hipEventDestroy(ev_copied[b]);
            if (ev_used[b]) (void)hipEventDestroy(ev_used[b]);
        }
        if (counters) (void)hipFree(counters);
        for (int q = 0; q < NLANE; q++) {
            if (queue[q]) (void)hipFree(queue[q]);
            if (ev_lane_done[q]) (void)hipEventDestroy(ev_lane_done[q]);
        }
        if (counters_host) (void)hipHostFree(counters_host);
        for (uint32_t i = 0; i < RING; i++) {
            if (ring_start[i]) (void)hipEventDestroy(ring_start[i]);
            if (ring_stop[i]) (void)hipEventDestroy(ring_stop[i]);
            if (ring_post[i]) (void)hipEventDestroy(ring_post[i]);
        }
        if (stream) (void)hipStreamDestroy(stream);
        for (hipStream_t &l : lane_st)
            if (l) (void)hipStreamDestroy(l);
    }
};

namespace {

// Instance::updateTransformArguments (src/AS/Instance.cu:4-17)
hm::V3 cos3(const rt_xform &x) {
    hm::V3 c, s;
    hm::rotate_cos_sin(x.rotate_deg.x, c.x, s.x);
    hm::rotate_cos_sin(x.rotate_deg.y, c.y, s.y);
    hm::rotate_cos_sin(x.rotate_deg.z, c.z, s.z);
    return c;
}
hm::V3 sin3(const rt_xform &x) {
    hm::V3 c, s;
    hm::rotate_cos_sin(x.rotate_deg.x, c.x, s.x);
    hm::rotate_cos_sin(x.rotate_deg.y, c.y, s.y);
    hm::rotate_cos_sin(x.rotate_deg.z, c.z, s.z);
    return s;
}
void instance_update(InstState &in, const rt_xform &x) {
    in.x = x;
    in.fwd = hm::instance_matrix(hm::of(x.shift), cos3(x), sin3(x), hm::of(x.scale));
    in.inv = hm::inverse(in.fwd);
    in.nrm = hm::transpose(in.inv);
    in.tbox = hm::transform_box(in.box, in.fwd);
    in.tcentroid = hm::apply_point(in.fwd, in.centroid);
}

hm::Box prim_box(const rt_scene *s, uint32_t type, uint32_t i) {
    if (type == RT_PRIM_SPHERE) return hm::sphere_box(s->spheres[i]);
    if (type == RT_PRIM_PARALLELOGRAM) return hm::quad_box(s->quads[i]);
    return hm::tri_box(s->tris[i]);
}
hm::V3 prim_centroid(const rt_scene *s, uint32_t type, uint32_t i) {
    if (type == RT_PRIM_SPHERE) return hm::sphere_centroid(s->spheres[i]);
    if (type == RT_PRIM_PARALLELOGRAM) return hm::quad_centroid(s->quads[i]);
    return hm::tri_centroid(s->tris[i]);
}
size_t prim_len(const rt_scene *s, uint32_t type) {
    return type == RT_PRIM_SPHERE ? s->spheres.size() : (type == RT_PRIM_PARALLELOGRAM ? s->quads.size() : s->tris.size());
}

uint32_t material_slot(const rt_scene *s, uint32_t type, uint32_t index, bool &ok) {
    if (type == RT_MAT_ROUGH && index < s->roughs.size()) return index;
    if (type == RT_MAT_METAL && index < s->metals.size()) return (uint32_t)(s->roughs.size() + index) | MAT_METAL_BIT;
    ok = false;
    return 0;
}

void store_rows(float *dst, const hm::Mat &m) {   // rows 1..3, cols 1..4
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 4; j++) dst[4 * i + j] = m.d[i + 1][j + 1];
}

rt_status gpu_build_blas(rt_scene *s);
bool record_inactive(const rt_scene *s, size_t i);
const InstState &record_state(const rt_scene *s, size_t i);
rt_status lbvh_sync_groups(rt_scene *s);

// Wait for a stream / an event of the scene.  With a communicator attached the wait polls (comm_wait.hpp):
// an asynchronous RCCL error or the rt_comm_set_timeout deadline aborts the communicators and fails with
// RT_ERR_DEVICE instead of blocking on a peer that will never send.
int query_result(hipError_t r) { return r == hipSuccess ? 1 : (r == hipErrorNotReady ? 0 : -1); }
rt_status comm_poll(rt_scene *s, hipStream_t st, hipEvent_t ev) {
    CommState *cm = s->comm;
    const Rccl &R = rccl();
    int code = 0;
    const WaitResult w = poll_wait(
        [&] { return st ? query_result(hipStreamQuery(st)) : query_result(hipEventQuery(ev)); },
        [&] {
            return first_async_error(cm->ncomm, [&](int q, int *st) {
                ncclResult_t a = ncclSuccess;
                const ncclResult_t r = cm->comm[q] ? R.CommGetAsyncError(cm->comm[q], &a) : ncclSuccess;
                *st = (int)a;
                return (int)r;
            });
        },
        cm->timeout_ms, &code);
    if (w == WaitResult::done) return RT_OK;
    if (w == WaitResult::failed) {
        const hipError_t e = st ? hipStreamSynchronize(st) : hipEventSynchronize(ev);
        return fail(RT_ERR_DEVICE, std::string("multi-GPU frame: ") + hipGetErrorString(e));
    }
    const std::string why = w == WaitResult::timeout
        ? "multi-GPU frame not complete after " + std::to_string(cm->timeout_ms) + " ms (a peer stopped?)"
        : std::string("RCCL asynchronous error: ") + R.GetErrorString((ncclResult_t)code);
    s->abort_comm();
    return fail(RT_ERR_DEVICE, why + "; communicators aborted, scene detached");
}
rt_status wait_stream(rt_scene *s, hipStream_t st) {
    if (s->comm) return comm_poll(s, st, nullptr);
    const hipError_t e = hipStreamSynchronize(st);
    return e == hipSuccess ? RT_OK : fail(RT_ERR_DEVICE, std::string("hipStreamSynchronize: ") + hipGetErrorString(e));
}
rt_status wait_event(rt_scene *s, hipEvent_t ev) {
    if (s->comm) return comm_poll(s, nullptr, ev);
    const hipError_t e = hipEventSynchronize(ev);
    return e == hipSuccess ? RT_OK : fail(RT_ERR_DEVICE, std::string("hipEventSynchronize: ") + hipGetErrorString(e));
}
// Wait for every enqueued launch of the scene: its own stream, the last caller stream, every lane.
rt_status drain(rt_scene *s) {
    if (s->last_stream) RT_TRY(wait_stream(s, s->last_stream));
    if (s->stream) RT_TRY(wait_stream(s, s->stream));
    for (int q = 0; q < rt_scene::NLANE; q++)
        if (s->r_lane[q]) RT_TRY(wait_event(s, s->r_lane[q]));
    return RT_OK;
}

// Order stream `st` after the last GPU BLAS build (ev_blas_built, recorded on the scene stream).  A build that has
// already finished needs no wait (a host query, ~1 us): anything enqueued now runs after it.
rt_status wait_blas_built(rt_scene *s, hipStream_t st) {
    if (s->blas_build_done == s->blas_build_seq) return RT_OK;
    const hipError_t q = hipEventQuery(s->ev_blas_built);
    if (q == hipSuccess) {
        s->blas_build_done = s->blas_build_seq;
        return RT_OK;
    }
    if (q != hipErrorNotReady) return fail(RT_ERR_DEVICE, std::string("hipEventQuery: ") + hipGetErrorString(q));
    HIP_TRY(hipStreamWaitEvent(st, s->ev_blas_built, 0));
    return RT_OK;
}

// Every enqueued launch of the scene and the build of the current frame block (GPU-built frames build it on the
// lane stream of the frame that staged it): the scene's own streams and events only, with the communicator's
// bounded polls when one is attached (never a device-wide synchronisation).
rt_status wait_frame_block(rt_scene *s) {
    RT_TRY(drain(s));
    if (s->active >= 0 && s->r_copied[s->active]) RT_TRY(wait_event(s, s->r_copied[s->active]));
    return RT_OK;
}

// Host half of one frame: update callback, instance matrices, TLAS rebuild, staging, upload.
// RT_BUILD_LBVH: the host stages matrices and transformed instance boxes only; the BLAS roots are
// patched into the instance records and the TLAS is built by kernels on the scene's stream.
// `upload` (host-built trees): the stream the upload is enqueued on — rt_render passes the stream the
// trace will run on, so upload -> schedule -> trace stay in one queue (a wait on an event of another
// queue cost ~35 us per frame, measured).
// defer (rt_render): the copy itself is left to the next launch on `upload` (pending_copy).
rt_status frame_update(rt_scene *s, uint64_t frame, hipStream_t upload, bool defer = false) {
    const int b = s->active < 0 ? 0 : (s->active + 1) % rt_scene::NLANE;
    const auto w0 = std::chrono::steady_clock::now();
    const int si = s->stage_next % s->stage_depth;      // this frame's staging buffer
    s->stage_next = (si + 1) % s->stage_depth;
    if (s->r_staged[si]) RT_TRY(wait_event(s, s->r_staged[si]));   // no longer read by a pending copy
    if (!s->staging[si]) {
        // every buffer of the cycle at once, on the first frame that needs one: a pinned allocation inside a run of
        // pipelined frames stalls the host's submission (one per frame for the first stage_depth frames)
        for (int i = 0; i < s->stage_depth; i++) {
            if (s->staging[i]) continue;
            HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&s->staging[i]), s->frame_block, hipHostMallocDefault));
            HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&s->staging_dev[i]), s->staging[i], 0));
        }
    }
    s->update_wait_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    if (s->update) {                                  // Renderer.cu:269
        std::vector<rt_xform> xs(s->inst.size());
        for (size_t i = 0; i < xs.size(); i++) xs[i] = s->inst[i].x;
        s->update(s->update_user, xs.data(), xs.size(), frame);
        // matrices are a pure function of (local box, xform): only instances whose xform changed are
        // recomputed (the demo animates 5 of C2's 73 instances) — on the GPU for GPU-built frames
        for (size_t i = 0; i < xs.size(); i++)
            if (std::memcmp(&xs[i], &s->inst[i].x, sizeof(rt_xform)) != 0) {
                if (s->gpu_tlas()) { s->inst[i].x = xs[i]; s->inst_dirty[i] = rt_scene::ALL_BLOCKS; }
                else instance_update(s->inst[i], xs[i]);
            }
    }
    uint8_t *st = s->staging[si];
    InstHot *hot = reinterpret_cast<InstHot *>(st + s->off_hot);
    InstCold *cold = reinterpret_cast<InstCold *>(st + s->off_cold);
    if (s->gpu_tlas()) {
        RT_TRY(lbvh_sync_groups(s));                  // option "group": which records are TLAS items
        s->block_by_slot[b] = false;                  // until the slot-order copy below
        // records: the instances, then (LBVH, option "group") the groups as instances of their merged BLAS
        const size_t nrec = s->inst.size() + s->groups.size();
        // only the changed records cross PCIe: (index, shift, cos / sin of the angles, scale, local box, inactive)
        InstDelta *dl = reinterpret_cast<InstDelta *>(st + s->off_delta);
        uint32_t nd = 0;
        const uint16_t bit = (uint16_t)(1u << b);
        for (size_t i = 0; i < nrec; i++) {
            if (!(s->inst_dirty[i] & bit)) continue;
            s->inst_dirty[i] &= (uint16_t)~bit;
            const InstState &in = record_state(s, i);
            InstDelta &d = dl[nd++];
            std::memset(&d, 0, sizeof d);
            d.index = (uint32_t)i;
            const hm::V3 c = cos3(in.x), sn = sin3(in.x);
            for (int a = 0; a < 3; a++) {
                d.p.shift[a] = hm::of(in.x.shift)[a];
                d.p.cos[a] = c[a];
                d.p.sin[a] = sn[a];
                d.p.scale[a] = hm::of(in.x.scale)[a];
                d.p.centroid[a] = in.centroid[a];
            }
            in.box.store(d.p.box);
            d.p.pad[0] = record_inactive(s, i) ? 1.0f : 0.0f;
        }
        uint8_t *fd = s->frame_dev[b];
        uint32_t live = 0;                              // records in this frame's TLAS
        for (size_t i = 0; i < nrec; i++) live += record_inactive(s, i) ? 0u : 1u;
        const bool small = s->tlas_small && live > 0 && live <= SMALL_TLAS_MAX;
        const uint32_t n = (uint32_t)nrec;
        // the one-workgroup TLAS path touches only block b's buffers, so it runs on the trace's own stream
        // (no cross-queue wait before the trace); the multi-kernel builder's scratch is shared: scene stream
        const hipStream_t cs = small ? upload : s->stream;
        if (s->blas_builder && (s->rebuild_blas || s->blas_dirty)) {    // GPU-built BLASes only (scene stream)
            RT_TRY(gpu_build_blas(s));
            if (!s->ev_blas_built) HIP_TRY(hipEventCreateWithFlags(&s->ev_blas_built, hipEventDisableTiming));
            HIP_TRY(hipEventRecord(s->ev_blas_built, s->stream));
            s->blas_build_seq++;
        }
        // Every frame whose records / TLAS / trace run off the scene stream waits for the last BLAS build once per
        // stream, not only the frame that enqueued it: a build swaps blas_roots / the primitive records to the set
        // being written ("blas_double") or rewrites them in place, and a later frame on another lane stream that
        // builds nothing would otherwise read them mid-build (rt_scene_update_triangles once, a group break)
        if (cs != s->stream && s->blas_build_seq != 0) RT_TRY(wait_blas_built(s, cs));
        if (s->r_used[b]) HIP_TRY(hipStreamWaitEvent(cs, s->r_used[b], 0));      // block b no longer read
        // Instance::updateTransformArguments for every record of block b, on the GPU, with its BLAS root
        // (instances.hip); the deltas are read from the pinned staging block directly
        HIP_TRY(launch_instance_update(reinterpret_cast<const InstDelta *>(s->staging_dev[si] + s->off_delta), nd,
                                       s->inst_params.p + (size_t)b * n, n,
                                       reinterpret_cast<InstHot *>(fd + s->off_hot), reinterpret_cast<InstCold *>(fd + s->off_cold),
                                       reinterpret_cast<float *>(fd + s->off_tbox), reinterpret_cast<float4 *>(fd + s->off_tcent),
                                       s->inst_blas.p, s->blas_roots.p, s->blas_wide_refs.p, /*inf_inactive=*/!small, cs));
        s->chain_stream[b] = cs;
        if (small) {
            // one workgroup: the LBVH TLAS over the live records, quads, slots, slot-ordered records (lbvh.hip)
            SmallTlasArgs a{};
            a.n = n;
            a.hot = reinterpret_cast<const InstHot *>(fd + s->off_hot); a.cold = reinterpret_cast<const InstCold *>(fd + s->off_cold);
            a.tbox = reinterpret_cast<const float *>(fd + s->off_tbox); a.tcent = reinterpret_cast<const float4 *>(fd + s->off_tcent);
            a.pairs = reinterpret_cast<NodePair *>(fd + s->off_pairs); a.root = reinterpret_cast<TreeRoot *>(fd + s->off_root);
            a.root_wide = reinterpret_cast<TreeRoot *>(fd + s->off_root_wide);
            a.quads = reinterpret_cast<NodeQuad *>(fd + s->off_quads); a.slots = reinterpret_cast<uint32_t *>(fd + s->off_slots);
            a.hot_s = reinterpret_cast<InstHot *>(fd + s->off_hot_s); a.cold_s = reinterpret_cast<InstCold *>(fd + s->off_cold_s);
            a.pair_count = s->gpu_counts.p + 2 + b;
            a.leaf_cap = s->tlas_leaf;
            HIP_TRY(launch_tlas_small(a, cs));
            s->block_by_slot[b] = s->inst_by_slot;
            // the trace indexes the slot-ordered copy (live records) or, without "inst_by_slot", the record-order
            // array, whose TLAS slots hold record indices up to n - 1 (lds_scene copies instance_count records)
            s->frame_items[b] = s->inst_by_slot ? live : n;
            HIP_TRY(hipEventRecord(s->ev_copied[b], cs));
            s->r_copied[b] = s->r_staged[si] = s->ev_copied[b];
            s->active = b;
            s->frame = frame;
            return RT_OK;
        }
        s->frame_items[b] = n;
        HIP_TRY(s->tlas_builder->set_items(reinterpret_cast<const float *>(fd + s->off_tbox),
                                           reinterpret_cast<const float4 *>(fd + s->off_tcent)));
        HIP_TRY(s->tlas_builder->build(reinterpret_cast<NodePair *>(fd + s->off_pairs), reinterpret_cast<TreeRoot *>(fd + s->off_root),
                                       s->gpu_counts.p + 2 + b, s->stream));
        HIP_TRY(s->tlas_builder->collapse_wide(reinterpret_cast<const NodePair *>(fd + s->off_pairs),
                                               reinterpret_cast<const TreeRoot *>(fd + s->off_root),
                                               reinterpret_cast<NodeQuad *>(fd + s->off_quads),
                                               reinterpret_cast<TreeRoot *>(fd + s->off_root_wide), s->stream));
        HIP_TRY(s->tlas_builder->gather_items(reinterpret_cast<uint32_t *>(fd + s->off_slots), s->stream));
        if (s->inst_by_slot) {
            HIP_TRY(launch_instance_slot_order(reinterpret_cast<const uint32_t *>(fd + s->off_slots),
                                               reinterpret_cast<const InstHot *>(fd + s->off_hot),
                                               reinterpret_cast<const InstCold *>(fd + s->off_cold), n,
                                               reinterpret_cast<InstHot *>(fd + s->off_hot_s),
                                               reinterpret_cast<InstCold *>(fd + s->off_cold_s), s->stream));
            s->block_by_slot[b] = true;
        }
        HIP_TRY(hipEventRecord(s->ev_copied[b], s->stream));
        s->r_copied[b] = s->r_staged[si] = s->ev_copied[b];
        s->active = b;
        s->frame = frame;
        return RT_OK;
    }
    // TLAS::constructTLAS over transformed instance boxes (Renderer.cu:275, TLAS.cu:4-129)
    // option "group": a group still holding its transform is one item (n + g), else its members are
    std::vector<uint8_t> intact(s->groups.size(), 0);
    for (size_t g = 0; g < s->groups.size(); g++) {
        const InstGroup &G = s->groups[g];
        bool ok = G.valid;
        for (size_t k = 0; ok && k < G.members.size(); k++)
            ok = std::memcmp(&s->inst[G.members[k]].x, &G.st.x, sizeof(rt_xform)) == 0;
        intact[g] = ok;
    }
    std::vector<BuildItem> items;
    items.reserve(s->inst.size() + s->groups.size());
    for (size_t i = 0; i < s->inst.size(); i++)
        if (!s->group_of[i] || !intact[s->group_of[i] - 1]) items.push_back({s->inst[i].tbox, s->inst[i].tcentroid, (uint32_t)i});
    for (size_t g = 0; g < s->groups.size(); g++)
        if (intact[g]) items.push_back({s->groups[g].st.tbox, s->groups[g].st.tcentroid, (uint32_t)(s->inst.size() + g)});
    // RT_BUILD_SAH builds an SAH TLAS (option "tlas_sah" 0: the reference's median split, TLAS.cu:4-129).  The TLAS
    // decides the order in which instances are visited, and with the parallelogram's q-centred box
    // (Parallelogram.cu:48-50) that order is visible: a ray that hits the parallelogram outside its box keeps the hit
    // only when the box is tested before a farther surface shrinks the range.  The reference's median trees test the
    // ground sphere first for the demo's view (a subtree holding it and anything above the camera contains the camera,
    // so its entry is t_min); an SAH TLAS isolates the ground at the root, and visited by entry t (the SAH scenes'
    // quad order) it tests the ground first too — in the reference's pair order it would not (303 of C2's pixels at
    // depth 1; profiles/r05/order/).
    s->tlas = s->build_mode == RT_BUILD_SAH && s->tlas_sah
                  ? build_sah_tree(std::move(items), s->tlas_leaf)
                  : build_median_tree(std::move(items),
                                      s->build_mode == RT_BUILD_SAH && s->tlas_median_leaf ? s->tlas_median_leaf : TLAS_LEAF_CAP,
                                      hm::tlas_axis_state(s->build_seed, frame));
    s->tlas_flat = flatten_tree(s->tlas, 0, 0, 0, false);
    s->tlas_wide = flatten_tree_wide(s->tlas, 0, 0, 0, false, s->quad_halves());

    TreeRoot root{};
    std::memcpy(root.box, s->tlas_flat.root_box, sizeof root.box);
    root.ref = s->tlas_flat.root_ref;
    root.height = s->tlas_flat.height;
    std::memcpy(st + s->off_root, &root, sizeof root);
    root.ref = s->tlas_wide.root_ref;
    root.height = s->tlas_wide.height;
    std::memcpy(st + s->off_root_wide, &root, sizeof root);
    std::memcpy(st + s->off_quads, s->tlas_wide.quads.data(), s->tlas_wide.quads.size() * sizeof(NodeQuad));
    std::memcpy(st + s->off_pairs, s->tlas_flat.pairs.data(), s->tlas_flat.pairs.size() * sizeof(NodePair));
    std::memcpy(st + s->off_slots, s->tlas.refs.data(), s->tlas.refs.size() * sizeof(uint32_t));
    // instance records in TLAS leaf-slot order (SceneGPU::inst_by_slot): record j = the instance in slot j
    const size_t nrec = s->inst_by_slot ? s->tlas.refs.size() : s->inst.size() + s->groups.size();
    s->block_by_slot[b] = s->inst_by_slot;
    s->frame_items[b] = (uint32_t)nrec;
    for (size_t j = 0; j < nrec; j++) {
        const size_t id = s->inst_by_slot ? s->tlas.refs[j] : j;
        const InstState &in = id < s->inst.size() ? s->inst[id] : s->groups[id - s->inst.size()].st;
        const BlasHost &bl = s->blas[in.blas];
        store_rows(hot[j].inv, in.inv);
        std::memcpy(hot[j].root_box, bl.flat.root_box, sizeof hot[j].root_box);
        hot[j].root_ref = bl.flat.root_ref;
        hot[j].root_ref_wide = bl.wide.root_ref;
        store_rows(cold[j].fwd, in.fwd);
        store_rows(cold[j].nrm, in.nrm);
    }
    // Measured: the upload on a dedicated copy stream (the reference's copyStream, Renderer.cu:281-303)
    // went through an SDMA engine whose first use stalled a frame by ~7.6 ms; enqueued on the trace's
    // stream it is a ~4 us blit kernel between two traces.
    HIP_TRY(hipStreamWaitEvent(upload, s->r_used[b], 0));            // frame_dev[b] free on device
    if (defer) {
        s->pending_copy = b;
        s->pending_stage = si;
    } else {
        HIP_TRY(hipMemcpyAsync(s->frame_dev[b], st, s->frame_block, hipMemcpyHostToDevice, upload));
        HIP_TRY(hipEventRecord(s->ev_copied[b], upload));
        s->r_copied[b] = s->r_staged[si] = s->ev_copied[b];
    }
    s->active = b;
    s->frame = frame;
    return RT_OK;
}

SceneGPU scene_gpu(const rt_scene *s) {
    SceneGPU g{};
    const int b = s->active;
    g.blas_pairs = s->blas_pairs.p;
    g.tlas_pairs = reinterpret_cast<const NodePair *>(s->frame_dev[b] + s->off_pairs);
    g.tlas_root = reinterpret_cast<const TreeRoot *>(s->frame_dev[b] + s->off_root);
    g.tlas_root_wide = reinterpret_cast<const TreeRoot *>(s->frame_dev[b] + s->off_root_wide);
    g.tlas_quads = reinterpret_cast<const NodeQuad *>(s->frame_dev[b] + s->off_quads);
    g.blas_quads = s->blas_quads.p;
    // quad trees (GPU-built: from collapse_wide): 1 = host SAH BLASes collapsed greedily, visited by entry t; 2 = two
    // binary levels per quad visited in the reference's order (GPU-built trees); 3 = the same with every box decision
    // inside the FAST slab's error margin re-taken with the reference's slab (the reference's own trees; GPU-built
    // trees with option "exact_decisions")
    g.wide = s->wide && s->blas_quads.p != nullptr
                 ? (s->quad_halves() ? ((s->build_mode == RT_BUILD_COMPAT_MEDIAN || s->exact_decisions) ? 3u : 2u) : 1u)
                 : 0u;
    g.tlas_slots = reinterpret_cast<const uint32_t *>(s->frame_dev[b] + s->off_slots);
    const bool gpu_slots = s->gpu_tlas() && s->block_by_slot[b];   // the slot-ordered copies of GPU-built frames
    g.inst_hot = reinterpret_cast<const InstHot *>(s->frame_dev[b] + (gpu_slots ? s->off_hot_s : s->off_hot));
    g.inst_cold = reinterpret_cast<const InstCold *>(s->frame_dev[b] + (gpu_slots ? s->off_cold_s : s->off_cold));
    g.inst_by_slot = s->block_by_slot[b] ? 1u : 0u;   // how frame block b's instance records were staged
    g.tri_hot = s->tri_hot.p; g.tri_cold = s->raw_shading() ? nullptr : s->tri_cold.p;
    g.raw_tris = s->raw_shading() ? s->raw_tris.p : nullptr;
    g.sph_hot = s->sph_hot.p; g.sph_cold = s->sph_cold.p;
    g.quad_hot = s->quad_hot.p; g.quad_cold = s->quad_cold.p;
    g.materials = s->materials.p;
    g.instance_count = s->frame_items[b];   // records the frame's TLAS holds (GPU-built, small path: the live ones)
    g.rough_count = (uint32_t)s->roughs.size();
    g.material_count = (uint32_t)(s->materials.n / 4);
    // fixed setting "lds_scene" (an option until round 5): the quads the frame's TLAS refs can index (host-built: this frame's quad count;
    // GPU-built: quad q is rooted at pair q, < n - 1) and, if they fit too, the instance hot records
    // then, in this order while they fit: sphere and parallelogram records (hot + cold), instance cold records
    g.lds_icold = g.lds_sph_hot = g.lds_sph_cold = g.lds_q_hot = g.lds_q_cold = LDS_NONE;
    if (s->lds_scene && g.wide) {
        const uint32_t n = g.instance_count;
        const uint32_t nq = s->gpu_tlas() ? (n > 1 ? n - 1 : 0) : (uint32_t)s->tlas_wide.quads.size();   // GPU: <= items - 1
        if (nq > 0 && nq * LDS_QUAD_F4 <= LDS_SCENE_F4) {
            g.lds_quads = nq;
            if (nq * LDS_QUAD_F4 + n * LDS_INST_F4 <= LDS_SCENE_F4) g.lds_insts = n;
        }
        uint32_t at = s->lds_scene >= 2 ? g.lds_quads * LDS_QUAD_F4 + g.lds_insts * LDS_INST_F4 : LDS_SCENE_F4;
        const uint32_t ns = (uint32_t)s->sph_hot.n, nqd = (uint32_t)s->quad_hot.n;
        if (ns > 0 && at + 2 * ns <= LDS_SCENE_F4) { g.lds_sph_hot = at; g.lds_sph_cold = at + ns; at += 2 * ns; }
        if (nqd > 0 && at + (LDS_QPRIM_F4 + 1) * nqd <= LDS_SCENE_F4) {
            g.lds_q_hot = at; g.lds_q_cold = at + LDS_QPRIM_F4 * nqd; at += (LDS_QPRIM_F4 + 1) * nqd;
        }
        if (g.lds_insts && at + n * LDS_ICOLD_F4 <= LDS_SCENE_F4) { g.lds_icold = at; at += n * LDS_ICOLD_F4; }
        // option "group": the top levels of the first group's BLAS in what is left (quads in level order)
        if (s->lds_scene >= 2 && s->lds_blas && g.lds_insts && !s->groups.empty() && !s->gpu_tlas()) {
            const BlasHost &bh = s->blas[s->groups[0].st.blas];
            const uint32_t room = (LDS_SCENE_F4 - std::min(at, LDS_SCENE_F4)) / LDS_QUAD_F4;
            const uint32_t nq_b = std::min<uint32_t>(room, (uint32_t)bh.wide.quads.size());
            if (nq_b > 0 && !(bh.wide.root_ref & REF_LEAF)) {
                g.lds_bq0 = bh.wide.root_ref & REF_INDEX_MASK;
                g.lds_bqn = nq_b;
                g.lds_bq_at = at;
                at += nq_b * LDS_QUAD_F4;
            }
        }
    }
    return g;
}

template <typename T>
rt_status upload(DevBuf<T> &buf, const std::vector<T> &v) {
    buf.release();
    const size_t n = v.empty() ? 1 : v.size();
    HIP_TRY(hipMalloc(&buf.p, n * sizeof(T)));
    buf.n = v.size();
    if (!v.empty()) HIP_TRY(hipMemcpy(buf.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return RT_OK;
}

template <typename T>
rt_status alloc_buf(DevBuf<T> &buf, size_t n) {
    buf.release();
    HIP_TRY(hipMalloc(&buf.p, (n ? n : 1) * sizeof(T)));
    buf.n = n;
    return RT_OK;
}

// RT_BUILD_LBVH + option "group": record i (instances, then groups) kept out of the GPU TLAS — a member of an
// intact group (the group is the TLAS item) or a broken group (its members are)
bool record_inactive(const rt_scene *s, size_t i) {
    if (s->build_mode != RT_BUILD_LBVH || s->groups.empty()) return false;
    if (i < s->inst.size()) return s->group_of[i] && s->lbvh_intact[s->group_of[i] - 1];
    return !s->lbvh_intact[i - s->inst.size()];
}
const InstState &record_state(const rt_scene *s, size_t i) {
    return i < s->inst.size() ? s->inst[i] : s->groups[i - s->inst.size()].st;
}
// a group is one TLAS item while it is valid (no rt_scene_update_instances on a member) and every member still
// has the group's transform (SAH: frame_update; LBVH: lbvh_sync_groups)
bool group_intact(const rt_scene *s, size_t g) {
    const InstGroup &G = s->groups[g];
    bool ok = G.valid;
    for (size_t k = 0; ok && k < G.members.size(); k++)
        ok = std::memcmp(&s->inst[G.members[k]].x, &G.st.x, sizeof(rt_xform)) == 0;
    return ok;
}

// RT_BUILD_LBVH: (re)configure the builder's segments for the current group states: the segments of the BLASes
// in use (item ranges re-tiled in BLAS order), the group member tables, the BLAS arrays sized for them, the
// record -> segment map.  Called at the build and when a group breaks or re-forms (the device is drained).
rt_status lbvh_segments(rt_scene *s) {
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    std::vector<uint8_t> use(s->blas.size(), 1);
    for (size_t g = 0; g < s->groups.size(); g++) {
        if (s->lbvh_intact[g]) for (uint32_t m : s->groups[g].members) use[s->inst[m].blas] = 0;
        else use[s->groups[g].st.blas] = 0;
    }
    std::vector<LbvhSeg> segs;
    std::vector<uint32_t> members;
    s->seg_of_blas.assign(s->blas.size(), NONE);
    uint32_t item = 0;
    for (size_t b = 0; b < s->blas.size(); b++) {
        if (!use[b]) continue;
        LbvhSeg sg = s->lbvh_segs[b];
        sg.item_base = item;
        sg.node_base = item - (uint32_t)segs.size();
        if (!s->blas[b].members.empty()) {
            sg.member_base = (uint32_t)(members.size() / 2);
            sg.member_count = (uint32_t)s->blas[b].members.size();
            for (const auto &m : s->blas[b].members) { members.push_back(m[0]); members.push_back(m[2]); }
        }
        s->seg_of_blas[b] = (uint32_t)segs.size();
        segs.push_back(sg);
        item += sg.count;
    }
    if (!s->blas_builder) s->blas_builder = new LbvhBuilder();
    HIP_TRY(s->blas_builder->init(segs, s->stream));
    HIP_TRY(s->blas_builder->set_members(members, s->stream));
    rt_status st;
    if ((st = alloc_buf(s->blas_pairs, s->blas_builder->max_pairs())) != RT_OK) return st;
    if ((st = alloc_buf(s->blas_quads, s->blas_builder->max_pairs())) != RT_OK) return st;   // quad q = rooted at pair q
    if ((st = alloc_buf(s->blas_roots, segs.size())) != RT_OK) return st;
    const size_t n = s->inst.size() + s->groups.size();
    std::vector<uint32_t> ib(n);
    for (size_t i = 0; i < n; i++) {
        uint32_t sg = s->seg_of_blas[record_state(s, i).blas];
        if (sg == NONE && i < s->inst.size() && s->group_of[i]) sg = s->seg_of_blas[s->groups[s->group_of[i] - 1].st.blas];
        ib[i] = sg == NONE ? 0u : sg;                      // an inactive record's root is never entered
    }
    if ((st = upload(s->inst_blas, ib)) != RT_OK) return st;
    s->blas_dirty = true;
    return RT_OK;
}

// RT_BUILD_LBVH, per frame: a group that broke (a member moved, rt_scene_update_instances) or re-formed switches
// the BLASes built and the records in the TLAS (their inactive flags travel with the next instance deltas)
rt_status lbvh_sync_groups(rt_scene *s) {
    if (s->build_mode != RT_BUILD_LBVH || s->groups.empty()) return RT_OK;
    bool changed = false;
    std::vector<uint8_t> now(s->groups.size());
    for (size_t g = 0; g < s->groups.size(); g++) {
        now[g] = group_intact(s, g) ? 1 : 0;
        changed = changed || now[g] != s->lbvh_intact[g];
    }
    if (!changed) return RT_OK;
    RT_TRY(drain(s));
    for (size_t g = 0; g < s->groups.size(); g++) {
        if (now[g] == s->lbvh_intact[g]) continue;
        for (uint32_t m : s->groups[g].members) s->inst_dirty[m] = rt_scene::ALL_BLOCKS;
        s->inst_dirty[s->inst.size() + g] = rt_scene::ALL_BLOCKS;
    }
    s->lbvh_intact = now;
    for (rt_scene::BlasSet &sp : s->spare) sp.release();   // re-sized with the next double-buffered build
    return lbvh_segments(s);
}

// RT_BUILD_LBVH: rebuild every BLAS on the GPU (prep -> Morton -> sort -> Karras -> boxes -> pairs ->
// leaf-ordered primitive records), on the scene stream, after the last trace that read them.
rt_status gpu_build_blas(rt_scene *s) {
    if (s->blas_double && s->blas_builds > 0) {
        // into the spare set: wait only for the traces that read it (each lane's last one), then swap it in
        rt_scene::BlasSet &sp = s->spare[0];
        rt_status st;
        if (sp.pairs.n != s->blas_pairs.n || sp.tri_hot.n != s->tri_hot.n || sp.sph_hot.n != s->sph_hot.n ||
            sp.quad_hot.n != s->quad_hot.n || sp.roots.n != s->blas_roots.n) {
            RT_TRY(drain(s));
            sp.release();
            if ((st = alloc_buf(sp.pairs, s->blas_pairs.n)) != RT_OK) return st;
            if ((st = alloc_buf(sp.quads, s->blas_quads.n)) != RT_OK) return st;
            if ((st = alloc_buf(sp.roots, s->blas_roots.n)) != RT_OK) return st;
            if ((st = alloc_buf(sp.tri_hot, s->tri_hot.n)) != RT_OK) return st;
            if ((st = alloc_buf(sp.tri_cold, s->tri_cold.n)) != RT_OK) return st;
            if ((st = alloc_buf(sp.sph_hot, s->sph_hot.n)) != RT_OK) return st;
            if ((st = alloc_buf(sp.sph_cold, s->sph_cold.n)) != RT_OK) return st;
            if ((st = alloc_buf(sp.quad_hot, s->quad_hot.n)) != RT_OK) return st;
            if ((st = alloc_buf(sp.quad_cold, s->quad_cold.n)) != RT_OK) return st;
        }
        for (int q = 0; q < rt_scene::NLANE; q++)      // created with the first set (gpu_setup_blas); never recorded: no wait
            HIP_TRY(hipStreamWaitEvent(s->stream, sp.ev_lane[q], 0));
        const RawPrimsGPU raw{s->raw_tris.p, s->raw_verts.p, s->raw_sph.p, s->raw_quad.p, (uint32_t)s->roughs.size()};
        const PrimOutGPU out{sp.tri_hot.p, s->raw_shading() ? nullptr : sp.tri_cold.p, sp.sph_hot.p, sp.sph_cold.p,
                             sp.quad_hot.p, sp.quad_cold.p};
        HIP_TRY(s->blas_builder->set_timing(s->timeline_on));      // option "timeline": stage events (debug_read)
        HIP_TRY(s->blas_builder->prep_blas_items(raw, s->stream, !out.tri_cold));
        HIP_TRY(s->blas_builder->build(sp.pairs.p, sp.roots.p, s->gpu_counts.p, s->stream, &raw, &out));   // + gather
        HIP_TRY(s->blas_builder->collapse_wide(sp.pairs.p, sp.roots.p, sp.quads.p, nullptr, s->stream));
        std::swap(s->blas_pairs, sp.pairs); std::swap(s->blas_quads, sp.quads); std::swap(s->blas_roots, sp.roots);
        std::swap(s->tri_hot, sp.tri_hot); std::swap(s->tri_cold, sp.tri_cold);
        std::swap(s->sph_hot, sp.sph_hot); std::swap(s->sph_cold, sp.sph_cold);
        std::swap(s->quad_hot, sp.quad_hot); std::swap(s->quad_cold, sp.quad_cold);
        for (int q = 0; q < rt_scene::NLANE; q++) std::swap(s->ev_blas_lane[q], sp.ev_lane[q]);
        // the set just retired (frame k read it) becomes the newest spare; the one read longest ago is written next
        std::rotate(s->spare, s->spare + 1, s->spare + (s->blas_sets - 1));
        s->blas_dirty = false;
        s->blas_builds++;
        return RT_OK;
    }
    if (s->blas_builds && s->r_done) HIP_TRY(hipStreamWaitEvent(s->stream, s->r_done, 0));
    for (int q = 0; q < rt_scene::NLANE; q++)           // "overlap": the other lane's trace may still be running
        if (s->blas_builds && s->r_lane[q]) HIP_TRY(hipStreamWaitEvent(s->stream, s->r_lane[q], 0));
    const RawPrimsGPU raw{s->raw_tris.p, s->raw_verts.p, s->raw_sph.p, s->raw_quad.p, (uint32_t)s->roughs.size()};
    const PrimOutGPU out{s->tri_hot.p, s->raw_shading() ? nullptr : s->tri_cold.p, s->sph_hot.p, s->sph_cold.p,
                         s->quad_hot.p, s->quad_cold.p};
    HIP_TRY(s->blas_builder->set_timing(s->timeline_on));      // option "timeline": stage events (debug_read)
    HIP_TRY(s->blas_builder->prep_blas_items(raw, s->stream, !out.tri_cold));
    HIP_TRY(s->blas_builder->build(s->blas_pairs.p, s->blas_roots.p, s->gpu_counts.p, s->stream, &raw, &out));   // + gather
    HIP_TRY(s->blas_builder->collapse_wide(s->blas_pairs.p, s->blas_roots.p, s->blas_quads.p, nullptr, s->stream));
    s->blas_dirty = false;
    s->blas_builds++;
    return RT_OK;
}

// RT_BUILD_LBVH: upload the raw primitives, allocate the leaf-ordered arrays, build every BLAS once.
rt_status gpu_setup_blas(rt_scene *s, const uint32_t *slot_count) {
    const std::vector<LbvhSeg> &segs = s->lbvh_segs;
    bool ok = true;                                  // the host builds check the same materials
    for (const LbvhSeg &g : segs)
        for (uint32_t k = 0; k < g.count; k++) {
            const uint32_t pi = g.prim_base + k;
            if (g.ptype == RT_PRIM_TRIANGLE) material_slot(s, s->tris[pi].material_type, s->tris[pi].material_index, ok);
            else if (g.ptype == RT_PRIM_SPHERE) material_slot(s, s->spheres[pi].material_type, s->spheres[pi].material_index, ok);
            else material_slot(s, s->quads[pi].material_type, s->quads[pi].material_index, ok);
        }
    if (!ok) return fail(RT_ERR_INVALID_ARGUMENT, "primitive references a material out of range");
    rt_status st;
    if ((st = upload(s->raw_tris, s->tris)) != RT_OK) return st;
    if ((st = alloc_buf(s->raw_verts, 9 * s->tris.size())) != RT_OK) return st;
    HIP_TRY(extract_tri_verts(s->raw_tris.p, s->raw_verts.p, 0, s->tris.size(), s->stream));
    if ((st = upload(s->raw_sph, s->spheres)) != RT_OK) return st;
    if ((st = upload(s->raw_quad, s->quads)) != RT_OK) return st;
    if ((st = alloc_buf(s->tri_hot, slot_count[RT_PRIM_TRIANGLE])) != RT_OK) return st;
    if (s->cold_eff) {
        if ((st = alloc_buf(s->tri_cold, slot_count[RT_PRIM_TRIANGLE])) != RT_OK) return st;
    } else {
        s->tri_cold.release();                          // raw_shading(): no TriCold records
    }
    if ((st = alloc_buf(s->sph_hot, slot_count[RT_PRIM_SPHERE])) != RT_OK) return st;
    if ((st = alloc_buf(s->sph_cold, slot_count[RT_PRIM_SPHERE])) != RT_OK) return st;
    if ((st = alloc_buf(s->quad_hot, slot_count[RT_PRIM_PARALLELOGRAM])) != RT_OK) return st;
    if ((st = alloc_buf(s->quad_cold, slot_count[RT_PRIM_PARALLELOGRAM])) != RT_OK) return st;
    delete s->blas_builder;
    s->blas_builder = nullptr;
    s->lbvh_intact.assign(s->groups.size(), 1);       // members start with the group's transform (frame 0 re-checks)
    for (rt_scene::BlasSet &sp : s->spare) sp.release();
    if ((st = lbvh_segments(s)) != RT_OK) return st;
    if ((st = alloc_buf(s->gpu_counts, 2 + rt_scene::NLANE)) != RT_OK) return st;
    if (!s->ev_render_done) HIP_TRY(hipEventCreateWithFlags(&s->ev_render_done, hipEventDisableTiming));
    if (!s->r_done) s->r_done = s->ev_render_done;
    for (int q = 0; q < rt_scene::NLANE; q++) {       // "blas_double": every trace records its lane's event from now on
        if (!s->ev_blas_lane[q]) HIP_TRY(hipEventCreateWithFlags(&s->ev_blas_lane[q], hipEventDisableTiming));
        for (rt_scene::BlasSet &sp : s->spare)
            if (!sp.ev_lane[q]) HIP_TRY(hipEventCreateWithFlags(&sp.ev_lane[q], hipEventDisableTiming));
    }
    s->blas_builds = 0;
    if ((st = gpu_build_blas(s)) != RT_OK) return st;
    // one-time readback for introspection (rt_scene_get_info)
    uint32_t pairs = 0;
    std::vector<TreeRoot> roots(s->blas_roots.n);
    RT_TRY(drain(s));
    HIP_TRY(hipMemcpy(&pairs, s->gpu_counts.p, sizeof pairs, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(roots.data(), s->blas_roots.p, roots.size() * sizeof(TreeRoot), hipMemcpyDeviceToHost));
    s->blas_pair_count = pairs;
    s->blas_leaf_count = pairs + roots.size();       // binary trees: leaves = interior nodes + 1
    for (const TreeRoot &r : roots) s->max_blas_height = std::max(s->max_blas_height, r.height);
    return RT_OK;
}

uint32_t tiles_for_rank(uint32_t w, uint32_t h, uint32_t tw, uint32_t th, uint32_t rank, uint32_t count) {
    if (tw == 0 || th == 0 || count == 0) return 0;
    const uint32_t total = ((w + tw - 1) / tw) * ((h + th - 1) / th);
    return rank < total ? (total - rank + count - 1) / count : 0;
}

}  // namespace

template <typename T>
static hipError_t read_back(std::vector<T> &v, const T *src, size_t n) {
    v.resize(n);
    return n ? hipMemcpy(v.data(), src, n * sizeof(T), hipMemcpyDeviceToHost) : hipSuccess;
}

static void fill_stats(rt_stats *st, const unsigned long long *c);

extern "C" {

uint32_t rt_abi_version(void) { return RT_ABI_VERSION; }

const char *rt_last_error(void) { return g_error.c_str(); }

int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

rt_status rt_scene_create(const rt_scene_desc *d, int device, rt_scene **out) {
    if (!d || !out) return fail(RT_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    if (d->instance_count == 0) return fail(RT_ERR_INVALID_ARGUMENT, "scene has no instances");
    if ((d->sphere_count && !d->spheres) || (d->parallelogram_count && !d->parallelograms) ||
        (d->triangle_count && !d->triangles) || (d->rough_count && !d->roughs) || (d->metal_count && !d->metals) ||
        !d->instances)
        return fail(RT_ERR_INVALID_ARGUMENT, "count without array");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RT_ERR_DEVICE, "no HIP device present");
    if (device < 0 || device >= ndev) return fail(RT_ERR_INVALID_ARGUMENT, "device index out of range");
    auto *s = new (std::nothrow) rt_scene();
    if (!s) return fail(RT_ERR_OUT_OF_MEMORY, "host allocation failed");
    s->device = device;
    s->spheres.assign(d->spheres, d->spheres + d->sphere_count);
    s->quads.assign(d->parallelograms, d->parallelograms + d->parallelogram_count);
    s->tris.assign(d->triangles, d->triangles + d->triangle_count);
    s->roughs.assign(d->roughs, d->roughs + d->rough_count);
    s->metals.assign(d->metals, d->metals + d->metal_count);
    s->inst_desc.assign(d->instances, d->instances + d->instance_count);
    s->update = d->update;
    s->update_user = d->update_user;
    // validate instance map (RenderPin.cu:119-172 would read out of bounds instead)
    for (const auto &id : s->inst_desc) {
        if (id.primitive_type > RT_PRIM_TRIANGLE) { delete s; return fail(RT_ERR_INVALID_ARGUMENT, "bad primitive type"); }
        const size_t len = prim_len(s, id.primitive_type);
        const size_t cnt = id.primitive_count ? id.primitive_count : 1;
        if ((size_t)id.primitive_index + cnt > len) { delete s; return fail(RT_ERR_INVALID_ARGUMENT, "instance primitive range out of bounds"); }
    }
    *out = s;
    return RT_OK;
}

rt_status rt_scene_build(rt_scene *s, rt_build_mode mode, uint64_t seed) {
    if (!s) return fail(RT_ERR_INVALID_ARGUMENT, "null scene");
    if (mode != RT_BUILD_COMPAT_MEDIAN && mode != RT_BUILD_SAH && mode != RT_BUILD_LBVH)
        return fail(RT_ERR_UNSUPPORTED, "unsupported build mode");
    HIP_TRY(hipSetDevice(s->device));
    if (s->built) RT_TRY(drain(s));              // a rebuild frees buffers earlier frames may still read
    s->build_seed = seed;
    s->build_mode = mode;
    s->cold_eff = s->cold_records == 1 || (s->cold_records < 0 && !s->rebuild_blas);
    s->inst.clear();
    s->blas.clear();
    s->groups.clear();
    s->group_of.clear();
    s->max_blas_height = 0;
    for (bool &v : s->block_by_slot) v = false;    // a rebuild may change the mode: no block is slot-ordered yet

    // buildBLASPinMem (RenderPin.cu:99-201): complete instances, one BLAS per unique (type, index).
    // The reference's map stores the instance index instead of the BLAS index (RenderPin.cu:151);
    // the BLAS index is stored here (identical whenever the reference's demo order is used).
    std::vector<std::pair<uint64_t, uint32_t>> seen;
    std::vector<LbvhSeg> &segs = s->lbvh_segs;  // RT_BUILD_LBVH: one tree per unique BLAS
    segs.clear();
    uint64_t item_total = 0;
    uint32_t pair_base = 0, quad_base = 0;
    uint32_t slot_base[3] = {0, 0, 0};
    for (size_t i = 0; i < s->inst_desc.size(); i++) {
        const rt_instance_desc &id = s->inst_desc[i];
        InstState in{};
        in.ptype = id.primitive_type; in.pindex = id.primitive_index; in.pcount = id.primitive_count;
        if (in.pcount == 0) {
            in.pcount = 1;                                           // objectPrimitiveCount()
            in.box = prim_box(s, in.ptype, in.pindex);
            in.centroid = prim_centroid(s, in.ptype, in.pindex);
        } else if (id.has_local_bounds) {                            // VTKReader.cu:204-209
            in.box = hm::Box::from_ranges({id.local_bounds[0], id.local_bounds[1]}, {id.local_bounds[2], id.local_bounds[3]},
                                          {id.local_bounds[4], id.local_bounds[5]});
            in.centroid = hm::of(id.local_centroid);
        } else {                                                     // extension: union box, mean centroid
            hm::Box bb = prim_box(s, in.ptype, in.pindex);
            double c[3] = {0, 0, 0};
            for (uint32_t k = 0; k < in.pcount; k++) {
                if (k) bb = hm::Box::merge(bb, prim_box(s, in.ptype, in.pindex + k));
                const hm::V3 pc = prim_centroid(s, in.ptype, in.pindex + k);
                for (int a = 0; a < 3; a++) c[a] += pc[a];
            }
            in.box = bb;
            in.centroid = hm::v3((float)(c[0] / in.pcount), (float)(c[1] / in.pcount), (float)(c[2] / in.pcount));
        }
        const uint64_t key = ((uint64_t)in.ptype << 32) | in.pindex;
        bool dup = false;
        for (const auto &kv : seen)
            if (kv.first == key) { in.blas = kv.second; dup = true; break; }
        if (!dup) {
            in.blas = (uint32_t)s->blas.size();
            seen.push_back({key, in.blas});
            BlasHost bh;
            bh.type = in.ptype;
            if (mode == RT_BUILD_LBVH) {
                if ((uint64_t)slot_base[in.ptype] + in.pcount >= MAX_LEAF_SLOTS || item_total + in.pcount >= (1ull << 31))
                    return fail(RT_ERR_UNSUPPORTED, "too many primitives of one type (2^26 leaf slots)");
                bh.pair_base = 0;
                bh.slot_base = slot_base[in.ptype];
                segs.push_back(LbvhSeg{(uint32_t)item_total, in.pcount, slot_base[in.ptype], in.pindex, in.ptype,
                                       (uint32_t)(item_total - segs.size()), LBVH_BLAS_LEAF_CAP, 1u});
                item_total += in.pcount;
                slot_base[in.ptype] += in.pcount;
                s->blas.push_back(std::move(bh));
                s->inst.push_back(in);
                continue;
            }
            std::vector<BuildItem> items(in.pcount);
            for (uint32_t k = 0; k < in.pcount; k++)
                items[k] = {prim_box(s, in.ptype, in.pindex + k), prim_centroid(s, in.ptype, in.pindex + k), in.pindex + k};
            bh.tree = mode == RT_BUILD_SAH ? build_sah_tree(std::move(items), s->blas_leaf)
                                           : build_median_tree(std::move(items), BLAS_LEAF_CAP, hm::blas_axis_state(seed, in.blas));
            bh.pair_base = pair_base;
            bh.slot_base = slot_base[in.ptype];
            if ((uint64_t)slot_base[in.ptype] + in.pcount >= MAX_LEAF_SLOTS)
                return fail(RT_ERR_UNSUPPORTED, "too many primitives of one type (2^26 leaf slots)");
            bh.flat = flatten_tree(bh.tree, pair_base, bh.slot_base, in.ptype, true);
            bh.wide = flatten_tree_wide(bh.tree, quad_base, bh.slot_base, in.ptype, true, s->quad_halves());
            quad_base += (uint32_t)bh.wide.quads.size();
            s->max_blas_height = std::max(s->max_blas_height, bh.flat.height);
            pair_base += (uint32_t)bh.flat.pairs.size();
            slot_base[in.ptype] += in.pcount;
            s->blas.push_back(std::move(bh));
        }
        s->inst.push_back(in);
    }
    s->blas_own = s->blas.size();
    s->group_of.assign(s->inst.size(), 0u);
    if (s->group_inst && ((mode == RT_BUILD_SAH && !s->gpu_tlas()) || mode == RT_BUILD_LBVH)) {
        // option "group": triangle instances with bit-identical transforms and a BLAS of their own
        std::vector<uint32_t> users(s->blas.size(), 0u);
        for (const InstState &in : s->inst) users[in.blas]++;
        std::map<std::string, std::vector<uint32_t>> by_xform;
        for (size_t i = 0; i < s->inst.size(); i++) {
            const InstState &in = s->inst[i];
            if (in.ptype != RT_PRIM_TRIANGLE || users[in.blas] != 1) continue;
            const rt_xform &x = s->inst_desc[i].xform;
            by_xform[std::string(reinterpret_cast<const char *>(&x), sizeof x)].push_back((uint32_t)i);
        }
        for (auto &kv : by_xform) {
            if (kv.second.size() < 2) continue;
            InstGroup g;
            g.members = kv.second;
            std::vector<std::array<uint32_t, 3>> ranges;
            for (uint32_t i : g.members) ranges.push_back({s->inst[i].pindex, s->inst[i].pcount, i});
            std::sort(ranges.begin(), ranges.end());
            bool disjoint = true;          // every triangle of the group belongs to exactly one member
            for (size_t k = 1; k < ranges.size(); k++)
                disjoint = disjoint && ranges[k][0] >= ranges[k - 1][0] + ranges[k - 1][1];
            if (mode == RT_BUILD_LBVH) {
                // the group's LBVH segment is one contiguous primitive range and reuses its members' leaf slots:
                // their triangles back to back, their slot ranges too (the reference's VTK particles, C5)
                for (size_t k = 1; k < ranges.size() && disjoint; k++) {
                    const BlasHost &a = s->blas[s->inst[ranges[k - 1][2]].blas], &c = s->blas[s->inst[ranges[k][2]].blas];
                    disjoint = ranges[k][0] == ranges[k - 1][0] + ranges[k - 1][1] && c.slot_base == a.slot_base + ranges[k - 1][1];
                }
            }
            if (!disjoint) continue;
            const uint32_t gi = (uint32_t)s->groups.size();
            uint64_t total = 0;
            double c[3] = {0, 0, 0};
            BlasHost bh;
            bh.type = RT_PRIM_TRIANGLE;
            for (size_t k = 0; k < g.members.size(); k++) {
                const InstState &m = s->inst[g.members[k]];
                g.st.box = k ? hm::Box::merge(g.st.box, m.box) : m.box;
                for (int a = 0; a < 3; a++) c[a] += m.centroid[a];
                total += m.pcount;
                bh.members.push_back({m.pindex, m.pcount, g.members[k]});
                s->group_of[g.members[k]] = gi + 1;
            }
            if (mode != RT_BUILD_LBVH && (uint64_t)slot_base[RT_PRIM_TRIANGLE] + total >= MAX_LEAF_SLOTS)
                return fail(RT_ERR_UNSUPPORTED, "too many primitives of one type (2^26 leaf slots)");
            g.st.ptype = RT_PRIM_TRIANGLE;
            g.st.pindex = 0;
            g.st.pcount = (uint32_t)total;
            g.st.centroid = hm::v3((float)(c[0] / g.members.size()), (float)(c[1] / g.members.size()),
                                   (float)(c[2] / g.members.size()));
            g.st.x = s->inst_desc[g.members[0]].xform;
            if (mode == RT_BUILD_LBVH) {
                // one more segment over the members' triangles, in their leaf slots (lbvh_segments builds either
                // it or the members' own segments); item / node bases are assigned there
                bh.slot_base = s->blas[s->inst[ranges[0][2]].blas].slot_base;
                bh.pair_base = 0;
                segs.push_back(LbvhSeg{0u, (uint32_t)total, bh.slot_base, ranges[0][0], RT_PRIM_TRIANGLE, 0u,
                                       LBVH_BLAS_LEAF_CAP, 1u, 0u, 0u});
                std::sort(bh.members.begin(), bh.members.end());
                g.st.blas = (uint32_t)s->blas.size();
                s->blas.push_back(std::move(bh));
                s->groups.push_back(std::move(g));
                continue;
            }
            std::vector<BuildItem> items;
            items.reserve(total);
            for (const auto &mr : bh.members)
                for (uint32_t k = 0; k < mr[1]; k++)
                    items.push_back({prim_box(s, RT_PRIM_TRIANGLE, mr[0] + k), prim_centroid(s, RT_PRIM_TRIANGLE, mr[0] + k), mr[0] + k});
            bh.tree = build_sah_tree(std::move(items), s->blas_leaf);
            bh.pair_base = pair_base;
            bh.slot_base = slot_base[RT_PRIM_TRIANGLE];
            bh.flat = flatten_tree(bh.tree, pair_base, bh.slot_base, RT_PRIM_TRIANGLE, true);
            bh.wide = flatten_tree_wide(bh.tree, quad_base, bh.slot_base, RT_PRIM_TRIANGLE, true, s->quad_halves(),
                                        /*level_order=*/true);
            quad_base += (uint32_t)bh.wide.quads.size();
            s->max_blas_height = std::max(s->max_blas_height, bh.flat.height);
            pair_base += (uint32_t)bh.flat.pairs.size();
            slot_base[RT_PRIM_TRIANGLE] += (uint32_t)total;
            std::sort(bh.members.begin(), bh.members.end());
            g.st.blas = (uint32_t)s->blas.size();
            s->blas.push_back(std::move(bh));
            s->groups.push_back(std::move(g));
        }
    }

    std::vector<float> mats;
    for (const auto &r : s->roughs) { mats.push_back(r.albedo.x); mats.push_back(r.albedo.y); mats.push_back(r.albedo.z); mats.push_back(0.0f); }
    for (const auto &m : s->metals) { mats.push_back(m.albedo.x); mats.push_back(m.albedo.y); mats.push_back(m.albedo.z); mats.push_back(m.fuzz); }
    rt_status st;
    if (!s->stream) {
        // the scene stream (uploads, GPU BLAS builds) at normal priority: the highest measured neutral (round 3)
        HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    }
    if (!s->ev_render_done) HIP_TRY(hipEventCreateWithFlags(&s->ev_render_done, hipEventDisableTiming));
    if (!s->r_done) s->r_done = s->ev_render_done;
    for (bool &v : s->sched_valid) v = false;
    if (mode == RT_BUILD_LBVH) {
        if ((st = gpu_setup_blas(s, slot_base)) != RT_OK) return st;
    } else {
    // leaf-ordered primitive arrays + node pairs
    std::vector<NodePair> pairs;
    pairs.reserve(pair_base);
    std::vector<NodeQuad> quads;
    quads.reserve(quad_base);
    std::vector<TriHot> th; std::vector<TriCold> tc;
    std::vector<SphereHot> sh; std::vector<PrimCold> sc;
    std::vector<QuadHot> qh; std::vector<PrimCold> qc;
    th.reserve(slot_base[2]); tc.reserve(slot_base[2]);
    bool mat_ok = true;
    s->blas_leaf_count = 0;
    for (const BlasHost &bh : s->blas) {
        pairs.insert(pairs.end(), bh.flat.pairs.begin(), bh.flat.pairs.end());
        quads.insert(quads.end(), bh.wide.quads.begin(), bh.wide.quads.end());
        s->blas_leaf_count += bh.flat.leaves;
        for (uint32_t pi : bh.tree.refs) {
            if (bh.type == RT_PRIM_TRIANGLE) {
                const rt_triangle &t = s->tris[pi];
                const hm::TriDerived dv = hm::tri_derive(t);
                TriHot h{};
                TriCold c{};
                for (int a = 0; a < 3; a++) {
                    h.v0[a] = hm::of(t.vertex[0])[a]; h.e1[a] = dv.e1[a]; h.e2[a] = dv.e2[a];
                    c.n0[a] = dv.n[0][a]; c.n1[a] = dv.n[1][a]; c.n2[a] = dv.n[2][a];
                }
                c.material = material_slot(s, t.material_type, t.material_index, mat_ok);
                c.orig_index = pi;
                if (!bh.members.empty()) {        // a group's BLAS: the caller instance holding triangle pi, + 1
                    auto it = std::upper_bound(bh.members.begin(), bh.members.end(), std::array<uint32_t, 3>{pi, ~0u, ~0u});
                    c.pad = (*(it - 1))[2] + 1u;
                }
                th.push_back(h); tc.push_back(c);
            } else if (bh.type == RT_PRIM_SPHERE) {
                const rt_sphere &sp = s->spheres[pi];
                sh.push_back(SphereHot{{sp.center.x, sp.center.y, sp.center.z}, sp.radius});
                sc.push_back(PrimCold{material_slot(s, sp.material_type, sp.material_index, mat_ok), pi, 0, 0});
            } else {
                const rt_parallelogram &p = s->quads[pi];
                const hm::QuadDerived dv = hm::quad_derive(p);
                QuadHot q{};
                for (int a = 0; a < 3; a++) {
                    q.n[a] = dv.n[a]; q.q[a] = hm::of(p.q)[a]; q.u[a] = hm::of(p.u)[a]; q.v[a] = hm::of(p.v)[a];
                    q.nx[a] = dv.nx[a];
                }
                q.d = dv.d; q.den = dv.den;
                qh.push_back(q);
                qc.push_back(PrimCold{material_slot(s, p.material_type, p.material_index, mat_ok), pi, 0, 0});
            }
        }
    }
    if (!mat_ok) return fail(RT_ERR_INVALID_ARGUMENT, "primitive references a material out of range");
    s->blas_pair_count = pairs.size();

    if ((st = upload(s->blas_pairs, pairs)) != RT_OK) return st;
    if ((st = upload(s->blas_quads, quads)) != RT_OK) return st;
    if ((st = upload(s->tri_hot, th)) != RT_OK) return st;
    if ((st = upload(s->tri_cold, tc)) != RT_OK) return st;
    if ((st = upload(s->sph_hot, sh)) != RT_OK) return st;
    if ((st = upload(s->sph_cold, sc)) != RT_OK) return st;
    if ((st = upload(s->quad_hot, qh)) != RT_OK) return st;
    if ((st = upload(s->quad_cold, qc)) != RT_OK) return st;
    }
    if ((st = upload(s->materials, mats)) != RT_OK) return st;

    // per-frame double buffers (sized for every instance and every group as a TLAS item)
    const size_t n = s->inst.size() + s->groups.size();
    s->off_root = 0;
    s->off_pairs = 64;
    s->off_slots = align16(s->off_pairs + n * sizeof(NodePair));
    s->off_hot = align16(s->off_slots + n * sizeof(uint32_t));
    s->off_cold = align16(s->off_hot + n * sizeof(InstHot));
    s->off_tbox = align16(s->off_cold + n * sizeof(InstCold));
    s->off_tcent = align16(s->off_tbox + n * 6 * sizeof(float));
    s->off_root_wide = 32;                                         // second half of the root's 64 B
    s->off_quads = (s->off_tcent + n * 4 * sizeof(float) + 127) & ~size_t(127);
    s->off_delta = align16(s->off_quads + n * sizeof(NodeQuad));   // <= n - 1 quads
    s->frame_block = s->off_delta + (s->gpu_tlas() ? n * sizeof(InstDelta) : 0);
    if (s->gpu_tlas()) {       // GPU-built TLAS: the instance records again, in TLAS leaf-slot order
        s->off_hot_s = align16(s->frame_block);
        s->off_cold_s = align16(s->off_hot_s + n * sizeof(InstHot));
        s->frame_block = s->off_cold_s + n * sizeof(InstCold);
    }
    if (s->gpu_tlas() && mode == RT_BUILD_SAH) {
        // host-built BLASes under the GPU TLAS: their roots (box, pair ref, quad ref) and the instance map
        std::vector<TreeRoot> roots(s->blas.size());
        std::vector<uint32_t> wide_refs(s->blas.size()), ib(n);
        for (size_t b = 0; b < s->blas.size(); b++) {
            std::memcpy(roots[b].box, s->blas[b].flat.root_box, sizeof roots[b].box);
            roots[b].ref = s->blas[b].flat.root_ref;
            roots[b].height = s->blas[b].flat.height;
            wide_refs[b] = s->blas[b].wide.root_ref;
        }
        for (size_t i = 0; i < s->inst.size(); i++) ib[i] = s->inst[i].blas;
        if ((st = upload(s->blas_roots, roots)) != RT_OK) return st;
        if ((st = upload(s->blas_wide_refs, wide_refs)) != RT_OK) return st;
        if ((st = upload(s->inst_blas, ib)) != RT_OK) return st;
        if ((st = alloc_buf(s->gpu_counts, 2 + rt_scene::NLANE)) != RT_OK) return st;
    }
    if (s->gpu_tlas()) {
        if ((st = alloc_buf(s->inst_params, n * rt_scene::NLANE)) != RT_OK) return st;   // one copy per frame block
        s->inst_dirty.assign(n, rt_scene::ALL_BLOCKS);              // each block's first frame uploads every record
        delete s->tlas_builder;
        s->tlas_builder = new LbvhBuilder();
        const std::vector<LbvhSeg> tseg{LbvhSeg{0u, (uint32_t)n, 0u, 0u, 0u, 0u, s->tlas_leaf, 0u}};
        HIP_TRY(s->tlas_builder->init(tseg, s->stream));
    }
    for (int i = 0; i < rt_scene::NSTAGE; i++) {
        if (s->staging[i]) { (void)hipHostFree(s->staging[i]); s->staging[i] = nullptr; }   // frame_update allocates
        s->staging_dev[i] = nullptr;
        s->r_staged[i] = nullptr;
    }
    s->stage_next = 0;
    for (int b = 0; b < rt_scene::NLANE; b++) {
        if (s->frame_dev[b]) { (void)hipFree(s->frame_dev[b]); s->frame_dev[b] = nullptr; }
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&s->frame_dev[b]), s->frame_block));
        if (!s->ev_copied[b]) HIP_TRY(hipEventCreateWithFlags(&s->ev_copied[b], hipEventDisableTiming));
        if (!s->ev_used[b]) HIP_TRY(hipEventCreateWithFlags(&s->ev_used[b], hipEventDisableTiming));
        if (!s->r_copied[b]) s->r_copied[b] = s->ev_copied[b];
        if (!s->r_used[b]) s->r_used[b] = s->ev_used[b];
    }
    for (uint32_t i = 0; i < rt_scene::RING; i++) {
        if (!s->ring_start[i]) HIP_TRY(hipEventCreate(&s->ring_start[i]));
        if (!s->ring_stop[i]) HIP_TRY(hipEventCreate(&s->ring_stop[i]));
        if (!s->ring_post[i]) HIP_TRY(hipEventCreateWithFlags(&s->ring_post[i], hipEventDisableTiming));
    }
    if (!s->counters) {
        HIP_TRY(hipMalloc(&s->counters, rt_scene::NLANE * CNT_NUM * sizeof(unsigned long long)));
        HIP_TRY(hipMemset(s->counters, 0, rt_scene::NLANE * CNT_NUM * sizeof(unsigned long long)));
    }
    for (int q = 0; q < rt_scene::NLANE; q++) {
        if (!s->queue[q]) {   // band heads, then (option "reorder") band item counts, one 128 B line each
            HIP_TRY(hipMalloc(&s->queue[q], QUEUE_WORDS * sizeof(uint32_t)));
            HIP_TRY(hipMemset(s->queue[q], 0, QUEUE_WORDS * sizeof(uint32_t)));
        }
        if (!s->ev_lane_done[q]) HIP_TRY(hipEventCreateWithFlags(&s->ev_lane_done[q], hipEventDisableTiming));
        if (!s->r_lane[q]) s->r_lane[q] = s->ev_lane_done[q];
    }
    {
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, s->device));
        s->cus = (uint32_t)prop.multiProcessorCount;
        if (const char *k = std::getenv("RTAMD_KERNEL")) s->use_persistent = std::string(k) != "grid";
        if (const char *t = std::getenv("RTAMD_THRESHOLD")) {
            const long v = std::strtol(t, nullptr, 10);
            if (v >= 1 && v <= 64) s->threshold = (uint32_t)v;
        }
    }
    if (!s->counters_host)
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&s->counters_host), rt_scene::NLANE * CNT_NUM * sizeof(unsigned long long),
                              hipHostMallocDefault));
    s->active = -1;

    // initial transforms, then the frame-0 update + TLAS (Renderer.cu:110-111, 148-150)
    for (size_t i = 0; i < s->inst.size(); i++) instance_update(s->inst[i], s->inst_desc[i].xform);
    for (InstGroup &g : s->groups) instance_update(g.st, g.st.x);
    s->built = true;
    return frame_update(s, 0, s->stream);
}

rt_status rt_camera_set(rt_scene *s, const rt_camera_input *c, uint32_t w, uint32_t h) {
    if (!s || !c) return fail(RT_ERR_INVALID_ARGUMENT, "null argument");
    if (w == 0 || h == 0 || w > 32768 || h > 32768) return fail(RT_ERR_INVALID_ARGUMENT, "bad framebuffer size");
    if (c->sample_count == 0) return fail(RT_ERR_INVALID_ARGUMENT, "sample_count must be >= 1");
    // RendererImpl::calculateCameraProperties (src/Global/RenderPin.cu:73-95)
    using namespace hm;
    const V3 center = of(c->center), target = of(c->target), up = of(c->up);
    const float fd = distance(center, target);
    const float theta = c->fov * PI / 180.0f;
    const float vw = 2.0f * std::tan(theta / 2.0f) * fd;
    const float vh = vw / ((float)w * 1.0f / (float)h);
    const V3 W = unit(target - center);
    const V3 U = unit(cross(W, up));
    const V3 V = unit(cross(U, W));
    const V3 vx = U * vw, vy = V * vh;
    const V3 dx = vx / (float)w, dy = vy / (float)h;
    const V3 vorg = center + W * fd - vx * 0.5f - vy * 0.5f;
    const V3 po = vorg + dx * 0.5f + dy * 0.5f;
    CameraGPU &g = s->cam;
    for (int a = 0; a < 3; a++) {
        g.pixel_origin[a] = po[a]; g.dx[a] = dx[a]; g.dy[a] = dy[a]; g.center[a] = center[a];
        g.cu[a] = U[a]; g.cv[a] = V[a]; g.background[a] = of(c->background)[a];
    }
    g.focus_radius = c->focus_disk_radius;
    g.sqrt_s = (uint32_t)std::sqrt((double)c->sample_count);            // RenderPin.cu:93
    g.recip_sqrt = 1.0f / (float)g.sqrt_s;                              // RenderPin.cu:94
    g.depth = c->ray_trace_depth;
    g.width = w; g.height = h;
    g.pitch = (w + 15u) / 16u * 16u;                                    // 16x16 blocks (SDL_OpenGLWindow.cu:119-122)
    s->width = w; s->height = h;
    s->cam_ok = true;
    return RT_OK;
}

rt_status rt_scene_update(rt_scene *s, uint64_t frame) {
    if (!s) return fail(RT_ERR_INVALID_ARGUMENT, "null scene");
    if (!s->built) return fail(RT_ERR_STATE, "rt_scene_build has not been called");
    HIP_TRY(hipSetDevice(s->device));
    return frame_update(s, frame, s->stream);
}

uint32_t rt_tiles_for_rank(const rt_scene *s, uint32_t tw, uint32_t th, uint32_t rank, uint32_t count) {
    if (!s || !s->cam_ok) return 0;
    return tiles_for_rank(s->width, s->height, tw, th, rank, count);
}

uint32_t rt_slab_tiles(uint32_t w, uint32_t h, uint32_t tw, uint32_t th, uint32_t count) {
    if (w == 0 || h == 0 || tw == 0 || th == 0 || count == 0) return 0;
    return slab_tile_count(w, h, tw, th, count);
}

rt_status rt_tile_pixels(uint32_t w, uint32_t h, uint32_t tw, uint32_t th, uint32_t rank, uint32_t count, uint64_t first,
                         uint64_t n, int32_t *xy) {
    if ((n && !xy) || w == 0 || h == 0 || tw == 0 || th == 0 || count == 0 || rank >= count)
        return fail(RT_ERR_INVALID_ARGUMENT, "bad tile geometry");
    for (uint64_t i = 0; i < n; i++) {
        uint32_t x = 0, y = 0;
        const bool in = tile_pixel(w, h, tw, th, rank, count, first + i, x, y);
        xy[2 * i] = in ? (int32_t)x : -1;
        xy[2 * i + 1] = in ? (int32_t)y : -1;
    }
    return RT_OK;
}

rt_status rt_comm_unique_id(rt_comm_id *id) {
    if (!id) return fail(RT_ERR_INVALID_ARGUMENT, "null argument");
    static_assert(sizeof(rt_comm_id) == sizeof(ncclUniqueId), "rt_comm_id must be an ncclUniqueId");
    const Rccl &R = rccl();
    if (!R.ok) return fail(RT_ERR_UNSUPPORTED, R.error);
    ncclUniqueId u;
    const ncclResult_t e = R.GetUniqueId(&u);
    if (e != ncclSuccess) return fail(RT_ERR_DEVICE, std::string("ncclGetUniqueId: ") + R.GetErrorString(e));
    std::memcpy(id, &u, sizeof u);
    return RT_OK;
}

rt_status rt_scene_attach_comm(rt_scene *s, const rt_comm_id *id, int rank, int world, uint32_t tw, uint32_t th) {
    if (!s || !id) return fail(RT_ERR_INVALID_ARGUMENT, "null argument");
    if (world < 1 || rank < 0 || rank >= world) return fail(RT_ERR_INVALID_ARGUMENT, "rank must be in [0, world)");
    if (tw == 0 || th == 0 || tw % 8 || th % 8) return fail(RT_ERR_INVALID_ARGUMENT, "tiles must be multiples of 8");
    const Rccl &R = rccl();
    if (!R.ok) return fail(RT_ERR_UNSUPPORTED, R.error);
    HIP_TRY(hipSetDevice(s->device));
    RT_TRY(drain(s));
    s->release_comm();
    auto *cm = new (std::nothrow) CommState();
    if (!cm) return fail(RT_ERR_OUT_OF_MEMORY, "host allocation failed");
    cm->rank = rank; cm->world = world; cm->tile_w = tw; cm->tile_h = th;
    // one per lane in use (auto lanes: the 8 a rank's share runs on, auto_lanes)
    cm->ncomm = (int)std::max<uint32_t>(1u, s->overlap_auto && world > 1 ? 8u : (s->overlap ? s->lanes : 1u));
    cm->timeout_ms = s->comm_timeout_ms;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclResult_t e = R.CommInitRank(&cm->comm[0], world, u, rank);
    for (int q = 1; q < cm->ncomm && e == ncclSuccess; q++) e = R.CommSplit(cm->comm[0], 0, rank, &cm->comm[q], nullptr);
    s->comm = cm;
    if (e != ncclSuccess) {
        const std::string msg = std::string("RCCL communicator: ") + R.GetErrorString(e);
        s->release_comm();
        return fail(RT_ERR_DEVICE, msg);
    }
    return RT_OK;
}

rt_status rt_comm_set_timeout(rt_scene *s, uint32_t timeout_ms) {
    if (!s) return fail(RT_ERR_INVALID_ARGUMENT, "null scene");
    s->comm_timeout_ms = timeout_ms;
    if (s->comm) s->comm->timeout_ms = timeout_ms;
    return RT_OK;
}

rt_status rt_scene_detach_comm(rt_scene *s) {
    if (!s) return fail(RT_ERR_INVALID_ARGUMENT, "null scene");
    if (!s->comm) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    RT_TRY(drain(s));
    s->release_comm();
    return RT_OK;
}

// Option "overlap" -1: the lane count (and staging depth) bench.py measured best per frame kind:
// with a per-frame BLAS rebuild 2 lanes (the rebuild is the frame's critical path and starves behind traces in
// flight: C5 8.8 against 9.8 ms/frame with 4 lanes; a C5 1/8 share 4.1 against 5.5 with 8; C2-LBVH 0.38 against 1.04
// with 3; profiles/r04/c5_rebuild/, profiles/r05/c5_rebuild/); else a rank's share of a multi-GPU frame (tiles, or a
// communicator of world > 1) 8 lanes and 64 staging buffers, any other frame 4 lanes.  Changing the count drains the
// scene (a new frame kind, e.g. attaching a communicator).
rt_status auto_lanes(rt_scene *s, const rt_render_opts &o) {
    const bool share = o.tile_count > 0 || (s->comm && s->comm->world > 1);
    const uint32_t L = s->rebuild_blas ? 2u : (share ? 8u : 4u);
    const int depth = share ? rt_scene::NSTAGE : 16;
    if (L == s->lanes && (s->stage_depth_set || depth == s->stage_depth)) return RT_OK;
    RT_TRY(drain(s));
    s->lanes = L;
    s->overlap = L > 1;
    s->lane = 0;
    if (!s->stage_depth_set) {
        s->stage_depth = depth;
        s->stage_next = 0;
    }
    return RT_OK;
}

rt_status rt_render(rt_scene *s, uint64_t frame, const rt_render_opts *opts, uint8_t *rgba_host, float *rgb_host,
                    rt_stats *stats) {
    const auto t0 = std::chrono::steady_clock::now();
    if (!s) return fail(RT_ERR_INVALID_ARGUMENT, "null scene");
    if (!s->built) return fail(RT_ERR_STATE, "rt_scene_build has not been called");
    if (!s->cam_ok) return fail(RT_ERR_STATE, "rt_camera_set has not been called");
    rt_render_opts o{};
    if (opts) o = *opts;
    if (o.frame_seed == 0) o.frame_seed = 0x5EED;
    CommState *cm = s->comm;
    if (cm) {                                  // multi-GPU frame: the communicator owns the tiling
        if (o.tile_count) return fail(RT_ERR_INVALID_ARGUMENT, "tile options are set by rt_scene_attach_comm");
        if (o.rgb32_device || rgb_host) return fail(RT_ERR_UNSUPPORTED, "rgb32 outputs are not gathered across ranks");
        o.tile_w = cm->tile_w; o.tile_h = cm->tile_h;
        o.tile_rank = (uint32_t)cm->rank; o.tile_count = (uint32_t)cm->world;
    }
    // a trace that skips the frame update after rt_scene_update_triangles would traverse the old trees while its hits
    // read the new triangles (raw_tris): the next frame update rebuilds the BLASes first
    if ((o.flags & RT_RENDER_SKIP_UPDATE) && s->blas_dirty)
        return fail(RT_ERR_STATE, "triangles were updated since the last frame update: render a frame with the update first");
    HIP_TRY(hipSetDevice(s->device));
    if (s->overlap_auto) RT_TRY(auto_lanes(s, o));
    // the frame's stream: the caller's; else, with "overlap", the lane's own stream (created on first use), else the
    // scene's stream (every frame of the scene in order)
    hipStream_t stream = static_cast<hipStream_t>(o.stream);
    const bool lib_lane = !stream && s->overlap;
    if (lib_lane) {
        hipStream_t &ls = s->lane_st[s->lane];
        if (!ls) {
            int lo = 0, hi = 0;                    // option "lane_priority": 1 = the device's highest stream priority
            HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
            HIP_TRY(hipStreamCreateWithPriority(&ls, hipStreamNonBlocking, s->lane_priority ? hi : 0));
        }
        stream = ls;
    } else if (!stream) {
        stream = s->stream;
    }
    double update_ms = 0.0;
    if (!(o.flags & RT_RENDER_SKIP_UPDATE)) {
        const auto u0 = std::chrono::steady_clock::now();
        const rt_status st = frame_update(s, frame, stream, /*defer=*/true);
        if (st != RT_OK) return st;
        update_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - u0).count();
    }

    // Launches of one lane never overlap, whatever streams callers pass (queue heads, unit costs).
    // Without "overlap" every launch is lane 0.  With it, frames alternate lanes: a launch waits only
    // for the previous launch of its own lane (and, below, for its frame block), so the caller can run
    // consecutive frames concurrently on two streams.
    const int q = s->overlap ? (int)s->lane : 0;
    OutputGPU out{};
    out.leaf_early = s->leaf_early >= 0 ? (uint32_t)s->leaf_early
                                        : (s->cam.depth * s->cam.sqrt_s * s->cam.sqrt_s <= 2u ? 0u : rt_scene::LEAF_EARLY_AUTO);
    const uint32_t W = s->width, H = s->height;
    size_t npix;
    if (o.tile_count == 0) {
        out.units_x = (W + 7) / 8;
        out.units = out.units_x * ((H + 7) / 8);
        npix = (size_t)W * H;
    } else {
        if (o.tile_w == 0 || o.tile_h == 0 || o.tile_w % 8 || o.tile_h % 8 || o.tile_rank >= o.tile_count)
            return fail(RT_ERR_INVALID_ARGUMENT, "tiles must be multiples of 8 and tile_rank < tile_count");
        const uint32_t mine = tiles_for_rank(W, H, o.tile_w, o.tile_h, o.tile_rank, o.tile_count);
        out.tile_w = o.tile_w; out.tile_h = o.tile_h; out.tile_rank = o.tile_rank; out.tile_count = o.tile_count;
        out.tiles_x = (W + o.tile_w - 1) / o.tile_w;
        out.units = mine * (o.tile_w / 8) * (o.tile_h / 8);
        npix = (size_t)mine * o.tile_w * o.tile_h;
        const uint32_t upr = o.tile_w / 8;
        out.div_upr = make_fastdiv(upr);
        out.div_upt = make_fastdiv(upr * (o.tile_h / 8));
        out.div_tiles_x = make_fastdiv(out.tiles_x);
        if ((uint64_t)out.tiles_x * ((H + o.tile_h - 1) / o.tile_h) >= (1ull << FASTDIV_BITS))
            return fail(RT_ERR_INVALID_ARGUMENT, "too many tiles");
    }
    if ((uint64_t)out.units * 64u >= (1ull << FASTDIV_BITS))       // work items index pixels of whole units
        return fail(RT_ERR_INVALID_ARGUMENT, "frame too large: more than 2^27 pixels per launch");
    out.div_units_x = make_fastdiv(out.units_x ? out.units_x : 1u);
    // outputs: caller device buffers, else scene-owned; a rank of a multi-GPU frame traces into its lane's slab
    uint8_t *frame_out = nullptr;              // multi-GPU, rank 0: the assembled frame
    if (cm) {
        const size_t slab_bytes = (size_t)slab_tile_count(W, H, cm->tile_w, cm->tile_h, (uint32_t)cm->world) * cm->tile_w *
                                  cm->tile_h * 4;
        if (slab_bytes != cm->slab_bytes) {    // first frame, or the camera size changed: lanes may be in flight
            RT_TRY(drain(s));
            for (int l = 0; l < CommState::NLANE; l++) { cm->slab[l].release(); cm->gathered[l].release(); }
            cm->slab_bytes = slab_bytes;
        }
        DevBuf<uint8_t> &buf = cm->rank == 0 ? cm->gathered[q] : cm->slab[q];
        const size_t need = cm->rank == 0 ? slab_bytes * (size_t)cm->world : slab_bytes;
        if (!buf.p) {                          // slab padding is never assembled: no clearing needed
            HIP_TRY(hipMalloc(&buf.p, need));
            buf.n = need;
        }
        out.rgba = buf.p;                      // rank 0: slab 0 of the gather buffer
        if (cm->rank == 0) {
            if (o.rgba8_device) {
                frame_out = static_cast<uint8_t *>(o.rgba8_device);
            } else {
                if (s->out_rgba.n < (size_t)W * H * 4) {
                    s->out_rgba.release();
                    HIP_TRY(hipMalloc(&s->out_rgba.p, (size_t)W * H * 4));
                    s->out_rgba.n = (size_t)W * H * 4;
                }
                frame_out = s->out_rgba.p;
            }
        }
    } else if (o.rgba8_device) {
        out.rgba = static_cast<uint8_t *>(o.rgba8_device);
    } else {
        if (s->out_rgba.n < npix * 4) {
            s->out_rgba.release();
            HIP_TRY(hipMalloc(&s->out_rgba.p, npix * 4));
            s->out_rgba.n = npix * 4;
        }
        out.rgba = s->out_rgba.p;
    }
    if (o.rgb32_device) {
        out.rgb = static_cast<float *>(o.rgb32_device);
    } else if (rgb_host) {
        if (s->out_rgb.n < npix * 3) {
            s->out_rgb.release();
            HIP_TRY(hipMalloc(&s->out_rgb.p, npix * 3 * sizeof(float)));
            s->out_rgb.n = npix * 3;
        }
        out.rgb = s->out_rgb.p;
    }
    CameraGPU cam = s->cam;
    cam.frame_seed = o.frame_seed;
    const SceneGPU g = scene_gpu(s);
    const bool exact = (o.flags & RT_RENDER_EXACT) != 0;
    const bool count = (o.flags & RT_RENDER_COUNT_WORK) != 0;

    if (s->use_persistent) {
        out.queue_parts = s->queue_parts;
        out.grab = s->grab;
        out.supertile = s->supertile;
        if (s->timeline_on) {
            const uint32_t blocks = s->cus * (exact ? persistent_blocks_per_cu_exact(0u, false)
                                                    : (s->fast_math ? persistent_blocks_per_cu_fastmath(g.wide, g.raw_tris != nullptr)
                                                                   : persistent_blocks_per_cu_fast(g.wide, g.raw_tris != nullptr)));
            const size_t words = (size_t)blocks * 4 * TIMELINE_WORDS;
            if (s->timeline.n < words) {
                s->timeline.release();
                HIP_TRY(hipMalloc(&s->timeline.p, words * sizeof(unsigned long long)));
                s->timeline.n = words;
            }
            HIP_TRY(hipMemsetAsync(s->timeline.p, 0, words * sizeof(unsigned long long), stream));
            out.timeline = s->timeline.p;
            s->timeline_waves = blocks * 4;
        }
        if (s->costmap_on && count) {
            if (s->costmap.n < npix) {
                s->costmap.release();
                HIP_TRY(hipMalloc(&s->costmap.p, npix * sizeof(uint32_t)));
                s->costmap.n = npix;
            }
            HIP_TRY(hipMemsetAsync(s->costmap.p, 0, npix * sizeof(uint32_t), stream));
            out.costmap = s->costmap.p;
            s->costmap_pixels = npix;
        }
    }
    s->lane = s->overlap ? (s->lane + 1) % s->lanes : 0u;
    s->last_lane = q;
    if (hipEvent_t prev = s->overlap ? s->r_lane[q] : s->r_done) HIP_TRY(hipStreamWaitEvent(stream, prev, 0));
    // Device outputs and no stream: the trace runs on a non-blocking stream of the scene, which HIP does not order
    // with the caller's null-stream work, so it waits for what the caller enqueued there before the call (e.g. a fill
    // of the buffer), and — without "overlap" — the null stream waits for the frame (a read of it after the call).  The
    // reference draws into a surface it owns on its own stream (Renderer.cu:305-317), so a drop-in caller expects no
    // ordering of its own.  With "overlap" the frames run side by side on the scene's lanes; a null-stream wait per
    // frame would serialise them, so their device outputs are complete once rt_synchronize returns.
    // (A null stream with nothing pending needs no wait: one host query instead of a cross-queue wait, ~5 us of GPU
    // idle time per frame, profiles/r02_gaps.txt.)
    const bool order_null = !o.stream && (o.rgba8_device || o.rgb32_device);
    if (order_null && hipStreamQuery(nullptr) == hipErrorNotReady) {
        if (!s->ev_caller) HIP_TRY(hipEventCreateWithFlags(&s->ev_caller, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(s->ev_caller, nullptr));
        HIP_TRY(hipStreamWaitEvent(stream, s->ev_caller, 0));
    }
    unsigned long long *lane_counters = s->counters + (size_t)q * CNT_NUM;   // only this lane's launches add here
    if (!(o.flags & RT_RENDER_KEEP_COUNTERS)) s->cnt_epoch++;
    bool zero_lane = s->lane_epoch[q] != s->cnt_epoch;                      // cleared before this launch
    s->lane_epoch[q] = s->cnt_epoch;
    bool reset_queue = true;
    bool copied_here = false;                  // this call enqueued the frame block's upload on `stream`
    // ... of this frame block: no event between the copy and the trace (each event record between two kernels
    // of a stream costs ~4.5 us of GPU idle: copy -> trace gap 10.6 -> 6.1 us, profiles/r02_gaps.txt); its
    // r_copied is the trace's completion event (the host waits on it only before reusing the staging buffer)
    int copied_block = -1, copied_stage = -1;
    if (s->use_persistent && s->reorder && s->grab == 64u) {
        DevBuf<uint32_t> &unit_cost = s->unit_cost[q], &unit_order = s->unit_order[q];
        if (unit_cost.n < 2 * (size_t)out.units) {        // [recorded costs | costs of the last launch (debug)]
            unit_cost.release();
            unit_order.release();
            HIP_TRY(hipMalloc(&unit_cost.p, 2 * (size_t)out.units * sizeof(uint32_t)));
            unit_cost.n = 2 * (size_t)out.units;
            HIP_TRY(hipMemsetAsync(unit_cost.p, 0, unit_cost.n * sizeof(uint32_t), stream));
            HIP_TRY(hipMalloc(&unit_order.p, 4 * (size_t)out.units * sizeof(uint32_t)));   // <= 4 items per unit
            unit_order.n = 4 * (size_t)out.units;
            s->sched_valid[q] = false;
        }
        const uint32_t sig[7] = {out.units, out.units_x, out.tile_w, out.tile_h, out.tile_rank, out.tile_count,
                                 out.queue_parts};
        // the costs the lane's previous launch recorded are for the layout it had
        const bool layout_ok = s->sched_valid[q] && std::memcmp(sig, s->sched_sig[q], sizeof sig) == 0;
        const uint32_t K = s->reorder_period;
        uint32_t &ph = s->sched_phase[q];
        // phase 0 records costs, phase 1 orders from them; K = 1: both on every launch.  A new layout
        // starts over: the schedule kernel clears the costs and this launch records in screen order.
        bool run_sched, track;
        if (!layout_ok) {
            run_sched = true; track = true; s->order_ok[q] = false; ph = K == 1 ? 0u : 1u;
        } else if (K == 1) {
            run_sched = true; track = true;
        } else {
            run_sched = ph == 1; track = ph == 0; ph = (ph + 1) % K;
        }
        const bool do_order = layout_ok && run_sched;
        if (run_sched) {
            const uint32_t rows = out.tile_count == 0 ? out.units / out.units_x : out.units;
            const uint32_t upr = out.tile_count == 0 ? out.units_x : 1u;
            const int pc = s->pending_copy;
            HIP_TRY(launch_schedule(unit_cost.p, unit_cost.p + out.units, unit_order.p, s->queue[q], rows, upr, out.queue_parts,
                                    do_order, s->split & 0xFFu, (s->split >> 8) & 0xFFu, s->merge,
                                    pc >= 0 ? s->frame_dev[pc] : nullptr,
                                    pc >= 0 ? s->staging_dev[s->pending_stage] : nullptr, pc >= 0 ? s->frame_block : 0,
                                    zero_lane ? lane_counters : nullptr, stream));
            zero_lane = false;
            copied_here = pc >= 0;
            copied_block = pc;
            copied_stage = s->pending_stage;
            s->pending_copy = -1;
            if (do_order) s->order_ok[q] = true;
            reset_queue = false;
        }
        std::memcpy(s->sched_sig[q], sig, sizeof sig);
        s->sched_valid[q] = true;
        out.order = s->order_ok[q] ? unit_order.p : nullptr;
        out.unit_cost = track ? unit_cost.p : nullptr;
    }
    if (s->pending_copy >= 0) {                // the frame block's upload (and the lane's counter / queue reset)
        HIP_TRY(launch_frame_copy(s->frame_dev[s->pending_copy], s->staging_dev[s->pending_stage], s->frame_block,
                                  zero_lane ? lane_counters : nullptr, reset_queue && s->use_persistent ? s->queue[q] : nullptr,
                                  stream));
        copied_block = s->pending_copy;
        copied_stage = s->pending_stage;
        s->pending_copy = -1;
        zero_lane = false;
        reset_queue = false;
        copied_here = true;
    }
    // the frame block's upload: stream-ordered when this call enqueued it
    if (!copied_here && !(s->gpu_tlas() && s->chain_stream[s->active] == stream))   // else built on this stream
        HIP_TRY(hipStreamWaitEvent(stream, s->r_copied[s->active], 0));
    if (zero_lane || (reset_queue && s->use_persistent)) {   // GPU-built frames: one small kernel instead of two fills
        HIP_TRY(launch_frame_copy(nullptr, nullptr, 0, zero_lane ? lane_counters : nullptr,
                                  reset_queue && s->use_persistent ? s->queue[q] : nullptr, stream));
        zero_lane = false;
        if (s->use_persistent) reset_queue = false;
    }
    const uint32_t slot = s->ring_head;
    s->ring_head = (s->ring_head + 1) % rt_scene::RING;
    if (s->ring_pending < rt_scene::RING) s->ring_pending++;
    s->last_stream = stream;
    HIP_TRY(hipEventRecord(s->ring_start[slot], stream));
    if (s->use_persistent) {
        const uint32_t cap = s->cus * (exact ? persistent_blocks_per_cu_exact(0u, false)
                                             : (s->fast_math ? persistent_blocks_per_cu_fastmath(g.wide, g.raw_tris != nullptr)
                                                            : persistent_blocks_per_cu_fast(g.wide, g.raw_tris != nullptr)));
        uint32_t blocks = s->overlap && cap > 2 * s->reserve ? cap - s->reserve : cap;
        uint32_t pct = s->grid_pct;
        if (pct == 0) {
            bool partner = false;             // another lane's launch not finished yet (host query, ~1 us)
            for (int l = 0; s->overlap && l < rt_scene::NLANE && !partner; l++)
                partner = l != q && s->r_lane[l] && hipEventQuery(s->r_lane[l]) == hipErrorNotReady;
            // with a partner: half the GPU for up to 3 lanes, 1 / lanes + 12 % of it with more (4 lanes: 37 %, 8 lanes:
            // 24 %: the measured best for a whole frame on 4 lanes and for a rank's 1/2, 1/4 and 1/8 share once every
            // lane runs off the null stream: C2 0.173 -> 0.164 ms/frame, C2 1/8 share 0.041 -> 0.038, 1/4 0.059 ->
            // 0.052; profiles/r03_session2/share_grid_*.txt, lanes_new*.txt); alone: all of it
            pct = !partner ? 100u : (s->lanes <= 3 ? 50u : 100u / s->lanes + 12u);
            // a launch of >= BIG_LAUNCH_PATHS camera paths (C5: 4K x 4 traced spp = 33 M) keeps all of it: its own
            // tail is a small part of its span, and a half grid only stretches the span (C5 5.88 -> 5.43 ms/frame
            // with trees built once, 13.3 -> 11.2 with the per-frame rebuild; profiles/r04/c5_rebuild/)
            if ((uint64_t)out.units * 64u * cam.sqrt_s * cam.sqrt_s >= rt_scene::BIG_LAUNCH_PATHS) pct = 100u;
        }
        if (pct < 100) blocks = std::max<uint32_t>(8u, blocks * pct / 100u);
        const uint32_t thr = s->threshold ? s->threshold : (cam.depth * cam.sqrt_s * cam.sqrt_s <= 2u ? 64u : 40u);
        HIP_TRY(exact ? launch_render_persistent_exact(g, cam, out, count, lane_counters, s->queue[q], blocks, thr,
                                                       reset_queue, stream)
                      : (s->fast_math ? launch_render_persistent_fastmath(g, cam, out, count, lane_counters, s->queue[q], blocks,
                                                                          thr, reset_queue, stream)
                                      : launch_render_persistent_fast(g, cam, out, count, lane_counters, s->queue[q], blocks, thr,
                                                                      reset_queue, stream)));
    }
    else
        HIP_TRY(exact ? launch_render_exact(g, cam, out, count, lane_counters, stream)
                      : (s->fast_math ? launch_render_fastmath(g, cam, out, count, lane_counters, stream)
                                      : launch_render_fast(g, cam, out, count, lane_counters, stream)));
    HIP_TRY(hipEventRecord(s->ring_stop[slot], stream));
    hipEvent_t done = s->ring_stop[slot];      // the launch's one completion event (see r_used)
    if (cm) {
        // gather the ranks' slabs to rank 0 (grouped point-to-point over xGMI: each rank's bytes take
        // their own link into rank 0), then scatter them into the frame there
        const Rccl &R = rccl();
        const size_t sb = cm->slab_bytes;
        if (cm->world > 1) {
            ncclResult_t e = R.GroupStart();
            if (cm->rank == 0) {
                for (int r = 1; r < cm->world && e == ncclSuccess; r++)
                    e = R.Recv(cm->gathered[q].p + (size_t)r * sb, sb, ncclUint8, r, cm->comm[q % cm->ncomm], stream);
            } else if (e == ncclSuccess) {
                e = R.Send(cm->slab[q].p, sb, ncclUint8, 0, cm->comm[q % cm->ncomm], stream);
            }
            const ncclResult_t e2 = R.GroupEnd();
            if (e != ncclSuccess || e2 != ncclSuccess)
                return fail(RT_ERR_DEVICE, std::string("RCCL tile gather: ") + R.GetErrorString(e != ncclSuccess ? e : e2));
        }
        if (cm->rank == 0)
            HIP_TRY(launch_assemble(cm->gathered[q].p, (uint32_t)(sb / (4ull * cm->tile_w * cm->tile_h)), cm->tile_w,
                                    cm->tile_h, (uint32_t)cm->world, W, H, frame_out, stream));
    }
    if (cm) {                                  // after the gather + assemble; one event per launch, never one
        HIP_TRY(hipEventRecord(s->ring_post[slot], stream));   // re-recorded by the lane's next frame (the
        done = s->ring_post[slot];                              // staging / block waits must see this launch)
    }
    s->r_used[s->active] = s->r_done = s->r_lane[q] = done;
    if (copied_block >= 0) s->r_copied[copied_block] = s->r_staged[copied_stage] = done;
    if (s->ev_blas_lane[q]) HIP_TRY(hipEventRecord(s->ev_blas_lane[q], stream));   // "blas_double": this set's reader
    if (order_null && !lib_lane) HIP_TRY(hipStreamWaitEvent(nullptr, done, 0));
    if (o.flags & RT_RENDER_NO_SYNC) {
        if (stats) { std::memset(stats, 0, sizeof *stats); stats->update_ms = update_ms; stats->update_wait_ms = s->update_wait_ms; }
        return RT_OK;
    }
    // counters: this lane's block; with "overlap" + RT_RENDER_KEEP_COUNTERS the accumulated totals of every lane
    // in the current epoch (as rt_scene_collect sums them), after every lane's launches finished
    const bool sum_lanes = s->overlap && (o.flags & RT_RENDER_KEEP_COUNTERS);
    if (!sum_lanes)
        HIP_TRY(hipMemcpyAsync(s->counters_host, lane_counters, CNT_NUM * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
    RT_TRY(wait_stream(s, stream));
    if (sum_lanes) {
        RT_TRY(drain(s));
        HIP_TRY(hipMemcpy(s->counters_host, s->counters, rt_scene::NLANE * CNT_NUM * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost));
        for (int l = 1; l < rt_scene::NLANE; l++)          // lane blocks of the current epoch, summed into block 0
            for (uint32_t k = 0; k < CNT_NUM; k++) {
                if (l == 1 && s->lane_epoch[0] != s->cnt_epoch) s->counters_host[k] = 0;
                if (s->lane_epoch[l] == s->cnt_epoch) s->counters_host[k] += s->counters_host[(size_t)l * CNT_NUM + k];
            }
    }
    s->ring_pending = 0;
    if (rgba_host && cm && cm->rank == 0) HIP_TRY(hipMemcpy(rgba_host, frame_out, (size_t)W * H * 4, hipMemcpyDeviceToHost));
    else if (rgba_host && !cm) HIP_TRY(hipMemcpy(rgba_host, out.rgba, npix * 4, hipMemcpyDeviceToHost));
    if (rgb_host) HIP_TRY(hipMemcpy(rgb_host, out.rgb, npix * 3 * sizeof(float), hipMemcpyDeviceToHost));
    if (stats) {
        float kms = 0.0f;
        HIP_TRY(hipEventElapsedTime(&kms, s->ring_start[slot], s->ring_stop[slot]));
        fill_stats(stats, s->counters_host);
        stats->kernel_ms = kms;
        stats->update_ms = update_ms;
        stats->update_wait_ms = s->update_wait_ms;
        stats->frame_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    if (count && s->counters_host[CNT_OVERFLOW] != 0)
        return fail(RT_ERR_UNSUPPORTED, "traversal stack overflow (tree deeper than 64 levels)");
    return RT_OK;
}

rt_status rt_assemble_tiles(rt_scene *s, const void *gathered, uint32_t slab_tiles, uint32_t tw, uint32_t th,
                            uint32_t tile_count, void *frame, void *stream) {
    if (!s || !gathered || !frame) return fail(RT_ERR_INVALID_ARGUMENT, "null argument");
    if (!s->cam_ok) return fail(RT_ERR_STATE, "rt_camera_set has not been called");
    if (tw == 0 || th == 0 || tile_count == 0) return fail(RT_ERR_INVALID_ARGUMENT, "bad tile geometry");
    if (((uintptr_t)gathered | (uintptr_t)frame) & 3u) return fail(RT_ERR_INVALID_ARGUMENT, "RGBA8 buffers must be 4-byte aligned");
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : s->stream;
    if (!stream) {                             // caller buffers on the scene's stream: ordered with the null stream
        if (!s->ev_caller) HIP_TRY(hipEventCreateWithFlags(&s->ev_caller, hipEventDisableTiming));   // (rt_render)
        HIP_TRY(hipEventRecord(s->ev_caller, nullptr));
        HIP_TRY(hipStreamWaitEvent(st, s->ev_caller, 0));
    }
    HIP_TRY(launch_assemble(gathered, slab_tiles, tw, th, tile_count, s->width, s->height, frame, st));
    if (!stream) {
        HIP_TRY(hipEventRecord(s->ev_caller, st));
        HIP_TRY(hipStreamWaitEvent(nullptr, s->ev_caller, 0));
    }
    return RT_OK;
}

rt_status rt_trace_rays(rt_scene *s, const float *rays, size_t n, uint32_t flags, rt_hit *hits) {
    if (!s || (n && (!rays || !hits))) return fail(RT_ERR_INVALID_ARGUMENT, "null argument");
    if (!s->built) return fail(RT_ERR_STATE, "rt_scene_build has not been called");
    if (n == 0) return RT_OK;
    if (n > 0xFFFFFFFFull) return fail(RT_ERR_INVALID_ARGUMENT, "too many rays");
    if (s->blas_dirty)
        return fail(RT_ERR_STATE, "triangles were updated since the last frame update: render a frame with the update first");
    HIP_TRY(hipSetDevice(s->device));
    float *d_rays = nullptr;
    rt_hit *d_hits = nullptr;
    HIP_TRY(hipMalloc(&d_rays, n * 6 * sizeof(float)));
    hipError_t e = hipMalloc(&d_hits, n * sizeof(rt_hit));
    if (e != hipSuccess) { (void)hipFree(d_rays); return fail(RT_ERR_OUT_OF_MEMORY, "hipMalloc hits"); }
    const SceneGPU g = scene_gpu(s);
    e = hipMemcpyAsync(d_rays, rays, n * 6 * sizeof(float), hipMemcpyHostToDevice, s->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(s->stream, s->r_copied[s->active], 0);
    if (e == hipSuccess)
        e = (flags & RT_RENDER_EXACT) ? launch_trace_rays_exact(g, d_rays, (uint32_t)n, d_hits, s->stream)
                                      : (s->fast_math ? launch_trace_rays_fastmath(g, d_rays, (uint32_t)n, d_hits, s->stream)
                                                      : launch_trace_rays_fast(g, d_rays, (uint32_t)n, d_hits, s->stream));
    if (e == hipSuccess) e = hipEventRecord(s->ev_used[s->active], s->stream);
    if (e == hipSuccess) { s->r_used[s->active] = s->ev_used[s->active]; s->r_done = s->ev_used[s->active]; }
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (e == hipSuccess) e = hipMemcpy(hits, d_hits, n * sizeof(rt_hit), hipMemcpyDeviceToHost);
    (void)hipFree(d_rays);
    (void)hipFree(d_hits);
    if (e != hipSuccess) return fail(RT_ERR_DEVICE, std::string("rt_trace_rays: ") + hipGetErrorString(e));
    return RT_OK;
}

rt_status rt_box_test(int device, const float *boxes, const float *rays, const float *tmax, size_t n, uint32_t mode,
                      uint8_t *hit, float *te) {
    if (n && (!boxes || !rays || !tmax || !hit || !te)) return fail(RT_ERR_INVALID_ARGUMENT, "null argument");
    if (mode > RT_BOX_QUAD_GREEDY) return fail(RT_ERR_INVALID_ARGUMENT, "mode must be an rt_box_mode");
    if (n > 0xFFFFFFFFull / 6) return fail(RT_ERR_INVALID_ARGUMENT, "too many boxes");
    if (n == 0) return RT_OK;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count)
        return fail(RT_ERR_INVALID_ARGUMENT, "no such device");
    HIP_TRY(hipSetDevice(device));
    const size_t fb = n * 6 * sizeof(float);
    char *d = nullptr;                          // boxes | rays | tmax | te | hit
    HIP_TRY(hipMalloc(&d, 2 * fb + 2 * n * sizeof(float) + n));
    float *db = reinterpret_cast<float *>(d), *dr = reinterpret_cast<float *>(d + fb);
    float *dt = reinterpret_cast<float *>(d + 2 * fb), *de = dt + n;
    uint8_t *dh = reinterpret_cast<uint8_t *>(de + n);
    hipError_t e = hipMemcpy(db, boxes, fb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dr, rays, fb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dt, tmax, n * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = mode == RT_BOX_REFERENCE ? launch_box_test_exact(db, dr, dt, (uint32_t)n, mode, dh, de, nullptr)
                                     : launch_box_test_fast(db, dr, dt, (uint32_t)n, mode, dh, de, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(hit, dh, n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(te, de, n * sizeof(float), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(RT_ERR_DEVICE, std::string("rt_box_test: ") + hipGetErrorString(e));
    return RT_OK;
}

// The caller-facing options (include/rt.h, 19 keys).  Round 6 removed the tuning switches whose only use was an A/B
// study (their measured defaults are fixed now: refill threshold, leaf_early, queue bands, claim size, supertile walk,
// merge / split claim items, reorder period, reserved slots, LDS scene levels, instance-record order, leaf sizes) and
// the measured-negative or neutral ones with their code (variant, nt_store, cost_max, tlas_classes, wide_merge,
// scene_priority): DESIGN.md §4 keeps their measurements.
rt_status rt_scene_set_option(rt_scene *s, const char *key, int64_t value) {
    if (!s || !key) return fail(RT_ERR_INVALID_ARGUMENT, "null argument");
    const std::string k(key);
    const auto boolean = [&](const char *name) -> rt_status {
        if (value != 0 && value != 1) return fail(RT_ERR_INVALID_ARGUMENT, std::string(name) + " must be 0 or 1");
        return RT_OK;
    };
    if (k == "kernel") {
        RT_TRY(boolean("kernel"));
        s->use_persistent = value == 1;
    } else if (k == "fast_math") {
        RT_TRY(boolean("fast_math"));
        s->fast_math = value == 1;
    } else if (k == "stage_depth") {
        // pinned staging buffers the host cycles through: it stages frame k once frame k - depth's trace is done
        if (value < 2 || value > rt_scene::NSTAGE) return fail(RT_ERR_INVALID_ARGUMENT, "stage_depth must be in 2..64");
        RT_TRY(drain(s));
        s->stage_depth = (int)value;
        s->stage_next = 0;
        s->stage_depth_set = true;
    } else if (k == "rebuild") {
        RT_TRY(boolean("rebuild"));
        if (value == 1 && s->built && s->build_mode != RT_BUILD_LBVH)
            return fail(RT_ERR_UNSUPPORTED, "per-frame BLAS rebuild needs RT_BUILD_LBVH");
        s->rebuild_blas = value == 1;
    } else if (k == "timeline") {
        RT_TRY(boolean("timeline"));
        s->timeline_on = value == 1;
    } else if (k == "costmap") {
        RT_TRY(boolean("costmap"));
        s->costmap_on = value == 1;
    } else if (k == "cold_records") {
        if (value < -1 || value > 1) return fail(RT_ERR_INVALID_ARGUMENT, "cold_records must be -1, 0 or 1");
        if (s->built) return fail(RT_ERR_STATE, "cold_records must be set before rt_scene_build");
        s->cold_records = (int)value;
    } else if (k == "blas_sets") {
        if (value < 2 || value > (int64_t)rt_scene::MAX_BLAS_SETS)
            return fail(RT_ERR_INVALID_ARGUMENT, "blas_sets must be in 2..8");
        RT_TRY(drain(s));
        s->blas_sets = (uint32_t)value;
    } else if (k == "blas_double") {
        RT_TRY(boolean("blas_double"));
        s->blas_double = value == 1;
    } else if (k == "grid_pct") {
        if (value < 0 || value > 100) return fail(RT_ERR_INVALID_ARGUMENT, "grid_pct must be in 0..100 (0 = auto)");
        s->grid_pct = (uint32_t)value;
    } else if (k == "wide") {
        RT_TRY(boolean("wide"));
        s->wide = value == 1;
    } else if (k == "exact_decisions") {
        RT_TRY(boolean("exact_decisions"));
        s->exact_decisions = value == 1;
    } else if (k == "tlas_small") {
        RT_TRY(boolean("tlas_small"));
        s->tlas_small = value == 1;
    } else if (k == "gpu_tlas") {
        RT_TRY(boolean("gpu_tlas"));
        if (s->built) return fail(RT_ERR_UNSUPPORTED, "gpu_tlas is set before rt_scene_build");
        s->gpu_tlas_sah = value == 1;
    } else if (k == "group") {
        RT_TRY(boolean("group"));
        s->group_inst = value == 1;                   // next rt_scene_build
    } else if (k == "lane_priority") {
        RT_TRY(boolean("lane_priority"));
        RT_TRY(drain(s));
        for (hipStream_t &l : s->lane_st) {
            if (!l) continue;
            // nothing may keep a handle to a destroyed lane stream: drain() waits on last_stream, frame_update
            // compares chain_stream[] with the frame's stream
            if (s->last_stream == l) s->last_stream = nullptr;
            for (hipStream_t &c : s->chain_stream)
                if (c == l) c = nullptr;
            (void)hipStreamDestroy(l);
            l = nullptr;                                                // recreated at the next frame
        }
        s->lane_priority = value == 1;
    } else if (k == "tlas_sah") {
        RT_TRY(boolean("tlas_sah"));
        s->tlas_sah = value == 1;                 // next frame's TLAS
    } else if (k == "overlap") {
        if (value < -1 || value > rt_scene::NLANE) return fail(RT_ERR_INVALID_ARGUMENT, "overlap must be -1 (auto) or 0..8 lanes");
        RT_TRY(drain(s));
        s->overlap_auto = value == -1;
        s->lanes = value < 1 ? (value == -1 ? 4u : 1u) : (uint32_t)value;      // auto: resolved per frame (auto_lanes)
        s->overlap = s->lanes > 1;
        s->lane = 0;
    } else if (k == "reorder") {
        RT_TRY(boolean("reorder"));
        if (s->reorder != (value == 1)) for (bool &v : s->sched_valid) v = false;
        s->reorder = value == 1;
    } else {
        return fail(RT_ERR_INVALID_ARGUMENT, "unknown option " + k);
    }
    return RT_OK;
}

rt_status rt_scene_debug_read(rt_scene *s, const char *name, void *dst, size_t capacity, size_t *bytes) {
    if (!s || !name || !bytes || (!dst && capacity)) return fail(RT_ERR_INVALID_ARGUMENT, "null argument");
    *bytes = 0;
    const std::string k(name);
    const void *src = nullptr;
    size_t size = 0;
    if (k == "rebuild_stages") {
        // option "timeline" and RT_BUILD_LBVH: the last BLAS build's items, interior nodes, node pairs written, items
        // in large trees (> 2048 items), large trees, then the duration in ms of each LbvhBuilder stage
        // (LbvhBuilder::STAGE_NAMES), as float64 (waits for the build)
        if (!s->blas_builder) return fail(RT_ERR_STATE, "no GPU BLAS build (RT_BUILD_LBVH)");
        constexpr int NS = LbvhBuilder::STAGES;
        *bytes = (5 + NS) * sizeof(double);
        if (!capacity) return RT_OK;
        if (capacity < *bytes) return fail(RT_ERR_INVALID_ARGUMENT, "buffer too small");
        HIP_TRY(hipSetDevice(s->device));
        float ms[NS];
        const hipError_t e = s->blas_builder->stage_ms(ms);
        if (e != hipSuccess) return fail(RT_ERR_STATE, "no timed BLAS build: set option \"timeline\" before the frame");
        uint32_t pairs = 0;
        HIP_TRY(hipMemcpy(&pairs, s->gpu_counts.p, sizeof pairs, hipMemcpyDeviceToHost));
        double v[5 + NS];
        v[0] = s->blas_builder->items();
        v[1] = s->blas_builder->max_pairs();
        v[2] = pairs;
        v[3] = s->blas_builder->large_items();
        v[4] = s->blas_builder->large_trees();
        for (int j = 0; j < NS; j++) v[5 + j] = ms[j];
        std::memcpy(dst, v, sizeof v);
        return RT_OK;
    }
    if (k == "timeline") {
        src = s->timeline.p;
        size = (size_t)s->timeline_waves * TIMELINE_WORDS * sizeof(uint64_t);
    } else if (k == "costmap") {
        src = s->costmap.p;
        size = s->costmap_pixels * sizeof(uint32_t);
    } else if (k == "launch_times") {
        // the trace launches not yet collected (rt_scene_collect), oldest first: (start, stop) in ms relative to
        // the first one's start, as float pairs — how lanes' launches interleave (scripts/lane_timeline.py)
        HIP_TRY(hipSetDevice(s->device));
        RT_TRY(drain(s));
        const uint32_t n = s->ring_pending;
        *bytes = (size_t)n * 2 * sizeof(float);
        if (capacity) {
            if (capacity < *bytes) return fail(RT_ERR_INVALID_ARGUMENT, "buffer too small");
            float *o = static_cast<float *>(dst);
            const uint32_t first = (s->ring_head + rt_scene::RING - n) % rt_scene::RING;
            for (uint32_t j = 0; j < n; j++) {
                const uint32_t slot = (first + j) % rt_scene::RING;
                HIP_TRY(hipEventElapsedTime(&o[2 * j], s->ring_start[first], s->ring_start[slot]));
                HIP_TRY(hipEventElapsedTime(&o[2 * j + 1], s->ring_start[first], s->ring_stop[slot]));
            }
        }
        return RT_OK;
    } else if (k == "instances") {
        // GPU-built frames: the instance records the GPU computed for the current frame, in instance order,
        // 45 floats each: inverse, forward, inverse-transpose rows 1-3 (12 each), transformed box, centroid
        if (!s->built || !s->gpu_tlas()) return fail(RT_ERR_UNSUPPORTED, "instance records are computed on the GPU for RT_BUILD_LBVH only");
        HIP_TRY(hipSetDevice(s->device));
        RT_TRY(drain(s));
        const size_t n = s->inst.size();
        *bytes = n * 45 * sizeof(float);
        if (capacity) {
            const uint8_t *fd = s->frame_dev[s->active];
            std::vector<InstHot> hot;
            std::vector<InstCold> cold;
            std::vector<float> tbox, tcent;
            HIP_TRY(read_back(hot, reinterpret_cast<const InstHot *>(fd + s->off_hot), n));
            HIP_TRY(read_back(cold, reinterpret_cast<const InstCold *>(fd + s->off_cold), n));
            HIP_TRY(read_back(tbox, reinterpret_cast<const float *>(fd + s->off_tbox), 6 * n));
            HIP_TRY(read_back(tcent, reinterpret_cast<const float *>(fd + s->off_tcent), 4 * n));
            std::vector<float> outv(n * 45);
            for (size_t i = 0; i < n; i++) {
                float *o = outv.data() + 45 * i;
                std::memcpy(o, hot[i].inv, 12 * sizeof(float));
                std::memcpy(o + 12, cold[i].fwd, 12 * sizeof(float));
                std::memcpy(o + 24, cold[i].nrm, 12 * sizeof(float));
                std::memcpy(o + 36, tbox.data() + 6 * i, 6 * sizeof(float));
                std::memcpy(o + 42, tcent.data() + 4 * i, 3 * sizeof(float));
            }
            std::memcpy(dst, outv.data(), std::min(capacity, *bytes));
        }
        return RT_OK;
    } else if (k == "blas_pairs" || k == "blas_quads" || k == "blas_roots") {
        // RT_BUILD_LBVH: the forest as built on the GPU (NodePair / NodeQuad / TreeRoot records, layout.hpp)
        if (!s->built || !s->gpu_tlas()) return fail(RT_ERR_UNSUPPORTED, "raw BLAS records are exported for RT_BUILD_LBVH only");
        HIP_TRY(hipSetDevice(s->device));
        RT_TRY(drain(s));
        const void *from = k == "blas_pairs" ? (const void *)s->blas_pairs.p
                                             : (k == "blas_quads" ? (const void *)s->blas_quads.p : (const void *)s->blas_roots.p);
        *bytes = k == "blas_roots" ? s->blas_roots.n * sizeof(TreeRoot)
                                   : s->blas_pair_count * (k == "blas_pairs" ? sizeof(NodePair) : sizeof(NodeQuad));
        if (capacity && *bytes) HIP_TRY(hipMemcpy(dst, from, std::min(capacity, *bytes), hipMemcpyDeviceToHost));
        return RT_OK;
    } else if (k == "leaf_prims") {
        // caller triangle index of every leaf-ordered triangle slot (TriCold::orig_index): BLAS b owns
        // the slots [slot_base, slot_base + count) of its primitives, in leaf order
        HIP_TRY(hipSetDevice(s->device));
        RT_TRY(drain(s));
        const bool raw = s->raw_shading();             // the index rides in TriHot::pad0 (option "cold_records" 0)
        const size_t n = s->tri_hot.n;
        *bytes = n * sizeof(uint32_t);
        if (capacity && n) {
            const size_t m = std::min(capacity / sizeof(uint32_t), n);
            const uint8_t *src0 = raw ? reinterpret_cast<const uint8_t *>(s->tri_hot.p) + offsetof(TriHot, pad0)
                                      : reinterpret_cast<const uint8_t *>(s->tri_cold.p) + offsetof(TriCold, orig_index);
            HIP_TRY(hipMemcpy2D(dst, sizeof(uint32_t), src0, raw ? sizeof(TriHot) : sizeof(TriCold), sizeof(uint32_t), m,
                                hipMemcpyDeviceToHost));
        }
        return RT_OK;
    } else if (k == "unit_cost" || k == "unit_order") {
        const int q = s->last_lane;
        const size_t units = s->sched_sig[q][0];
        src = k == "unit_cost" ? s->unit_cost[q].p + units : s->unit_order[q].p;
        size = s->sched_valid[q] ? units * (k == "unit_cost" ? 1 : 4) * sizeof(uint32_t) : 0;
    } else {
        return fail(RT_ERR_INVALID_ARGUMENT, "unknown debug buffer " + k);
    }
    if (!src || size == 0) return fail(RT_ERR_STATE, "debug buffer " + k + " not recorded (set the option first)");
    HIP_TRY(hipSetDevice(s->device));
    RT_TRY(drain(s));
    if (capacity) HIP_TRY(hipMemcpy(dst, src, capacity < size ? capacity : size, hipMemcpyDeviceToHost));
    *bytes = size;
    return RT_OK;
}

static void fill_stats(rt_stats *st, const unsigned long long *c) {
    std::memset(st, 0, sizeof *st);
    st->rays = c[CNT_RAYS];
    st->pixels = c[CNT_PIXELS];
    st->aabb_tests = 2ull * c[CNT_PAIRS];
    st->triangle_tests = c[CNT_TRI];
    st->sphere_quad_tests = c[CNT_SPHQUAD];
    st->quad_tests = c[CNT_QUAD];
    st->instance_visits = c[CNT_INST];
    st->hits = c[CNT_HITS];
}

rt_status rt_scene_collect(rt_scene *s, rt_stats *acc, float *kernel_ms, uint32_t capacity, uint32_t *count) {
    if (!s) return fail(RT_ERR_INVALID_ARGUMENT, "null scene");
    if (!s->built) return fail(RT_ERR_STATE, "rt_scene_build has not been called");
    HIP_TRY(hipSetDevice(s->device));
    RT_TRY(drain(s));
    HIP_TRY(hipMemcpy(s->counters_host, s->counters, rt_scene::NLANE * CNT_NUM * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    unsigned long long sum[CNT_NUM] = {};
    for (int l = 0; l < rt_scene::NLANE; l++)          // lanes whose block belongs to the current epoch
        if (s->lane_epoch[l] == s->cnt_epoch)
            for (uint32_t k = 0; k < CNT_NUM; k++) sum[k] += s->counters_host[(size_t)l * CNT_NUM + k];
    if (acc) fill_stats(acc, sum);
    // collected: the next KEEP_COUNTERS frames accumulate from zero (every block is clear and current)
    HIP_TRY(hipMemset(s->counters, 0, rt_scene::NLANE * CNT_NUM * sizeof(unsigned long long)));
    for (uint64_t &e : s->lane_epoch) e = s->cnt_epoch;
    const uint32_t n = s->ring_pending;
    uint32_t written = 0;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t slot = (s->ring_head + rt_scene::RING - n + k) % rt_scene::RING;
        float ms = 0.0f;
        HIP_TRY(hipEventElapsedTime(&ms, s->ring_start[slot], s->ring_stop[slot]));
        if (kernel_ms && written < capacity) kernel_ms[written] = ms;
        written++;
    }
    if (count) *count = written < capacity ? written : capacity;
    s->ring_pending = 0;
    return RT_OK;
}

rt_status rt_scene_update_triangles(rt_scene *s, size_t first, size_t count, const rt_triangle *tris) {
    if (!s || (count && !tris)) return fail(RT_ERR_INVALID_ARGUMENT, "null argument");
    if (!s->built) return fail(RT_ERR_STATE, "rt_scene_build has not been called");
    if (s->build_mode != RT_BUILD_LBVH) return fail(RT_ERR_UNSUPPORTED, "triangle updates need RT_BUILD_LBVH");
    if (first > s->tris.size() || count > s->tris.size() - first) return fail(RT_ERR_INVALID_ARGUMENT, "triangle range out of bounds");
    if (count == 0) return RT_OK;
    bool ok = true;
    for (size_t k = 0; k < count; k++) material_slot(s, tris[k].material_type, tris[k].material_index, ok);
    if (!ok) return fail(RT_ERR_INVALID_ARGUMENT, "triangle references a material out of range");
    HIP_TRY(hipSetDevice(s->device));
    // no drain: the copy is ordered behind the scene stream's pending BLAS builds (the next build, which the frame
    // update enqueues after it, reads the new triangles); with raw_shading() traces read raw_tris at their hits too,
    // so it also waits for every lane's last trace (and the last synchronous one)
    if (s->ev_raw_staged) RT_TRY(wait_event(s, s->ev_raw_staged));      // the previous staged copy is done
    else HIP_TRY(hipEventCreateWithFlags(&s->ev_raw_staged, hipEventDisableTiming));
    if (count > s->raw_stage_cap) {
        if (s->raw_stage) HIP_TRY(hipHostFree(s->raw_stage));
        s->raw_stage = nullptr;
        s->raw_stage_cap = 0;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&s->raw_stage), count * sizeof(rt_triangle), hipHostMallocDefault));
        s->raw_stage_cap = count;
    }
    std::memcpy(s->raw_stage, tris, count * sizeof(rt_triangle));
    std::memcpy(s->tris.data() + first, tris, count * sizeof(rt_triangle));
    if (s->raw_shading()) {
        if (s->r_done) HIP_TRY(hipStreamWaitEvent(s->stream, s->r_done, 0));
        for (int q = 0; q < rt_scene::NLANE; q++)
            if (s->r_lane[q]) HIP_TRY(hipStreamWaitEvent(s->stream, s->r_lane[q], 0));
    }
    HIP_TRY(hipMemcpyAsync(s->raw_tris.p + first, s->raw_stage, count * sizeof(rt_triangle), hipMemcpyHostToDevice, s->stream));
    HIP_TRY(extract_tri_verts(s->raw_tris.p, s->raw_verts.p, first, count, s->stream));
    HIP_TRY(hipEventRecord(s->ev_raw_staged, s->stream));
    // instance boxes derived from the triangles (RenderPin.cu:124-139); VTK-style bounds stay as given
    for (size_t i = 0; i < s->inst.size(); i++) {
        InstState &in = s->inst[i];
        const rt_instance_desc &id = s->inst_desc[i];
        if (in.ptype != RT_PRIM_TRIANGLE || id.has_local_bounds) continue;
        if ((size_t)in.pindex + in.pcount <= first || in.pindex >= first + count) continue;
        hm::Box bb = prim_box(s, in.ptype, in.pindex);
        double c[3] = {0, 0, 0};
        for (uint32_t k = 0; k < in.pcount; k++) {
            if (k) bb = hm::Box::merge(bb, prim_box(s, in.ptype, in.pindex + k));
            const hm::V3 pc = prim_centroid(s, in.ptype, in.pindex + k);
            for (int a = 0; a < 3; a++) c[a] += pc[a];
        }
        in.box = bb;
        in.centroid = in.pcount == 1 ? prim_centroid(s, in.ptype, in.pindex)
                                     : hm::v3((float)(c[0] / in.pcount), (float)(c[1] / in.pcount), (float)(c[2] / in.pcount));
        instance_update(in, in.x);
        if (s->gpu_tlas()) s->inst_dirty[i] = rt_scene::ALL_BLOCKS;     // the GPU copies of its local box
    }
    for (size_t g = 0; g < s->groups.size(); g++) {   // option "group" (LBVH): the union of the members' boxes
        InstGroup &G = s->groups[g];
        double c[3] = {0, 0, 0};
        for (size_t k = 0; k < G.members.size(); k++) {
            const InstState &m = s->inst[G.members[k]];
            G.st.box = k ? hm::Box::merge(G.st.box, m.box) : m.box;
            for (int a = 0; a < 3; a++) c[a] += m.centroid[a];
        }
        G.st.centroid = hm::v3((float)(c[0] / G.members.size()), (float)(c[1] / G.members.size()), (float)(c[2] / G.members.size()));
        if (s->gpu_tlas()) s->inst_dirty[s->inst.size() + g] = rt_scene::ALL_BLOCKS;
    }
    s->blas_dirty = true;
    return RT_OK;
}

rt_status rt_scene_update_instances(rt_scene *s, size_t first, size_t count, const rt_instance_desc *d) {
    if (!s || (count && !d)) return fail(RT_ERR_INVALID_ARGUMENT, "null argument");
    if (!s->built) return fail(RT_ERR_STATE, "rt_scene_build has not been called");
    if (first > s->inst.size() || count > s->inst.size() - first) return fail(RT_ERR_INVALID_ARGUMENT, "instance range out of bounds");
    for (size_t k = 0; k < count; k++) {
        const rt_instance_desc &o = s->inst_desc[first + k], &n = d[k];
        if (o.primitive_type != n.primitive_type || o.primitive_index != n.primitive_index ||
            o.primitive_count != n.primitive_count)
            return fail(RT_ERR_INVALID_ARGUMENT, "an instance update may not change its primitives (type / index / count)");
    }
    for (size_t k = 0; k < count; k++) {
        const size_t i = first + k;
        s->inst_desc[i] = d[k];
        InstState &in = s->inst[i];
        if (d[k].has_local_bounds) {                                          // VTKReader.cu:204-209
            in.box = hm::Box::from_ranges({d[k].local_bounds[0], d[k].local_bounds[1]}, {d[k].local_bounds[2], d[k].local_bounds[3]},
                                          {d[k].local_bounds[4], d[k].local_bounds[5]});
            in.centroid = hm::of(d[k].local_centroid);
        }
        instance_update(in, d[k].xform);
        if (s->gpu_tlas()) s->inst_dirty[i] = rt_scene::ALL_BLOCKS;
        // option "group": the group's box and transform were taken at the build; its members go back to
        // their own TLAS items for good
        if (s->group_of[i]) s->groups[s->group_of[i] - 1].valid = false;
    }
    return RT_OK;
}

rt_status rt_synchronize(rt_scene *s) {
    if (!s) return fail(RT_ERR_INVALID_ARGUMENT, "null scene");
    HIP_TRY(hipSetDevice(s->device));
    RT_TRY(drain(s));
    if (s->r_done) RT_TRY(wait_event(s, s->r_done));
    return RT_OK;
}

void rt_scene_destroy(rt_scene *s) { delete s; }

rt_status rt_scene_get_info(const rt_scene *s, rt_scene_info *info) {
    if (!s || !info) return fail(RT_ERR_INVALID_ARGUMENT, "null argument");
    std::memset(info, 0, sizeof *info);
    info->blas_count = s->blas_own;     // per-instance BLASes (the groups' merged ones are not counted)
    info->overlap_lanes = s->lanes;
    info->stage_depth = (uint32_t)s->stage_depth;
    info->blas_node_pairs = s->blas_pair_count;
    info->blas_leaves = s->blas_leaf_count;
    info->tlas_node_pairs = s->tlas_flat.pairs.size();
    if (s->gpu_tlas() && s->built) {                 // GPU-built TLAS: read the last frame's count / root
        HIP_TRY(hipSetDevice(s->device));
        RT_TRY(wait_frame_block(const_cast<rt_scene *>(s)));   // the frame's TLAS may have been built on a lane stream
        uint32_t np = 0;
        TreeRoot root{};
        HIP_TRY(hipMemcpy(&np, s->gpu_counts.p + 2 + s->active, sizeof np, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(&root, s->frame_dev[s->active] + s->off_root, sizeof root, hipMemcpyDeviceToHost));
        info->tlas_node_pairs = np;
        info->tlas_height = root.height;
    }
    info->device_bytes = s->blas_pairs.n * sizeof(NodePair) + s->tri_hot.n * sizeof(TriHot) + s->tri_cold.n * sizeof(TriCold) +
                         s->sph_hot.n * sizeof(SphereHot) + s->sph_cold.n * sizeof(PrimCold) +
                         s->quad_hot.n * sizeof(QuadHot) + s->quad_cold.n * sizeof(PrimCold) +
                         s->materials.n * sizeof(float) + 2 * s->frame_block + s->out_rgba.n + s->out_rgb.n * sizeof(float) +
                         s->raw_tris.n * sizeof(rt_triangle) + s->raw_sph.n * sizeof(rt_sphere) +
                         s->raw_quad.n * sizeof(rt_parallelogram) + s->blas_quads.n * sizeof(NodeQuad) +
                         s->raw_verts.n * sizeof(float);
    for (const auto &sp : s->spare)      // the spare BLAS sets of per-frame rebuilds ("blas_sets")
        info->device_bytes += sp.pairs.n * sizeof(NodePair) + sp.quads.n * sizeof(NodeQuad) + sp.roots.n * sizeof(TreeRoot) +
                              sp.tri_hot.n * sizeof(TriHot) + sp.tri_cold.n * sizeof(TriCold) +
                              sp.sph_hot.n * sizeof(SphereHot) + sp.sph_cold.n * sizeof(PrimCold) +
                              sp.quad_hot.n * sizeof(QuadHot) + sp.quad_cold.n * sizeof(PrimCold);
    if (s->blas_builder) info->device_bytes += s->blas_builder->workspace_bytes();   // incl. the staged TriHot records
    if (s->tlas_builder) info->device_bytes += s->tlas_builder->workspace_bytes();
    info->width = s->width; info->height = s->height;
    info->sqrt_sample_count = s->cam.sqrt_s;
    info->ray_trace_depth = s->cam.depth;
    if (!s->gpu_tlas()) info->tlas_height = s->tlas_flat.height;
    info->blas_height_max = s->max_blas_height;
    return RT_OK;
}

static void export_tree(const Tree &t, float *boxes, uint32_t *ci) {
    for (size_t i = 0; i < t.nodes.size(); i++) {
        if (boxes) t.nodes[i].box.store(boxes + 6 * i);
        if (ci) { ci[2 * i] = t.nodes[i].count; ci[2 * i + 1] = t.nodes[i].index; }
    }
}

}  // extern "C"

// Reference node form (BLASNode/TLASNode arrays, children adjacent, DFS leaf order) of a tree held in
// the node-pair layout: used to export GPU-built trees.
static Tree tree_from_pairs(const TreeRoot &root, const std::vector<NodePair> &pairs, uint32_t slot_base,
                            const std::vector<uint32_t> &item_of_slot) {
    Tree t;
    if (root.ref == 0xFFFFFFFFu) return t;
    auto box_of = [](const float *b) { return hm::Box{{{b[0], b[1]}, {b[2], b[3]}, {b[4], b[5]}}}; };
    struct Work { uint32_t ref; hm::Box box; uint32_t node; };
    std::vector<Work> todo{{root.ref, box_of(root.box), 0u}};
    t.nodes.push_back(TreeNode{});
    while (!todo.empty()) {
        const Work w = todo.back();
        todo.pop_back();
        t.nodes[w.node].box = w.box;
        if (w.ref & REF_LEAF) {
            const uint32_t start = ref_leaf_start(w.ref) - slot_base, cnt = ref_leaf_count(w.ref);
            t.nodes[w.node].count = cnt;
            t.nodes[w.node].index = (uint32_t)t.refs.size();
            for (uint32_t k = 0; k < cnt; k++) t.refs.push_back(item_of_slot[start + k]);
            continue;
        }
        const NodePair &P = pairs[w.ref & REF_INDEX_MASK];
        const uint32_t left = (uint32_t)t.nodes.size();
        t.nodes.resize(left + 2);
        t.nodes[w.node].count = 0;
        t.nodes[w.node].index = left;
        todo.push_back({P.ref1, box_of(P.c1), left + 1});
        todo.push_back({P.ref0, box_of(P.c0), left});
    }
    return t;
}


extern "C" {

rt_status rt_scene_export_blas(const rt_scene *s, uint32_t b, float *boxes, uint32_t *ci, uint32_t *refs,
                               uint32_t *n_nodes, uint32_t *n_prims) {
    if (!s) return fail(RT_ERR_INVALID_ARGUMENT, "null scene");
    if (!s->built || b >= s->blas.size()) return fail(RT_ERR_INVALID_ARGUMENT, "no such BLAS");
    Tree gpu_tree;
    if (s->build_mode == RT_BUILD_LBVH) {
        HIP_TRY(hipSetDevice(s->device));
        HIP_TRY(hipStreamSynchronize(s->stream));
        std::vector<NodePair> pairs;
        std::vector<TreeRoot> roots;
        if (s->seg_of_blas[b] == 0xFFFFFFFFu)
            return fail(RT_ERR_STATE, "this BLAS is not built: its instance group is one BLAS (option \"group\")");
        HIP_TRY(read_back(pairs, s->blas_pairs.p, s->blas_pair_count));
        HIP_TRY(read_back(roots, s->blas_roots.p, s->blas_roots.n));
        const uint32_t type = s->blas[b].type;
        std::vector<uint32_t> orig;
        if (type == RT_PRIM_TRIANGLE && s->raw_shading()) {
            std::vector<TriHot> h;
            HIP_TRY(read_back(h, s->tri_hot.p, s->tri_hot.n));
            for (const TriHot &x : h) {
                uint32_t v;
                std::memcpy(&v, &x.pad0, sizeof v);
                orig.push_back(v);
            }
        } else if (type == RT_PRIM_TRIANGLE) {
            std::vector<TriCold> c;
            HIP_TRY(read_back(c, s->tri_cold.p, s->tri_cold.n));
            for (const TriCold &x : c) orig.push_back(x.orig_index);
        } else {
            std::vector<PrimCold> c;
            HIP_TRY(read_back(c, type == RT_PRIM_SPHERE ? s->sph_cold.p : s->quad_cold.p,
                              type == RT_PRIM_SPHERE ? s->sph_cold.n : s->quad_cold.n));
            for (const PrimCold &x : c) orig.push_back(x.orig_index);
        }
        gpu_tree = tree_from_pairs(roots[s->seg_of_blas[b]], pairs, 0, orig);
    }
    const Tree &t = s->build_mode == RT_BUILD_LBVH ? gpu_tree : s->blas[b].tree;
    if (n_nodes) *n_nodes = (uint32_t)t.nodes.size();
    if (n_prims) *n_prims = (uint32_t)t.refs.size();
    export_tree(t, boxes, ci);
    if (refs) std::memcpy(refs, t.refs.data(), t.refs.size() * sizeof(uint32_t));
    return RT_OK;
}

rt_status rt_scene_export_tlas(const rt_scene *s, float *boxes, uint32_t *ci, uint32_t *refs, uint32_t *n_nodes,
                               uint32_t *n_refs) {
    if (!s) return fail(RT_ERR_INVALID_ARGUMENT, "null scene");
    if (!s->built) return fail(RT_ERR_STATE, "rt_scene_build has not been called");
    Tree gpu_tree;
    if (s->gpu_tlas()) {
        HIP_TRY(hipSetDevice(s->device));
        RT_TRY(wait_frame_block(const_cast<rt_scene *>(s)));   // the frame's TLAS may have been built on a lane stream
        const uint8_t *fd = s->frame_dev[s->active];
        TreeRoot root{};
        std::vector<NodePair> pairs;
        std::vector<uint32_t> slots;
        HIP_TRY(hipMemcpy(&root, fd + s->off_root, sizeof root, hipMemcpyDeviceToHost));
        const size_t nrec = s->inst.size() + s->groups.size();
        HIP_TRY(read_back(pairs, reinterpret_cast<const NodePair *>(fd + s->off_pairs), nrec));
        HIP_TRY(read_back(slots, reinterpret_cast<const uint32_t *>(fd + s->off_slots), nrec));
        gpu_tree = tree_from_pairs(root, pairs, 0, slots);
    }
    const Tree &t = s->gpu_tlas() ? gpu_tree : s->tlas;
    if (n_nodes) *n_nodes = (uint32_t)t.nodes.size();
    if (n_refs) *n_refs = (uint32_t)t.refs.size();
    export_tree(t, boxes, ci);
    if (refs) std::memcpy(refs, t.refs.data(), t.refs.size() * sizeof(uint32_t));
    return RT_OK;
}

// updateInstance (src/Global/Main.cu:6-42)
void rt_demo_update(void *user, rt_xform *x, size_t n, uint64_t frame) {
    (void)user;
    const float ic[3] = {0.0f, 2.0f, 0.0f};
    const float radius = 2.0f, speed = 0.02f;
    const float angle = (float)frame * speed;
    const float c1[3] = {ic[0] + radius * std::cos(angle) * 1.5f, ic[1] + radius * std::sin(angle) * std::cos(angle),
                         ic[2] + radius * std::sin(angle) * 1.5f};
    const float c2[3] = {-c1[0], c1[1], -c1[2]};
    const float c3[3] = {-c1[0], c1[1] + 5.0f, c1[2]};
    const float rot = (float)frame * 0.4f;
    const rt_xform t[5] = {
        {{0.0f, -1000.0f, 0.0f}, {0.0f, 0.0f, 0.0f}, {1.0f, 1.0f, 1.0f}},
        {{c1[0], c1[1], c1[2]}, {0.0f, 0.0f, 0.0f}, {1.0f, 1.0f, 1.0f}},
        {{-5.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}, {1.0f, 1.0f, 1.0f}},
        {{c2[0], c2[1], c2[2]}, {rot, rot, rot}, {3.0f, 3.0f, 3.0f}},
        {{c3[0], c3[1], c3[2]}, {0.0f, 0.0f, 0.0f}, {1.0f, 1.0f, 1.0f}},
    };
    for (size_t i = 0; i < n && i < 5; i++) x[i] = t[i];
}

}  // extern "C"
