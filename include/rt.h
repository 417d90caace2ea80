/*
 * rt.h — C ABI of the MI355X-native trace path (drop-in for the reference's
 * Scene / Camera / render(framebuffer) lifecycle).
 *
 * The reference has no FFI; its boundary is the static C++ class `Renderer`
 * (include/Global/Renderer.cuh:109-146) plus the kernel contract
 * `render(const TraverseData*, cudaSurfaceObject_t)` with a `__constant__ Camera`
 * (include/Global/RendererImpl.cuh:196-199).  Every entry point below names the
 * reference call it replaces.  All types are plain C: no torch, no HIP types.
 *
 * Conventions
 *  - Every call returns rt_status; on failure rt_last_error() returns a
 *    thread-local message.  The library never exit()s (the reference exits with
 *    -200 on any CUDA error, src/Global/Global.cu:34-41).
 *  - A scene is not thread-safe; use one scene per host thread (the reference
 *    drives everything from one thread, src/Global/Renderer.cu:180-366).
 *  - Framebuffer layout matches the reference surface: row-major W x H RGBA8,
 *    row 0 = bottom of the image (viewport origin bottom-left,
 *    src/Global/RenderPin.cu:91-92).
 */
#ifndef RT_H
#define RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: rt_stats gained update_wait_ms; rt_comm_* / rt_slab_tiles / rt_tile_pixels / rt_scene_detach_comm;
 *    rt_camera_move / rt_frame_pacer_* / rt_comm_set_timeout (round 3)
 * 3: rt_scene_info gained overlap_lanes / stage_depth; "overlap" -1 = library-picked lanes on library streams */
#define RT_ABI_VERSION 3u

typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID_ARGUMENT = 1,
    RT_ERR_DEVICE = 2,          /* HIP runtime error, or no GPU present        */
    RT_ERR_OUT_OF_MEMORY = 3,
    RT_ERR_STATE = 4,           /* call out of lifecycle order                 */
    RT_ERR_UNSUPPORTED = 5
} rt_status;

/* include/Basic/BasicTypes.cuh:9-11 */
typedef enum rt_primitive_type {
    RT_PRIM_SPHERE = 0,
    RT_PRIM_PARALLELOGRAM = 1,
    RT_PRIM_TRIANGLE = 2
} rt_primitive_type;

/* include/Basic/BasicTypes.cuh:14-16 */
typedef enum rt_material_type {
    RT_MAT_ROUGH = 0,
    RT_MAT_METAL = 1
} rt_material_type;

typedef struct rt_vec3 { float x, y, z; } rt_vec3;

/* Sphere(MaterialType, size_t, Point3 center, float radius) — include/Geometry/Sphere.cuh:27 */
typedef struct rt_sphere {
    rt_vec3 center;
    float radius;
    uint32_t material_type;
    uint32_t material_index;
} rt_sphere;

/* Parallelogram(MaterialType, size_t, q, u, v) — include/Geometry/Parallelogram.cuh:26-39 */
typedef struct rt_parallelogram {
    rt_vec3 q, u, v;
    uint32_t material_type;
    uint32_t material_index;
} rt_parallelogram;

/* Triangle(MaterialType, size_t, vertexes[, vertexNormals]) — include/Geometry/Triangle.cuh:26-46.
 * has_normals = 0 selects the 3-vertex constructor (all three normals = unit(e1 x e2)). */
typedef struct rt_triangle {
    rt_vec3 vertex[3];
    rt_vec3 normal[3];
    uint32_t material_type;
    uint32_t material_index;
    uint32_t has_normals;
    uint32_t reserved;
} rt_triangle;

/* Rough{albedo} — include/Material/Rough.cuh:11-12; Metal{albedo, fuzz} — include/Material/Metal.cuh:11-13 */
typedef struct rt_rough { rt_vec3 albedo; } rt_rough;
typedef struct rt_metal { rt_vec3 albedo; float fuzz; } rt_metal;

/* Instance::updateTransformArguments(shift, rotate(degrees, x->y->z), scale)
 * — src/AS/Instance.cu:4-17, src/Util/Matrix.cu:183-249. */
typedef struct rt_xform {
    rt_vec3 shift;
    rt_vec3 rotate_deg;
    rt_vec3 scale;
} rt_xform;

/* One entry of the reference instance map {PrimitiveType, primitiveIndex}
 * (src/Global/Main.cu:93-99) plus the fields VTK instances carry
 * (src/Global/VTKReader.cu:204-214).
 *  primitive_count == 0 -> single-primitive instance; local bounds / centroid come
 *    from the primitive (src/Global/RenderPin.cu:124-139).
 *  primitive_count  > 0 -> a group of primitive_count primitives of one type starting at
 *    primitive_index; has_local_bounds = 1 supplies the pre-transform bounds/centroid the
 *    VTK reader would (bounds = [xmin,xmax,ymin,ymax,zmin,zmax]); has_local_bounds = 0
 *    uses the union of the primitive boxes and the mean of primitive centroids (extension).
 */
typedef struct rt_instance_desc {
    uint32_t primitive_type;
    uint32_t primitive_index;
    uint32_t primitive_count;
    uint32_t has_local_bounds;
    float local_bounds[6];
    rt_vec3 local_centroid;
    rt_xform xform;           /* initial transform (used when no update callback is set) */
} rt_instance_desc;

/* Per-frame instance update, replaces
 * void (*updateInstances)(Instance*, size_t instanceCount, size_t frameCount)
 * (include/Global/Renderer.cuh:94).  The callback rewrites the (shift, rotate, scale)
 * triple of each instance; the library then recomputes matrices and bounds exactly like
 * Instance::updateTransformArguments and rebuilds the TLAS (src/Global/Renderer.cu:269-276). */
typedef void (*rt_update_fn)(void *user, rt_xform *xforms, size_t instance_count, uint64_t frame);

/* GeometryData + MaterialData + instance map (include/Global/Renderer.cuh:33-43,
 * src/Global/Renderer.cu:9-121).  The caller keeps ownership; the library copies. */
typedef struct rt_scene_desc {
    const rt_sphere *spheres;               size_t sphere_count;
    const rt_parallelogram *parallelograms; size_t parallelogram_count;
    const rt_triangle *triangles;           size_t triangle_count;
    const rt_rough *roughs;                 size_t rough_count;
    const rt_metal *metals;                 size_t metal_count;
    const rt_instance_desc *instances;      size_t instance_count;
    rt_update_fn update;
    void *update_user;
} rt_scene_desc;

/* CameraInput — include/Global/Renderer.cuh:54-64 (field for field). */
typedef struct rt_camera_input {
    rt_vec3 background;
    rt_vec3 center;
    rt_vec3 target;
    float fov;                 /* horizontal field of view, degrees */
    rt_vec3 up;
    float focus_disk_radius;
    float sample_range;        /* carried, unused (as in the reference) */
    uint32_t sample_count;     /* traced samples = floor(sqrt(n))^2 (RenderPin.cu:93) */
    uint32_t ray_trace_depth;
} rt_camera_input;

/* BVH build policy.  COMPAT_MEDIAN restates BLAS::constructBLAS / TLAS::constructTLAS
 * (src/AS/BLAS.cu:4-117, src/AS/TLAS.cu:4-129): top-down median split on a pseudo-random
 * axis, leaf <= 4 primitives (BLAS) / <= 2 instances (TLAS).  The reference draws the axis
 * from std::mt19937(random_device); here the axis stream is a pinned function of `seed`
 * so builds are reproducible, and centroid ties are broken by primitive index. */
typedef enum rt_build_mode {
    RT_BUILD_COMPAT_MEDIAN = 0,
    /* Surface-area-heuristic BLAS and per-frame TLAS (leaf <= 4 items).  Different trees than the
     * reference: hits agree except where two surfaces tie within the 1e-6 window. */
    RT_BUILD_SAH = 1,
    /* GPU builder: every BLAS and the per-frame TLAS are linear BVHs
     * (30-bit Morton order per tree, Karras radix-tree hierarchy, subtrees of <= 4 primitives /
     * <= 2 instances collapsed into leaves) built by HIP kernels on the scene's stream.  The host
     * still runs the update callback and the instance matrices (Instance.cu:4-17); the TLAS build
     * never blocks the host.  With rt_scene_set_option("rebuild", 1) every BLAS is rebuilt on the
     * GPU each frame (config C5's per-frame rebuild); rt_scene_update_triangles marks them stale. */
    RT_BUILD_LBVH = 2
} rt_build_mode;

typedef enum rt_render_flags {
    RT_RENDER_EXACT = 1u << 0,        /* bit-faithful arithmetic (IEEE division, no FMA) */
    RT_RENDER_COUNT_WORK = 1u << 1,   /* fill rt_stats work counters (slower)              */
    RT_RENDER_NO_SYNC = 1u << 2,      /* return after enqueue (device outputs only)        */
    RT_RENDER_SKIP_UPDATE = 1u << 3,  /* do not run the instance update / TLAS rebuild (with
                                         "overlap": the frame waits for the whole launch that
                                         uploaded its frame block, i.e. it serialises with it);
                                         RT_ERR_STATE after rt_scene_update_triangles until a
                                         frame has run its update (which rebuilds the BLASes) */
    RT_RENDER_KEEP_COUNTERS = 1u << 4 /* accumulate device counters (see rt_scene_collect); a
                                         synchronous frame with "overlap" then waits for every lane
                                         and reports the totals over all lanes                 */
} rt_render_flags;

/* Per-call options for rt_render.  Zero-initialise, then set what you need. */
typedef struct rt_render_opts {
    uint64_t frame_seed;       /* replaces clock64() in curand_init (Kernel.cu:114); 0 -> 0x5EED */
    uint32_t flags;            /* rt_render_flags */
    /* Screen-tile sharding (multi-GPU): the frame is cut into tile_w x tile_h tiles in
     * row-major tile order; this call renders tiles t with t % tile_count == tile_rank.
     * tile_count == 0 renders the whole frame into the frame-layout outputs.
     * With tile_count > 0, device outputs are written tile-compact: local tile k occupies
     * pixels [k*tile_w*tile_h, (k+1)*tile_w*tile_h), row-major inside the tile. */
    uint32_t tile_w, tile_h;
    uint32_t tile_rank, tile_count;
    /* Optional device outputs (hipMalloc'd / torch device memory on this scene's GPU). */
    void *rgba8_device;        /* uchar4 per pixel */
    void *rgb32_device;        /* 3 floats per pixel, linear average before gamma */
    void *stream;              /* hipStream_t to enqueue on; NULL -> the scene's stream, and when a device
                                * output is given the frame is ordered after the caller's null-stream work
                                * enqueued before the call, and that null stream's later work after the frame */
} rt_render_opts;

typedef struct rt_stats {
    uint64_t rays;             /* closest-hit traversals (one per TLAS::hit call, Kernel.cu:68) */
    uint64_t pixels;
    uint64_t aabb_tests;       /* filled with RT_RENDER_COUNT_WORK */
    uint64_t triangle_tests;
    uint64_t sphere_quad_tests;  /* sphere + parallelogram tests                                */
    uint64_t quad_tests;         /* parallelogram tests                                         */
    uint64_t instance_visits;
    uint64_t hits;               /* closest hits found (rays - misses)                          */
    double kernel_ms;          /* device time of the trace kernel (HIP events)             */
    double frame_ms;           /* host wall time of the call                               */
    double update_ms;          /* host time of instance update + TLAS rebuild + upload     */
    double update_wait_ms;     /* part of update_ms blocked on the GPU (a staging buffer still
                                  read by an earlier frame's copy); the rest is host compute */
} rt_stats;
/* sizeof(rt_stats) == 96 on LP64 (RT_ABI_VERSION 3) */

/* Closest-hit record for rt_trace_rays (per-ray parity tests). */
typedef struct rt_hit {
    float t;
    uint32_t instance;         /* 0xFFFFFFFF = miss */
    uint32_t primitive_type;
    uint32_t primitive_index;  /* index into the caller's primitive array */
    rt_vec3 point;             /* world-space hit point   (Instance.cu:41) */
    rt_vec3 normal;            /* world-space unit normal (Instance.cu:44) */
    uint32_t material_type;
    uint32_t material_index;
} rt_hit;

typedef struct rt_scene rt_scene;

/* --- lifecycle ---------------------------------------------------------------- */

uint32_t rt_abi_version(void);
const char *rt_last_error(void);
/* Number of visible GPUs (0 when no HIP device is present). */
int rt_device_count(void);

/* Renderer::commitGeometryData + commitMaterialData + configureInstances
 * (src/Global/Renderer.cu:9-121).  Copies the description; no device work yet. */
rt_status rt_scene_create(const rt_scene_desc *desc, int device, rt_scene **out_scene);

/* Renderer::buildAccelerationStructure (src/Global/Renderer.cu:123-155): builds every BLAS
 * (deduplicated per (type, primitiveIndex), RenderPin.cu:99-201), uploads geometry, BVHs
 * and materials to HBM, and builds the frame-0 TLAS. */
rt_status rt_scene_build(rt_scene *scene, rt_build_mode mode, uint64_t seed);

/* Renderer::configureCamera (src/Global/Renderer.cu:157-178) ->
 * RendererImpl::calculateCameraProperties (src/Global/RenderPin.cu:73-95). */
rt_status rt_camera_set(rt_scene *scene, const rt_camera_input *camera,
                        uint32_t width, uint32_t height);

/* Host half of one iteration of startRender (src/Global/Renderer.cu:264-303): run the
 * instance update for `frame`, rebuild the TLAS and upload it (double-buffered). */
rt_status rt_scene_update(rt_scene *scene, uint64_t frame);

/* Device half of one iteration of startRender (src/Global/Renderer.cu:305-317) = the
 * `render` kernel (src/Global/Kernel.cu:105-147).  Unless RT_RENDER_SKIP_UPDATE is set,
 * first calls rt_scene_update(scene, frame).  Host outputs (may be NULL) receive the
 * frame after completion; device outputs are described in rt_render_opts. */
rt_status rt_render(rt_scene *scene, uint64_t frame, const rt_render_opts *opts,
                    uint8_t *rgba8_host, float *rgb32_host, rt_stats *stats);

/* Assemble tile-compact buffers gathered from `tile_count` ranks into a frame-layout RGBA8
 * device buffer (the multi-GPU gather's scatter step).  `gathered` holds tile_count slabs of
 * slab_tiles tiles each (rank r's slab = its tiles in render order, padded). */
rt_status rt_assemble_tiles(rt_scene *scene, const void *gathered_device, uint32_t slab_tiles,
                            uint32_t tile_w, uint32_t tile_h, uint32_t tile_count,
                            void *frame_rgba8_device, void *stream);

/* Number of tiles rank `tile_rank` owns for the current camera size. */
uint32_t rt_tiles_for_rank(const rt_scene *scene, uint32_t tile_w, uint32_t tile_h,
                           uint32_t tile_rank, uint32_t tile_count);

/* --- multi-GPU frames: screen tiles + RCCL gather inside the library --------------
 * One process (or thread) per GPU, each holding its own scene built from the same inputs (the
 * reference is single-GPU: Renderer.cu:305-317 launches one kernel over the whole surface).  After
 * rt_scene_attach_comm, every rt_render of the scene traces only this rank's screen tiles (tile t of
 * the row-major tile grid belongs to rank t mod world), gathers the tiles to rank 0 over RCCL (grouped
 * ncclSend / ncclRecv, xGMI) and assembles the frame there (csrc/assemble.hip), all enqueued on the
 * call's stream.  Rank 0's rgba8 outputs receive the whole frame; other ranks' output arguments are
 * ignored.  Every rank must make the same sequence of rt_render calls (with "overlap", the same lane
 * sequence).  rgb32 outputs and rt_render_opts tile fields are rejected while attached; rt_stats count
 * this rank's work.  The assembled frame is byte-identical for any world size: the RNG is keyed by the
 * global padded pixel index. */
typedef struct rt_comm_id { char internal[128]; } rt_comm_id;      /* an ncclUniqueId */

/* Rank 0 creates the id (ncclGetUniqueId) and passes it to every rank out of band. */
rt_status rt_comm_unique_id(rt_comm_id *id);
/* Collective over the `world` ranks (same id, world, tile size); world == 1 is allowed.  librccl.so.1 is
 * resolved at this call (the one already in the process, else ROCm's): single-GPU callers never need it. */
rt_status rt_scene_attach_comm(rt_scene *scene, const rt_comm_id *id, int rank, int world,
                               uint32_t tile_w, uint32_t tile_h);
rt_status rt_scene_detach_comm(rt_scene *scene);

/* Tile bookkeeping shared by the kernels and the host (no GPU needed): the largest number of tiles a
 * rank owns (slabs are padded to it), and the frame pixel of slab pixels [first, first + n) of `rank`
 * (xy[2i], xy[2i+1]; -1, -1 for pixels outside the frame). */
uint32_t rt_slab_tiles(uint32_t width, uint32_t height, uint32_t tile_w, uint32_t tile_h, uint32_t tile_count);
rt_status rt_tile_pixels(uint32_t width, uint32_t height, uint32_t tile_w, uint32_t tile_h, uint32_t tile_rank,
                         uint32_t tile_count, uint64_t first, uint64_t n, int32_t *xy);

/* Trace arbitrary world rays (origin xyz, direction xyz per ray) against the current TLAS
 * with t in [0.001, inf) and return the closest hit (TLAS::hit, src/AS/TLAS.cu:131-201).
 * RT_ERR_STATE after rt_scene_update_triangles until a frame has run its update. */
rt_status rt_trace_rays(rt_scene *scene, const float *rays_host, size_t ray_count,
                        uint32_t flags, rt_hit *hits_host);

/* The box decisions of the trace kernels on caller data, for parity tests (no scene needed): box i =
 * {xmin, xmax, ymin, ymax, zmin, zmax} (6 floats), ray i = origin xyz, direction xyz, range [0.001, tmax[i]].
 * hit[i] = 1 when the kernel the mode names keeps the box; te[i] = the entry t it orders children by (+inf on a
 * miss).  RT_BOX_REFERENCE is BoundingBox::hit (src/AS/BoundingBox.cu:34-72) as the EXACT kernel computes it; the
 * FAST modes are the reciprocal-plane slabs the persistent kernel culls with, conservative (a box the reference keeps
 * is never culled), and — in the exact-decision modes — with every decision inside their error margin re-taken with
 * the reference's slab, so they keep exactly the boxes the reference keeps. */
typedef enum rt_box_mode {
    RT_BOX_REFERENCE = 0,      /* EXACT kernel: the reference's division slab */
    RT_BOX_CULL = 1,           /* FAST single-box cull (SAH / GPU-built scenes' instance and root boxes) */
    RT_BOX_DECIDE = 2,         /* FAST single box, exact decisions (binary pairs; the reference's trees; "exact_decisions") */
    RT_BOX_QUAD_PAIR = 3,      /* FAST quad slot, pair order, exact decisions (the reference's trees; "exact_decisions") */
    RT_BOX_QUAD_GREEDY = 4     /* FAST quad slot, conservative cull (host SAH trees; GPU-built trees by default) */
} rt_box_mode;
rt_status rt_box_test(int device, const float *boxes_host, const float *rays_host, const float *tmax_host, size_t count,
                      uint32_t mode, uint8_t *hit_host, float *te_host);

/* Scene options (19 keys; every default is the measured best, so a drop-in caller sets none of them but
 * "overlap").  Unknown keys return RT_ERR_INVALID_ARGUMENT.
 * Frames and lanes:
 *   "overlap"   : L = consecutive rt_render calls cycle through L (2..8) internal lanes (work-queue heads, unit costs,
 *                 schedule); a launch waits only for the previous launch of its own lane and for its frame block, so
 *                 frame k+1's launch runs in the CUs frame k's tail leaves idle.  Frames with opts.stream NULL run on
 *                 lane streams the scene creates; a caller that passes streams cycles its own.  -1 = auto: the scene
 *                 also picks L and the staging depth per frame kind (2 lanes with a per-frame rebuild, else 8 lanes /
 *                 64 buffers for a rank's tile share, else 4).  With lanes the caller orders its own output buffers:
 *                 device outputs of NO_SYNC frames without a stream are complete once rt_synchronize returns
 *                 (default 0 = 1 lane: every launch of the scene is serialised)
 *   "stage_depth": pinned host staging buffers the per-frame upload cycles through (2..64, default 16, allocated on
 *                 first use): the host stages frame k once frame k - depth's trace is done (drains the scene)
 *   "lane_priority": the lane streams the scene creates for "overlap" frames without a caller stream: 1 (default) =
 *                 the device's highest stream priority (hardware queues of their own: full overlap at the default
 *                 GPU_MAX_HW_QUEUES of 4), 0 = normal priority
 *   "grid_pct"  : persistent grid as a percentage of the resident workgroup capacity (1..100; default 0 = auto:
 *                 100 when no other lane's launch is in flight, else 50 with up to 3 lanes and 100 / lanes + 12
 *                 with more, so several lanes' launches run side by side; a launch of >= 16 M camera paths: 100)
 * GPU-built scenes (RT_BUILD_LBVH; the builder's options are set before rt_scene_build):
 *   "rebuild"   : 1 = rebuild every BLAS on the GPU every frame (default 0)
 *   "cold_records": 1 = the GPU builder writes TriCold records (normals, material, caller index) beside TriHot;
 *                 0 = a hit reads the caller's triangle instead; -1 (default) = 1 unless "rebuild" is 1 at
 *                 rt_scene_build (same pixels either way)
 *   "blas_double": per-frame rebuilds: 1 = write a spare BLAS set and swap it in, so a frame's rebuild overlaps the
 *                 previous frames' traces (default 1; 0 = one set, a rebuild waits for every lane's trace)
 *   "blas_sets" : with "blas_double": BLAS sets cycled (2..8, default 3): frame k+1's rebuild waits only for the trace
 *                 of frame k + 1 - sets
 *   "tlas_small": 1 (default) = a GPU TLAS of at most 512 records is built by one workgroup in one launch; 0 = the
 *                 multi-kernel builder (results identical up to the tree's shape)
 *   "exact_decisions": 1 = the FAST kernel re-takes every box decision and pair-order comparison inside its slabs'
 *                 error margin with the reference's slab, as it always does on the reference's own trees, so its
 *                 frames equal the EXACT kernel's on the same trees bit for bit (C5: ~34 % slower per frame: sibling
 *                 boxes' entry t's often tie); 0 (default) = conservative culls (frames within SURVEY's bars)
 * Host-built scenes:
 *   "group"     : triangle instances with bit-identical transforms (each with a BLAS of its own) share one BLAS over
 *                 all their triangles, entered as one TLAS item while every member keeps that transform (default 1;
 *                 set before rt_scene_build; hits report the member instance; 0 = one TLAS item per instance)
 *   "gpu_tlas"  : RT_BUILD_SAH: 1 = keep the host-built SAH BLASes but compute the instance records and build the
 *                 TLAS on the GPU every frame, as RT_BUILD_LBVH does.  Set before rt_scene_build (default 0)
 *   "tlas_sah"  : RT_BUILD_SAH: 1 (default) = build the per-frame host TLAS with SAH; 0 = the reference's median
 *                 split (TLAS.cu:4-129)
 * Kernel:
 *   "kernel"    : 0 = one-thread-per-pixel grid kernel, 1 = persistent-wave megakernel (default)
 *   "wide"      : FAST persistent kernel: 1 (default) = quad trees (the reference's trees and GPU-built ones: two
 *                 binary levels per quad visited in the binary tree's order; RT_BUILD_SAH: the greedy collapse
 *                 visited by entry t), 0 = binary node pairs
 *   "fast_math" : FAST frames only: 1 = hardware reciprocal / rsq and FMA contraction in the primitive tests, transforms
 *                 and shading (about 8 % faster; 0.01-0.09 % of pixels then differ from the reference's arithmetic);
 *                 0 (default) = the reference's correctly rounded arithmetic wherever a value reaches a hit or a pixel
 *   "reorder"   : 1 (default) = each launch claims its band's 8x8 units heaviest-first, ordered by the traversal work
 *                 the lane's last recording launch measured per unit (schedule.hip); 0 = screen order.  Images are
 *                 identical either way (the RNG is keyed by pixel)
 * Debug:
 *   "timeline"  : 1 = record a per-wave timeline of each persistent launch
 *   "costmap"   : 1 = with RT_RENDER_COUNT_WORK, record per-pixel traversal steps
 * (Removed in round 6, measured defaults kept: threshold, leaf_early, queue_parts, grab, supertile, merge, split,
 * reorder_period, reserve, lds_scene, lds_blas, inst_by_slot, blas_leaf, tlas_leaf, tlas_median_leaf; removed with
 * their code as measured negative or neutral: variant, nt_store, cost_max, tlas_classes, wide_merge, scene_priority.
 * DESIGN.md §4 keeps the measurements.) */
rt_status rt_scene_set_option(rt_scene *scene, const char *key, int64_t value);

/* Debug buffers of the last launch that recorded them (synchronises the scene's stream):
 *   "timeline": 16 u64 per wave of the persistent kernel: start and end s_memrealtime (100 MHz),
 *               (HW_ID << 32) | XCC_ID, pixels finished by the wave, time the queue ran dry,
 *               traversal rounds, shade phases, queue grabs, and (diagnostic builds only) shader
 *               cycles spent refilling, descending, testing leaves and shading, descent-loop
 *               iterations, refill-loop iterations, 2 reserved;
 *   "costmap" : 1 u32 per output pixel: traversal steps (interior steps + leaf phases) of its path;
 *   "unit_cost", "unit_order": option "reorder" — per 8x8 unit, the work the lane's last launch recorded
 *               (after the next launch's schedule: the costs that schedule read), and the claim order the
 *               last launch used (band b's items start at 4 x its first unit: unit << 4 | piece << 2 | log2 pieces);
 *   "instances": RT_BUILD_LBVH or "gpu_tlas": 45 floats per instance, the records the GPU computed for the current frame
 *               (instances.hip): inverse, forward and inverse-transpose rows 1-3 (12 each), transformed box
 *               {xmin,xmax,ymin,ymax,zmin,zmax} (may be all +inf for a record kept out of the TLAS: a member of
 *               an intact instance group, option "group"), transformed centroid;
 *   "blas_pairs", "blas_quads", "blas_roots": RT_BUILD_LBVH: the GPU-built forest as NodePair / NodeQuad /
 *               TreeRoot records (csrc/layout.hpp; quad q is the 4-wide node rooted at pair q);
 *   "leaf_prims": 1 u32 per leaf-ordered triangle slot: the caller's triangle index stored there (each
 *               BLAS owns the contiguous slots of its primitives, in leaf order);
 *   "rebuild_stages": RT_BUILD_LBVH with option "timeline" set before the frame: float64 values — the last BLAS
 *               build's items, interior nodes, node pairs written, items in trees of > 2048 items, such trees, then
 *               the ms of each builder stage (prep, bounds, morton, sort, hierarchy_small, hierarchy_large, scan,
 *               emit_roots, collapse); RT_ERR_STATE when the last build ran untimed.
 * Copies min(capacity, size) bytes to dst and stores the buffer's full size in *bytes. */
rt_status rt_scene_debug_read(rt_scene *scene, const char *name, void *dst, size_t capacity, size_t *bytes);

/* Pipelined frames (RT_RENDER_NO_SYNC): wait for the last enqueued frame, return the device
 * counters accumulated since the last frame rendered without RT_RENDER_KEEP_COUNTERS (rays, pixels
 * and, with RT_RENDER_COUNT_WORK, the work counters) and the kernel duration of every frame
 * rendered since the previous collect (HIP events on the kernel's stream; up to 256 kept). */
rt_status rt_scene_collect(rt_scene *scene, rt_stats *accumulated, float *kernel_ms, uint32_t capacity,
                           uint32_t *count);

/* Replace triangles [first, first + count) of the scene's triangle array (deforming geometry,
 * e.g. the next frame of a VTK series, Renderer.cu:394-443).  RT_BUILD_LBVH scenes only: the
 * BLASes are rebuilt on the GPU by the next frame update, before that frame traces; until then a
 * trace that skips the update (RT_RENDER_SKIP_UPDATE, rt_trace_rays) returns RT_ERR_STATE, since it
 * would traverse the old trees while its hits read the new triangles.  Instances keep the local
 * bounds their description supplied (has_local_bounds), as the reference keeps the VTK reader's. */
rt_status rt_scene_update_triangles(rt_scene *scene, size_t first, size_t count, const rt_triangle *triangles);

/* Replace instance descriptions [first, first + count) — local bounds / centroid and the transform
 * used when no update callback is set (the next VTK frame's particles, VTKReader.cu:203-215).  The
 * primitives an instance refers to (type, index, count) may not change.  Takes effect with the next
 * TLAS build (rt_scene_update / rt_render); any build mode. */
rt_status rt_scene_update_instances(rt_scene *scene, size_t first, size_t count, const rt_instance_desc *instances);

/* Blocks until all work the scene enqueued has finished. */
rt_status rt_synchronize(rt_scene *scene);

/* Renderer::cleanup (src/Global/Renderer.cu:368-391). */
void rt_scene_destroy(rt_scene *scene);

/* --- interactive loop without a window -------------------------------------------
 * The reference's frame loop (src/Global/Renderer.cu:232-338) reads SDL key / mouse events, moves the
 * camera (SDL_OpenGLWindow::calculateNewPosition, src/Global/SDL_OpenGLWindow.cu:182-256), recomputes the
 * camera (RenderPin.cu:73-95), steps the move speed on the mouse wheel and caps the frame rate at 120 fps.
 * These calls restate that host logic on caller-supplied input, so a scripted or remote input stream drives
 * the same camera path; the window, the GL surface and SDL itself stay out (presentation).  Host-only. */

/* OperateArgs (include/Global/SDL_OpenGLWindow.cuh:34-45, filled by getOperateArgs :63-74) plus the loop's
 * relative-mouse-mode state (Renderer.cu:230, toggled by a click :239-241). */
typedef struct rt_camera_control {
    float mouse_sensitivity;       /* radians per mouse count */
    float pitch_limit;             /* as getOperateArgs stores it: PI / degreeToRadian(pitch_limit_degree) */
    float move_speed;              /* world units per frame; the wheel steps it */
    float move_speed_change_step;
    float fps_limit;               /* INFINITY: no cap */
    uint32_t restrict_frame_count; /* fps_limit != INFINITY */
    int64_t target_frame_us;       /* microseconds((int64)(1e6f / fps_limit)) */
    int64_t sleep_margin_us;       /* 2000 */
    uint32_t relative_mouse;       /* mouse motion counts only in relative mode (on at loop start) */
    uint32_t reserved;
} rt_camera_control;

/* KeyMouseInputArgs (include/Global/SDL_OpenGLWindow.cuh:47-60) for one frame: held keys, the mouse motion
 * and wheel accumulated since the previous frame (getKeyMouseInput resets them per frame,
 * SDL_OpenGLWindow.cu:135-141), a click, quit. */
typedef struct rt_input_state {
    uint32_t key_w, key_a, key_s, key_d, key_space, key_lshift;
    int32_t dx, dy;
    int32_t d_speed;
    uint32_t mouse_click;
    uint32_t key_quit;
} rt_input_state;

/* getOperateArgs(fpsLimit, mouseSensitivity, pitchLimitDegree, moveSpeedNTimesStep, moveSpeedChangeStep); the
 * reference's loop uses (120, 0.001, 80, 2, 0.05) (Renderer.cu:224-225). */
rt_status rt_camera_control_init(rt_camera_control *ctl, float fps_limit, float mouse_sensitivity,
                                 float pitch_limit_degree, uint32_t move_speed_n_steps, float move_speed_change_step);

/* The camera half of one loop iteration (Renderer.cu:236-262): mouse motion (counted in relative mode) turns
 * the view (yaw about V, then pitch about U, pitch clamp), held keys translate center and target in the
 * horizontal plane / along up; a click toggles relative mode; the wheel steps ctl->move_speed (after the
 * move, as the reference does).  `camera` is updated in place (center, target); *moved = 1 when the camera
 * moved, i.e. when the reference recomputes the camera (the caller then passes it to rt_camera_set with the
 * framebuffer size; the U / V / W the move used are those rt_camera_set derives from `camera`). */
rt_status rt_camera_move(rt_camera_input *camera, rt_camera_control *ctl, const rt_input_state *input,
                         uint32_t *moved);

/* Monotonic clock (steady_clock) in nanoseconds. */
int64_t rt_clock_ns(void);

/* The frame limiter (Renderer.cu:327-337): when less than ctl->target_frame_us has passed since
 * frame_start_ns, sleep until sleep_margin_us before the target, then spin until it.  Returns the
 * nanoseconds spent waiting (0 when the frame took longer). */
int64_t rt_frame_pace(const rt_camera_control *ctl, int64_t frame_start_ns);

/* Abort a stuck multi-GPU frame instead of blocking: with a timeout set, every wait the library does on a
 * frame that gathers over RCCL polls ncclCommGetAsyncError; on an asynchronous RCCL error or when the
 * frame has not completed after `timeout_ms`, the communicators are aborted (ncclCommAbort), the scene is
 * detached and the call returns RT_ERR_DEVICE.  0 (default) = wait without limit, polling only for
 * asynchronous errors. */
rt_status rt_comm_set_timeout(rt_scene *scene, uint32_t timeout_ms);

/* --- introspection (tests / tooling) -------------------------------------------- */

typedef struct rt_scene_info {
    uint64_t blas_count;
    uint64_t blas_node_pairs;      /* interior nodes over all BLAS (= node-pair records) */
    uint64_t blas_leaves;
    uint64_t tlas_node_pairs;
    uint64_t device_bytes;         /* HBM held by the scene */
    uint32_t width, height;
    uint32_t sqrt_sample_count;
    uint32_t ray_trace_depth;
    uint32_t tlas_height;          /* interior levels on the longest TLAS root-to-leaf path */
    uint32_t blas_height_max;      /* the same, deepest BLAS */
    uint32_t overlap_lanes;        /* lanes consecutive frames cycle through (option "overlap"; -1 = auto, resolved
                                    * by the last rt_render) */
    uint32_t stage_depth;          /* pinned staging buffers of the per-frame upload */
} rt_scene_info;

rt_status rt_scene_get_info(const rt_scene *scene, rt_scene_info *info);

/* Export a BLAS in the reference's node form (BLASNode array + BLASIndex array,
 * include/AS/BLAS.cuh:20-34) for tree-identity tests.  Pass NULL buffers to query sizes.
 * nodes: 8 floats per node {xmin,xmax,ymin,ymax,zmin,zmax, count, index} (count/index as
 * exact float-encoded integers < 2^24 are NOT assumed: use the uint32 arrays). */
rt_status rt_scene_export_blas(const rt_scene *scene, uint32_t blas_index,
                               float *node_boxes /* 6 per node */, uint32_t *node_count_index /* 2 per node */,
                               uint32_t *prim_refs /* primitive index per slot */,
                               uint32_t *n_nodes, uint32_t *n_prims);

/* Export the current TLAS (include/AS/TLAS.cuh:24-39) in the same form; prim_refs receive
 * instance indices (option "group": a ref >= instance_count is group ref - instance_count, standing for
 * its member instances in this frame). */
rt_status rt_scene_export_tlas(const rt_scene *scene,
                               float *node_boxes, uint32_t *node_count_index,
                               uint32_t *instance_refs, uint32_t *n_nodes, uint32_t *n_refs);

/* Built-in copy of the demo animation (src/Global/Main.cu:6-42 updateInstance) so that
 * benchmarks do not cross into Python per frame.  Matches rt_update_fn; `user` unused. */
void rt_demo_update(void *user, rt_xform *xforms, size_t instance_count, uint64_t frame);

/* --- scene ingestion: legacy VTK particle files ------------------------------
 * VTKReader::readVTKFile (src/Global/VTKReader.cu:16-164): DATASET POLYDATA, ASCII or BINARY,
 * POINTS + TRIANGLE_STRIPS (one strip = one particle; other cell types are rejected), cell arrays
 * "id" and "vel".  Vertex normals restate vtkPolyDataNormals (VTKReader.cu:60-70) from its
 * documented behaviour — parity unpinned at that third-party boundary.
 * Host-only: no GPU is needed. */
typedef struct rt_vtk_file rt_vtk_file;

typedef struct rt_vtk_info {
    uint64_t point_count;
    uint64_t particle_count;       /* strip cells */
    uint64_t strip_vertex_count;   /* sum of strip lengths (VTKParticle::vertices, concatenated) */
    uint64_t triangle_count;       /* sum of (strip length - 2) */
} rt_vtk_info;

/* VTKParticle (include/Global/VTKReader.cuh:12-30) without its vertex arrays. */
typedef struct rt_vtk_particle {
    uint64_t id;
    rt_vec3 velocity;
    float bounds[6];               /* [xmin,xmax,ymin,ymax,zmin,zmax] of the cell's points */
    rt_vec3 centroid;              /* mean of the cell's points (double sum, cast to float) */
    uint32_t first_vertex;         /* into the concatenated strip vertex stream */
    uint32_t vertex_count;
} rt_vtk_particle;

rt_status rt_vtk_read(const char *path, rt_vtk_file **out);
void rt_vtk_free(rt_vtk_file *file);
rt_status rt_vtk_get_info(const rt_vtk_file *file, rt_vtk_info *info);
/* particles[particle_count] */
rt_status rt_vtk_particles(const rt_vtk_file *file, rt_vtk_particle *particles);
/* strip vertex stream: positions / normals [strip_vertex_count] (either may be NULL) */
rt_status rt_vtk_vertices(const rt_vtk_file *file, rt_vec3 *positions, rt_vec3 *normals);
/* VTKReader::convertToRendererData (VTKReader.cu:166-220): triangles[triangle_count] (METAL 0,
 * odd strip triangles swap vertices 2/3), instances[particle_count] (local bounds / centroid of the
 * particle, transform shift (0,4,0) rotate (90,0,0) scale 3).  triangle_index_base = index of the
 * first particle triangle in the scene's triangle array (0 when prepended, Renderer.cu:13-18). */
rt_status rt_vtk_convert(const rt_vtk_file *file, uint32_t triangle_index_base, rt_triangle *triangles,
                         rt_instance_desc *instances);

/* Renderer::configureVTKFiles (src/Global/Renderer.cu:394-443): the .vtk.series JSON index;
 * entry paths are resolved against the series file's directory. */
typedef struct rt_vtk_series rt_vtk_series;
rt_status rt_vtk_series_read(const char *path, rt_vtk_series **out);
size_t rt_vtk_series_count(const rt_vtk_series *series);
rt_status rt_vtk_series_entry(const rt_vtk_series *series, size_t index, const char **path, float *time);
void rt_vtk_series_free(rt_vtk_series *series);

#ifdef __cplusplus
}
#endif

#endif /* RT_H */
