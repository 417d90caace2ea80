/*
 * rt_oracle.h — CPU restatement of the reference trace path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product (librtamd.so) never links or calls it.
 *
 * PARITY UNPINNED: the reference (3169651074/real-time-gpu-ray-tracer) is CUDA C++ that
 * needs the CUDA toolkit headers (cuda_runtime.h, curand_kernel.h) and nvcc, none of which
 * exist in this image, and it ships no tests, golden images or fixtures.  This oracle is
 * therefore a line-by-line restatement of the reference's algorithm (each function cites
 * the reference file:line it follows), pinned only by analytic known-answer tests
 * (tests/test_oracle_kat.py) — not by outputs of the reference itself.  See DESIGN.md §3.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "../include/rt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_scene oracle_scene;

typedef struct oracle_counters {
    uint64_t rays;              /* TLAS::hit calls                */
    uint64_t aabb_tests;        /* BoundingBox::hit calls         */
    uint64_t triangle_tests;
    uint64_t sphere_quad_tests;
    uint64_t instance_visits;   /* Instance::hit calls            */
    uint64_t node_pops;         /* stack pops (TLAS + BLAS)       */
} oracle_counters;

/* Renderer::commitGeometryData .. buildAccelerationStructure (BLAS part). */
oracle_scene *oracle_scene_create(const rt_scene_desc *desc, uint64_t build_seed);
void oracle_scene_destroy(oracle_scene *s);
/* updateInstances(frame) + TLAS rebuild (Renderer.cu:269-276). */
int oracle_scene_update(oracle_scene *s, uint64_t frame);
/* calculateCameraProperties (RenderPin.cu:73-95). */
int oracle_camera_set(oracle_scene *s, const rt_camera_input *cam, uint32_t w, uint32_t h);

/* render kernel (Kernel.cu:105-147) over the pixel rectangle [x0,x0+w) x [y0,y0+h) of the
 * frame; outputs are w*h row-major (row 0 = frame row y0).  rgb may be NULL, rgba may be
 * NULL.  brute_force = 1 replaces TLAS/BLAS traversal by loops over all instances and
 * primitives (intent of the dead NO_AS path, Kernel.cu:10-62).  threads <= 0 -> 1. */
int oracle_render(const oracle_scene *s, uint64_t frame_seed,
                  uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                  float *rgb, uint8_t *rgba, int threads, int brute_force,
                  oracle_counters *counters);

/* Closest hit of world rays (ox,oy,oz,dx,dy,dz per ray) over [0.001, inf). */
int oracle_trace(const oracle_scene *s, const float *rays, size_t n, rt_hit *hits,
                 int brute_force, oracle_counters *counters);

/* Tree export in the reference node form (for tree-identity tests). */
int oracle_export_blas(const oracle_scene *s, uint32_t blas_index, float *node_boxes,
                       uint32_t *node_count_index, uint32_t *prim_refs,
                       uint32_t *n_nodes, uint32_t *n_prims);
int oracle_export_tlas(const oracle_scene *s, float *node_boxes, uint32_t *node_count_index,
                       uint32_t *instance_refs, uint32_t *n_nodes, uint32_t *n_refs);
uint32_t oracle_blas_count(const oracle_scene *s);

/* --- single-primitive known-answer entry points ----------------------------------
 * ray = {ox,oy,oz,dx,dy,dz}; range = {min,max}; out = {t, px,py,pz, nx,ny,nz, u, v}.
 * Return 1 on hit.  These run the same code the traversal runs. */
int oracle_hit_sphere(const rt_sphere *sp, const float *ray, const float *range, float *out);
int oracle_hit_parallelogram(const rt_parallelogram *pg, const float *ray, const float *range, float *out);
int oracle_hit_triangle(const rt_triangle *tr, const float *ray, const float *range, float *out);
/* box = {xmin,xmax,ymin,ymax,zmin,zmax} (used as stored, no ensureVolume). */
int oracle_hit_aabb(const float *box, const float *ray, const float *range, float *t_entry);
/* Primitive AABB after BoundingBox construction rules (ensureVolume). */
void oracle_prim_bounds(uint32_t type, const void *prim, float *box6);

/* Pinned RNG contract: curand_init / curand_uniform replacement. */
uint64_t oracle_rng_init(uint64_t seed, uint64_t subsequence, uint64_t offset);
float oracle_rng_uniform(uint64_t *state);

/* Instance matrices after Instance::updateTransformArguments (Instance.cu:4-17):
 * out = 16 floats forward (row-major 4x4) + 16 inverse + 16 normal (inverse^T). */
void oracle_instance_matrices(const rt_xform *x, float *out48);
int oracle_instance_state(const oracle_scene *s, uint32_t i, float *out45);

/* Camera after calculateCameraProperties: pixelOrigin, dx, dy, center, U, V (18 floats),
 * then recip_sqrt, sqrt_sample_count. */
int oracle_camera_export(const oracle_scene *s, float *out20);

/* Oracle's own copy of the demo animation (src/Global/Main.cu:6-42). */
void oracle_demo_update(void *user, rt_xform *x, size_t n, uint64_t frame);

#ifdef __cplusplus
}
#endif

#endif
