// instances.hip — per-frame instance update on the GPU.
//
// The reference recomputes every instance's matrices on the host each frame: the update callback
// rewrites (shift, rotate, scale) and Instance::updateTransformArguments (src/AS/Instance.cu:4-17)
// builds M = Shift * (Rx * Ry * Rz) * Scale (src/Util/Matrix.cu:207-249), its Gauss-Jordan inverse
// (Matrix.cu:101-130), the inverse transpose and the 8-corner transformed AABB
// (src/AS/BoundingBox.cu:4-32) before the TLAS rebuild (Renderer.cu:269-276).  For GPU-built frames
// (RT_BUILD_LBVH) the host now uploads only the instances whose transform or local box changed — index,
// shift, the cosines and sines of the three angles (host libm, so both sides share one evaluation) and
// scale, plus the local box and centroid — and these kernels keep the per-instance parameters resident
// in HBM and compute every instance's records for the frame block: the inverse (InstHot), forward and
// inverse-transpose rows (InstCold), the transformed box and centroid the GPU TLAS builder reads.
// Compiled with -ffp-contract=off and the host's evaluation order (host_math.hpp, __host__ __device__):
// the records are bit-identical to the host path's and to the oracle's (tests/test_gpu_instances.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "host_math.hpp"
#include "layout.hpp"

namespace rtamd {
namespace {

__global__ __launch_bounds__(256) void instance_apply_kernel(const InstDelta *__restrict__ deltas, uint32_t count,
                                                             InstParams *__restrict__ params, uint32_t n) {
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j >= count) return;
    const InstDelta &d = deltas[j];
    if (d.index < n) params[d.index] = d.p;
}

__device__ __forceinline__ void rows(float *dst, const hm::Mat &m) {   // rows 1..3, cols 1..4
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) dst[4 * i + j] = m.d[i + 1][j + 1];
}

// roots (optional): each record's BLAS root {box, ref} copied into its hot record (the roots of GPU-built BLASes
// live only in HBM; wide_refs: the quad roots of host-built BLASes under a GPU TLAS, null for GPU-built ones).
// inf_inactive: an inactive record's box is all +inf (the multi-kernel TLAS builder sorts it into a subtree no ray
// enters); else its real box is kept and only the centroid's w marks it (the one-workgroup builder skips it)
struct RootPatch { const uint32_t *inst_blas; const TreeRoot *roots; const uint32_t *wide_refs; };
__global__ __launch_bounds__(256) void instance_update_kernel(const InstParams *__restrict__ params, uint32_t n,
                                                              InstHot *__restrict__ hot, InstCold *__restrict__ cold,
                                                              float *__restrict__ tbox, float4 *__restrict__ tcent,
                                                              RootPatch rp, bool inf_inactive) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    if (rp.inst_blas) {
        const uint32_t b = rp.inst_blas[i];
        const TreeRoot R = rp.roots[b];
#pragma unroll
        for (int k = 0; k < 6; k++) hot[i].root_box[k] = R.box[k];
        hot[i].root_ref = R.ref;
        hot[i].root_ref_wide = rp.wide_refs ? rp.wide_refs[b] : R.ref;
    }
    const InstParams &P = params[i];
    const hm::V3 sh{P.shift[0], P.shift[1], P.shift[2]}, c{P.cos[0], P.cos[1], P.cos[2]};
    const hm::V3 s{P.sin[0], P.sin[1], P.sin[2]}, sc{P.scale[0], P.scale[1], P.scale[2]};
    const hm::Mat fwd = hm::instance_matrix(sh, c, s, sc);
    const hm::Mat inv = hm::inverse(fwd);
    const hm::Mat nrm = hm::transpose(inv);
    rows(hot[i].inv, inv);
    rows(cold[i].fwd, fwd);
    rows(cold[i].nrm, nrm);
    // the local box exactly as the host holds it (already volume-expanded): from_points would not move it
    hm::Box lb;
    for (int a = 0; a < 3; a++) lb.r[a] = hm::Range{P.box[2 * a], P.box[2 * a + 1]};
    const hm::V3 tc = hm::apply_point(fwd, hm::V3{P.centroid[0], P.centroid[1], P.centroid[2]});
    if (P.pad[0] != 0.0f && inf_inactive) {   // inactive record (an intact group's member, a broken group)
        const float inf = __builtin_huge_valf();
#pragma unroll
        for (int k = 0; k < 6; k++) tbox[6 * (size_t)i + k] = inf;
        tcent[i] = make_float4(tc.x, tc.y, tc.z, 1.0f);
        return;
    }
    hm::transform_box(lb, fwd).store(tbox + 6 * (size_t)i);
    tcent[i] = make_float4(tc.x, tc.y, tc.z, P.pad[0] != 0.0f ? 1.0f : 0.0f);
}

// GPU-built TLAS: the instance records copied into TLAS leaf-slot order (record j = the instance in slot
// j), so entering a TLAS leaf reads its InstHot directly instead of through tlas_slots first
__global__ __launch_bounds__(256) void slot_order_kernel(const uint32_t *__restrict__ slots, const InstHot *__restrict__ hot,
                                                         const InstCold *__restrict__ cold, uint32_t n,
                                                         InstHot *__restrict__ hot_s, InstCold *__restrict__ cold_s) {
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j >= n) return;
    const uint32_t i = slots[j];
    if (i >= n) return;
    hot_s[j] = hot[i];
    cold_s[j] = cold[i];
}

}  // namespace

hipError_t launch_instance_slot_order(const uint32_t *slots, const InstHot *hot, const InstCold *cold, uint32_t n,
                                      InstHot *hot_s, InstCold *cold_s, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(slot_order_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, slots, hot, cold, n, hot_s, cold_s);
    return hipGetLastError();
}

// deltas: `count` changed instances (device memory: the uploaded part of the frame block)
hipError_t launch_instance_update(const InstDelta *deltas, uint32_t count, InstParams *params, uint32_t n, InstHot *hot,
                                  InstCold *cold, float *tbox, float4 *tcent, const uint32_t *inst_blas,
                                  const TreeRoot *roots, const uint32_t *wide_refs, bool inf_inactive, hipStream_t stream) {
    if (count) {
        hipLaunchKernelGGL(instance_apply_kernel, dim3((count + 255) / 256), dim3(256), 0, stream, deltas, count, params, n);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(instance_update_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, params, n, hot, cold, tbox, tcent,
                       RootPatch{inst_blas, roots, wide_refs}, inf_inactive);
    return hipGetLastError();
}

}  // namespace rtamd
