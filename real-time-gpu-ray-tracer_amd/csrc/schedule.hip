// schedule.hip — per-frame upload of the TLAS / instance block, by a kernel.
//
// The block (TLAS nodes, slots, instance records: ~35 KB for C2) is built on the host into pinned
// staging memory and read by this kernel over PCIe.  hipMemcpyAsync of the same bytes is handed to an
// SDMA engine and, between two traces on one stream, cost ~35 us of idle GPU per frame (rocprofv3 trace,
// round 1).  The kernel uses 8 VGPRs, so with overlapped lanes it fits beside a full persistent render
// grid (3 waves x 168 VGPRs per SIMD) instead of waiting for a drained workgroup slot.  It also clears
// the lane's work counters when the next launch starts a new counting epoch.
//
// (The claim-order schedule that used to run here is built by the render kernel's last workgroup:
// build_schedule in trace_kernel.hip.)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "layout.hpp"

namespace rtamd {

__global__ __launch_bounds__(256) void frame_copy_kernel(uint4 *__restrict__ dst, const uint4 *__restrict__ src, uint32_t n16,
                                                         unsigned long long *zero_counters) {
    if (zero_counters && blockIdx.x == 0 && threadIdx.x < CNT_NUM) zero_counters[threadIdx.x] = 0ull;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n16; i += gridDim.x * 256u) dst[i] = src[i];
}

hipError_t launch_frame_copy(void *dst, const void *src, size_t bytes, unsigned long long *zero_counters, hipStream_t stream) {
    if (bytes % 16) return hipErrorInvalidValue;
    const uint32_t n16 = (uint32_t)(bytes / 16);
    if (n16 == 0 && !zero_counters) return hipSuccess;
    const uint32_t blocks = n16 / 256u + 1u < 64u ? n16 / 256u + 1u : 64u;
    hipLaunchKernelGGL(frame_copy_kernel, dim3(blocks), dim3(256), 0, stream, static_cast<uint4 *>(dst),
                       static_cast<const uint4 *>(src), n16, zero_counters);
    return hipGetLastError();
}

// Zero n u32 with write-through (sc1) stores: the unit costs are only ever touched by memory-side atomics
// and write-through stores, so no XCD's L2 holds a copy the render kernel's last workgroup could read
// stale (build_schedule in trace_kernel.hip).
__global__ __launch_bounds__(256) void zero_agent_kernel(uint32_t *__restrict__ p, uint32_t n) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u)
        __hip_atomic_store(p + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
hipError_t launch_zero_agent(uint32_t *p, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (n > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const uint32_t blocks = (uint32_t)std::min<size_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(zero_agent_kernel, dim3(blocks), dim3(256), 0, stream, p, (uint32_t)n);
    return hipGetLastError();
}

}  // namespace rtamd
