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

}  // namespace rtamd
