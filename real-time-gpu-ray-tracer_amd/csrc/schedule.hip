// schedule.hip — claim order of the persistent render kernel's work queue (option "reorder").
//
// The persistent kernel (trace_kernel.hip) ends when its last wave does.  A wave claims one 8x8 unit
// at a time and its lanes refill from that unit, so a unit holds a wave for as long as its 64 paths
// take, and that is very uneven: a sky unit averages ~5 traversal steps per pixel, a unit over the
// particle cluster ~100.  Claimed in screen order, the heavy units that sit late in a band start late
// and the GPU waits for them: measured on C2, the queue ran dry at ~270 us and the last wave ended
// at ~520 us.  Animated frames change little from one frame to the next, so each launch records the
// traversal work of every unit (unit_cost, one atomicAdd per unit and shade step) and this kernel
// orders the next launch's claims heaviest-first (longest-processing-time-first list scheduling).
// The image does not depend on the order: every pixel's RNG stream is keyed by its global pixel
// index.
//
// One 256-thread workgroup per band: a stable counting sort of the band's units over 16 cost classes
// (class order = heaviest first; equal classes keep screen order, so neighbouring units of one class are
// still claimed together).  A heavy unit becomes 2 or 4 claim items (32 / 16 pixels) so that its paths
// spread over several waves instead of holding one wave for the critical path.  The band's items go to
// order[4 b0 ...) as (unit << 4 | piece << 2 | log2 pieces), the item count to the band's count word (a
// line of its own, away from the atomically updated head); then the costs are cleared for the next launch
// and the queue heads are reset (this replaces the per-frame hipMemsetAsync of the heads).
//
// Footprint: a workgroup is sized like one workgroup of the persistent render kernel (4 waves, 16 KB of
// LDS), so with overlapped frames it runs in the workgroup slots the render grid leaves free (option
// "reserve", rt_api.cpp) while the other lane's launch holds the rest of the GPU.  The first version used
// one 1024-thread workgroup with 64 KB of LDS per band: it could only start once the other lane's
// launch began to drain, and averaged 172 us per frame instead of 10 us (profiles/r01_kernel_stats_final.csv).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.hpp"

namespace rtamd {
namespace {

constexpr int SCHED_THREADS = 256;      // 4 waves: the footprint of one render workgroup
constexpr int SCHED_CLASSES = 16;
constexpr int SCHED_WAVES = SCHED_THREADS / 64;
constexpr int SCAN_PER_LANE = SCHED_THREADS / 64;                    // threads' counts summed per lane in the scan

// class 0 = heaviest: half-octaves of the unit's mean traversal steps per pixel, floor(2 log2(c/64 + 1))
// (a sky unit averages ~5 steps per pixel, a unit over the particle cluster ~100; classes saturate at ~180)
// in integers: 2 log2(x/64) = log2(x^2) - 12 with x = c + 64
__device__ __forceinline__ uint32_t cost_class(uint32_t c) {
    const uint64_t x = (uint64_t)c + 64u;
    const int k = (63 - __builtin_clzll(x * x)) - 12;
    return (uint32_t)(SCHED_CLASSES - 1) - (uint32_t)min(max(k, 0), SCHED_CLASSES - 1);
}

// heavy units may be claimed in pieces so that several waves share them: 1/4 of a unit (16 pixels)
// from class level k_quarter up, 1/2 from k_half up (levels k = 15 - class; > 15 = never)
__device__ __forceinline__ uint32_t split_log2(uint32_t cls, uint32_t k_half, uint32_t k_quarter) {
    const uint32_t k = (uint32_t)(SCHED_CLASSES - 1) - cls;
    return k >= k_quarter ? 2u : (k >= k_half ? 1u : 0u);
}

constexpr uint32_t SCHED_LDS_UNITS = 32768;  // units per band whose cost classes are kept in LDS (1 B each)
constexpr uint32_t SCHED_LOAD_BATCH = 8;          // cost loads issued back to back per thread

__global__ __launch_bounds__(SCHED_THREADS) void schedule_kernel(uint32_t *__restrict__ cost, uint32_t *__restrict__ order,
                                                                 uint32_t *__restrict__ queue, uint32_t rows,
                                                                 uint32_t upr, uint32_t parts, uint32_t do_order,
                                                                 uint32_t k_half, uint32_t k_quarter, uint4 *copy_dst,
                                                                 const uint4 *copy_src, uint32_t copy_n16,
                                                                 unsigned long long *zero_counters) {
    __shared__ uint32_t cnt[SCHED_CLASSES][SCHED_THREADS];   // per-thread class counts -> exclusive offsets
    __shared__ uint8_t cls_of[SCHED_LDS_UNITS];              // class of each unit of the band (pass 1 -> pass 2)
    __shared__ uint32_t total[SCHED_CLASSES];
    __shared__ uint32_t base[SCHED_CLASSES];
    const uint32_t part = blockIdx.x, t = threadIdx.x;
    if (part == 0 && t < QUEUE_MAX_PARTS) queue[t * QUEUE_STRIDE] = 0u;      // every head: `parts` may change
    if (part == 0 && zero_counters && t < CNT_NUM) zero_counters[t] = 0ull;  // the lane's work counters
    // the frame's TLAS / instance block, read from pinned host staging (see launch_frame_copy)
    for (uint32_t i = part * SCHED_THREADS + t; i < copy_n16; i += parts * SCHED_THREADS) copy_dst[i] = copy_src[i];
    // the band's unit range, computed exactly as the render kernel computes it
    const uint32_t b0 = rows * part / parts * upr, b1 = rows * (part + 1) / parts * upr;
    const uint32_t n = b1 - b0, per = (n + SCHED_THREADS - 1) / SCHED_THREADS;
    const uint32_t lo = b0 + min(n, t * per), hi = b0 + min(n, (t + 1) * per);
    if (!do_order) {
        for (uint32_t u = lo; u < hi; u++) cost[u] = 0u;
        return;
    }
    const bool lds_cls = n <= SCHED_LDS_UNITS;
    for (int c = 0; c < SCHED_CLASSES; c++) cnt[c][t] = 0u;
    // pass 1: classes and per-thread item counts; the costs are read in batches of independent loads
    // (this kernel runs beside another lane's launch: each dependent round trip is ~1-2 us there) and
    // cleared for the next launch
    for (uint32_t u0 = lo; u0 < hi; u0 += SCHED_LOAD_BATCH) {
        uint32_t cv[SCHED_LOAD_BATCH];
#pragma unroll
        for (uint32_t k = 0; k < SCHED_LOAD_BATCH; k++) cv[k] = u0 + k < hi ? cost[u0 + k] : 0u;
#pragma unroll
        for (uint32_t k = 0; k < SCHED_LOAD_BATCH; k++) {
            if (u0 + k >= hi) break;
            const uint32_t c = cost_class(cv[k]);
            if (lds_cls) cls_of[u0 + k - b0] = (uint8_t)c;
            cnt[c][t] += 1u << split_log2(c, k_half, k_quarter);
            if (lds_cls) cost[u0 + k] = 0u;
        }
    }
    __syncthreads();
    // exclusive scan of each class's item counts over the threads (thread order = screen order):
    // wave w scans classes [4w, 4w + 4), each lane SCAN_PER_LANE consecutive threads' counts
    const uint32_t w = t >> 6, lane = t & 63u;
    for (int cc = 0; cc < SCHED_CLASSES / SCHED_WAVES; cc++) {
        const uint32_t c = w * (SCHED_CLASSES / SCHED_WAVES) + cc;
        uint32_t local[SCAN_PER_LANE], run = 0;
#pragma unroll
        for (int k = 0; k < SCAN_PER_LANE; k++) { local[k] = run; run += cnt[c][lane * SCAN_PER_LANE + k]; }
        uint32_t incl = run;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off, 64);
            if (lane >= (uint32_t)off) incl += y;
        }
        const uint32_t excl = incl - run;
#pragma unroll
        for (int k = 0; k < SCAN_PER_LANE; k++) cnt[c][lane * SCAN_PER_LANE + k] = excl + local[k];
        if (lane == 63u) total[c] = incl;
    }
    __syncthreads();
    if (t == 0) {
        uint32_t acc = 0;
        for (int c = 0; c < SCHED_CLASSES; c++) { base[c] = acc; acc += total[c]; }
        queue[(QUEUE_MAX_PARTS + part) * QUEUE_STRIDE] = acc;   // items in the band (own line)
    }
    __syncthreads();
    // pass 2: items of the band: [4 b0, 4 b0 + items) — at most 4 per unit
    uint32_t *items = order + 4u * b0;
    for (uint32_t u = lo; u < hi; u++) {
        const uint32_t c = lds_cls ? (uint32_t)cls_of[u - b0] : cost_class(cost[u]), ls = split_log2(c, k_half, k_quarter);
        const uint32_t at = base[c] + cnt[c][t];
        for (uint32_t k = 0; k < (1u << ls); k++) items[at + k] = (u << 4) | (k << 2) | ls;
        cnt[c][t] = at - base[c] + (1u << ls);
    }
    if (!lds_cls)
        for (uint32_t u = lo; u < hi; u++) cost[u] = 0u;
}

}  // namespace

// rows x upr units per frame split into `parts` bands as in render_persistent_body; do_order = 0 only
// clears the costs and the queue heads (first launch of a layout: no costs recorded yet).
// zero_counters (optional): CNT_NUM device counters cleared before the launch that follows.
hipError_t launch_schedule(uint32_t *cost, uint32_t *order, uint32_t *queue, uint32_t rows, uint32_t upr,
                           uint32_t parts, bool do_order, uint32_t k_half, uint32_t k_quarter, void *copy_dst,
                           const void *copy_src, size_t copy_bytes, unsigned long long *zero_counters, hipStream_t stream) {
    if (parts == 0 || parts > QUEUE_MAX_PARTS || copy_bytes % 16) return hipErrorInvalidValue;
    hipLaunchKernelGGL(schedule_kernel, dim3(parts), dim3(SCHED_THREADS), 0, stream, cost, order, queue, rows, upr, parts,
                       do_order ? 1u : 0u, k_half, k_quarter, static_cast<uint4 *>(copy_dst),
                       static_cast<const uint4 *>(copy_src), (uint32_t)(copy_bytes / 16), zero_counters);
    return hipGetLastError();
}

// Per-frame upload of the TLAS / instance block by a kernel reading the pinned staging buffer over
// PCIe.  hipMemcpyAsync of the same ~35 KB is handed to an SDMA engine and, between two traces on
// one stream, cost ~35 us of idle GPU per frame (rocprofv3 trace); the schedule kernel does this copy
// itself when option "reorder" is on.
__global__ __launch_bounds__(256) void frame_copy_kernel(uint4 *__restrict__ dst, const uint4 *__restrict__ src, uint32_t n16) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n16; i += gridDim.x * 256u) dst[i] = src[i];
}
hipError_t launch_frame_copy(void *dst, const void *src, size_t bytes, hipStream_t stream) {
    if (bytes % 16) return hipErrorInvalidValue;
    const uint32_t n16 = (uint32_t)(bytes / 16);
    if (n16 == 0) return hipSuccess;
    const uint32_t blocks = n16 / 256u + 1u < 64u ? n16 / 256u + 1u : 64u;
    hipLaunchKernelGGL(frame_copy_kernel, dim3(blocks), dim3(256), 0, stream, static_cast<uint4 *>(dst),
                       static_cast<const uint4 *>(src), n16);
    return hipGetLastError();
}

}  // namespace rtamd
