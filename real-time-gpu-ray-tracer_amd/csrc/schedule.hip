// schedule.hip — claim order of the persistent render kernel's work queue (option "reorder"), and the
// per-frame upload of the TLAS / instance block.
//
// The persistent launch (trace_kernel.hip) ends when its last wave does.  A wave claims one 8x8 unit at
// a time and its lanes refill from that unit, so a unit holds a wave for as long as its 64 paths take,
// and that is very uneven: a sky unit averages ~5 traversal steps per pixel, a unit over the particle
// cluster ~100.  Claimed in screen order, the heavy units that sit late in a band start late and the GPU
// waits for them (C2: the queue ran dry at ~270 us, the last wave ended at ~520 us).  Animated frames
// change little from one frame to the next, so each launch records the traversal work of every unit
// (unit_cost, one atomicAdd per unit and shade step) and this kernel orders the lane's next launch's
// claims heaviest-first (longest-processing-time-first list scheduling).  The image does not depend on
// the order: every pixel's RNG stream is keyed by its global pixel index.
//
// One 256-thread workgroup per band: the band's costs are read coalesced (8 B per lane, several loads in
// flight) into 4-bit class codes in LDS and cleared for the next launch, then a stable counting sort over
// 16 cost classes (class order = heaviest first; equal classes keep screen order, so neighbouring units
// of one class are still claimed together).  A heavy unit becomes 2 or 4 claim items (32 / 16 pixels) so
// that its paths spread over several waves.  The band's items go to order[4 b0 ...) as
// (unit << 4 | piece << 2 | log2 pieces), the item count to the band's count word (a line of its own,
// away from the atomically updated head), and the queue heads are reset.  The kernel also uploads the
// frame's TLAS / instance block from pinned staging and clears the lane's work counters.
//
// Footprint (measured, profiles/r02_*): with overlapped lanes this kernel runs while the other lane's
// persistent grid holds the GPU, in the workgroup slots the grid leaves free (setting "reserve": one per
// XCD).  Round 1's version (one 1024-thread workgroup, 64 KB of LDS per band) could only start once the
// other launch drained and averaged 172 us per frame; a 256-thread version with 49 KB of LDS still
// waited (84 us: a drained render workgroup leaves 32 KB holes of LDS); building the order in the render
// launch's last workgroup instead added ~90 us to every launch (one CU doing the whole frame's sort).
// So: 4 waves and <= 16.2 KB of LDS — half the LDS footprint of one render workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.hpp"

namespace rtamd {
namespace {

constexpr uint32_t SCHED_THREADS = 256;
constexpr uint32_t SCHED_NIB_UNITS = 16384;    // band units whose class nibbles fit in 8 KB of LDS
constexpr uint32_t SCHED_LOADS = 4;            // 8-byte cost loads in flight per thread
constexpr uint32_t COPY_AHEAD = 2;             // 16-byte frame-block pieces loaded before the cost loads

__global__ __launch_bounds__(SCHED_THREADS) void schedule_kernel(uint32_t *__restrict__ cost, uint32_t *__restrict__ cost_prev,
                                                                 uint32_t *__restrict__ order, uint32_t *__restrict__ queue,
                                                                 uint32_t rows, uint32_t upr, uint32_t parts, uint32_t do_order,
                                                                 uint32_t kh, uint32_t kq, uint32_t km, uint4 *copy_dst,
                                                                 const uint4 *copy_src, uint32_t copy_n16,
                                                                 unsigned long long *zero_counters) {
    __shared__ uint16_t cnt[SCHED_CLASSES * SCHED_THREADS];   // per-thread class item counts -> offsets (8 KB)
    __shared__ uint8_t nib[SCHED_NIB_UNITS / 2];               // class codes, 2 per byte (8 KB)
    __shared__ uint32_t total[SCHED_CLASSES], base[SCHED_CLASSES];
    const uint32_t part = blockIdx.x, t = threadIdx.x;
    if (part == 0 && t < 2 * QUEUE_MAX_PARTS) queue[(t >> 1) * QUEUE_STRIDE + (t & 1u)] = 0u;   // every head (front,
                                                                                               // back): `parts` may change
    if (part == 0 && zero_counters && t < CNT_NUM) zero_counters[t] = 0ull;  // the lane's work counters
    // the frame's TLAS / instance block, read from pinned host staging (see launch_frame_copy): the first
    // COPY_AHEAD pieces per thread are loaded now and stored after the first cost loads have been issued,
    // so the PCIe read and the cost reads overlap (vector loads return in order: one wait covers both)
    const uint32_t cstride = parts * SCHED_THREADS;
    uint4 ahead[COPY_AHEAD];
#pragma unroll
    for (uint32_t k = 0; k < COPY_AHEAD; k++) {
        const uint32_t i = part * SCHED_THREADS + t + k * cstride;
        ahead[k] = i < copy_n16 ? copy_src[i] : make_uint4(0u, 0u, 0u, 0u);
    }
    const auto finish_copy = [&]() {
#pragma unroll
        for (uint32_t k = 0; k < COPY_AHEAD; k++) {
            const uint32_t i = part * SCHED_THREADS + t + k * cstride;
            if (i < copy_n16) copy_dst[i] = ahead[k];
        }
        for (uint32_t i = part * SCHED_THREADS + t + COPY_AHEAD * cstride; i < copy_n16; i += cstride) copy_dst[i] = copy_src[i];
    };
    // the band's unit range, computed exactly as the render kernel's refill computes it
    const uint32_t b0 = rows * part / parts * upr, b1 = rows * (part + 1) / parts * upr;
    const uint32_t n = b1 - b0;
    if (!do_order) {
        finish_copy();
        for (uint32_t u = b0 + t; u < b1; u += SCHED_THREADS) { cost_prev[u] = cost[u]; cost[u] = 0u; }
        return;
    }
    // bands of < 16384 units (any frame up to 4K with 8 bands) sort from LDS class codes with 16-bit
    // offsets
    const uint32_t gbase = b0 & ~1u;
    const bool in_lds = b1 - gbase <= SCHED_NIB_UNITS && 4u * n < 65536u;
    bool copied = false;
    if (in_lds) {
        // pass A: pairs of costs, coalesced 8-byte loads -> class codes; costs kept (debug) and cleared
        const uint32_t npair = (b1 - gbase + 1) / 2;
        for (uint32_t i0 = t; i0 < npair; i0 += SCHED_THREADS * SCHED_LOADS) {
            uint2 v[SCHED_LOADS];
#pragma unroll
            for (uint32_t k = 0; k < SCHED_LOADS; k++) {
                const uint32_t i = i0 + k * SCHED_THREADS;
                v[k] = i < npair ? reinterpret_cast<const uint2 *>(cost + gbase)[i] : make_uint2(0u, 0u);
            }
            if (!copied) { finish_copy(); copied = true; }
#pragma unroll
            for (uint32_t k = 0; k < SCHED_LOADS; k++) {
                const uint32_t i = i0 + k * SCHED_THREADS;
                if (i >= npair) break;
                uint32_t code = 0;
#pragma unroll
                for (uint32_t h = 0; h < 2; h++) {
                    const uint32_t u = gbase + 2 * i + h;
                    if (u < b0 || u >= b1) continue;       // the neighbour band's unit: not ours to clear
                    const uint32_t c = h ? v[k].y : v[k].x;
                    code |= cost_class(c) << (4 * h);
                    cost_prev[u] = c;
                    cost[u] = 0u;
                }
                nib[i] = (uint8_t)code;
            }
        }
    }
    if (!copied) finish_copy();
    __syncthreads();
    if (!in_lds) {
        // a band of >= 16384 units (beyond 4K with 8 bands): screen order, one item per unit
        for (uint32_t u = b0 + t; u < b1; u += SCHED_THREADS) {
            cost_prev[u] = cost[u];
            cost[u] = 0u;
            order[4u * b0 + (u - b0)] = u << 4;
        }
        if (t == 0) queue[(QUEUE_MAX_PARTS + part) * QUEUE_STRIDE] = n;
        return;
    }
    // even per-thread ranges: a merged pair of light units (setting "merge") never spans two threads
    const uint32_t per = ((n + SCHED_THREADS - 1) / SCHED_THREADS + 1) & ~1u;
    const uint32_t lo = b0 + min(n, t * per), hi = b0 + min(n, (t + 1) * per);
    const auto cls = [&](uint32_t u) { return (uint32_t)(nib[(u - gbase) >> 1] >> (4 * ((u - gbase) & 1u))) & 15u; };
    for (uint32_t c = 0; c < SCHED_CLASSES; c++) cnt[c * SCHED_THREADS + t] = 0;
    // setting "merge": two adjacent light units (levels below km, pair offset even) become one 128-pixel item
    // in the pair's heavier class, so a claim over the sky / ground serves twice the pixels
    const auto light = [&](uint32_t c) { return (SCHED_CLASSES - 1u) - c < km; };
    for (uint32_t u = lo; u < hi; u++) {
        const uint32_t c = cls(u);
        if (km && u + 1 < hi && light(c) && light(cls(u + 1))) {
            cnt[min(c, cls(u + 1)) * SCHED_THREADS + t] += 1;
            u++;
            continue;
        }
        cnt[c * SCHED_THREADS + t] += (uint16_t)(1u << split_log2(c, kh, kq));
    }
    __syncthreads();
    // exclusive scan of each class's item counts over the threads (thread order = screen order):
    // wave w scans classes [4w, 4w + 4), each lane 4 consecutive threads' counts (< 65536 items per band)
    const uint32_t w = t >> 6, lane = t & 63u;
    for (uint32_t cc = 0; cc < SCHED_CLASSES / 4; cc++) {
        const uint32_t c = w * (SCHED_CLASSES / 4) + cc;
        uint32_t local[4], run = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) { local[k] = run; run += cnt[c * SCHED_THREADS + lane * 4 + k]; }
        uint32_t incl = run;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off, 64);
            if (lane >= (uint32_t)off) incl += y;
        }
        const uint32_t excl = incl - run;
        if (lane == 63u) total[c] = incl;
#pragma unroll
        for (int k = 0; k < 4; k++) cnt[c * SCHED_THREADS + lane * 4 + k] = (uint16_t)(excl + local[k]);
    }
    __syncthreads();
    if (t == 0) {
        uint32_t acc = 0;
        for (uint32_t c = 0; c < SCHED_CLASSES; c++) { base[c] = acc; acc += total[c]; }
        queue[(QUEUE_MAX_PARTS + part) * QUEUE_STRIDE] = acc;   // items in the band (own line)
    }
    __syncthreads();
    // pass 2: the band's items [4 b0, 4 b0 + items) — at most 4 per unit
    uint32_t *items = order + 4u * b0;
    for (uint32_t u = lo; u < hi; u++) {
        if (km && u + 1 < hi && light(cls(u)) && light(cls(u + 1))) {        // merged pair: log2 pieces field 3
            const uint32_t c = min(cls(u), cls(u + 1));
            const uint32_t at = base[c] + cnt[c * SCHED_THREADS + t];
            cnt[c * SCHED_THREADS + t] = (uint16_t)(at - base[c] + 1u);
            items[at] = (u << 4) | 3u;
            u++;
            continue;
        }
        const uint32_t c = cls(u), ls = split_log2(c, kh, kq);
        const uint32_t at = base[c] + cnt[c * SCHED_THREADS + t];
        cnt[c * SCHED_THREADS + t] = (uint16_t)(at - base[c] + (1u << ls));
        for (uint32_t k = 0; k < (1u << ls); k++) items[at + k] = (u << 4) | (k << 2) | ls;
    }
}

}  // namespace

// rows x upr units per frame split into `parts` bands as in render_persistent_body; do_order = 0 only
// clears the costs and the queue heads (first launch of a layout: no costs recorded yet).
// zero_counters (optional): CNT_NUM device counters cleared before the launch that follows.
hipError_t launch_schedule(uint32_t *cost, uint32_t *cost_prev, uint32_t *order, uint32_t *queue, uint32_t rows, uint32_t upr,
                           uint32_t parts, bool do_order, uint32_t k_half, uint32_t k_quarter, uint32_t k_merge, void *copy_dst,
                           const void *copy_src, size_t copy_bytes, unsigned long long *zero_counters, hipStream_t stream) {
    if (parts == 0 || parts > QUEUE_MAX_PARTS || copy_bytes % 16) return hipErrorInvalidValue;
    hipLaunchKernelGGL(schedule_kernel, dim3(parts), dim3(SCHED_THREADS), 0, stream, cost, cost_prev, order, queue, rows, upr,
                       parts, do_order ? 1u : 0u, k_half, k_quarter, k_merge, static_cast<uint4 *>(copy_dst),
                       static_cast<const uint4 *>(copy_src), (uint32_t)(copy_bytes / 16), zero_counters);
    return hipGetLastError();
}

// Per-frame upload of the TLAS / instance block by a kernel reading the pinned staging buffer over PCIe,
// when no schedule kernel carries it.  hipMemcpyAsync of the same ~35 KB is handed to an SDMA engine and,
// between two traces on one stream, cost ~35 us of idle GPU per frame (rocprofv3 trace, round 1).  8 VGPRs:
// it fits beside a full persistent grid.
__global__ __launch_bounds__(256) void frame_copy_kernel(uint4 *__restrict__ dst, const uint4 *__restrict__ src, uint32_t n16,
                                                         unsigned long long *zero_counters, uint32_t *zero_queue) {
    if (zero_counters && blockIdx.x == 0 && threadIdx.x < CNT_NUM) zero_counters[threadIdx.x] = 0ull;
    if (zero_queue && blockIdx.x == 0 && threadIdx.x < 2 * QUEUE_MAX_PARTS)
        zero_queue[(threadIdx.x >> 1) * QUEUE_STRIDE + (threadIdx.x & 1u)] = 0u;     // head words: front, back
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n16; i += gridDim.x * 256u) dst[i] = src[i];
}

// zero_queue (optional): the persistent launch's queue heads, reset here instead of by a fill kernel
hipError_t launch_frame_copy(void *dst, const void *src, size_t bytes, unsigned long long *zero_counters, uint32_t *zero_queue,
                             hipStream_t stream) {
    if (bytes % 16) return hipErrorInvalidValue;
    const uint32_t n16 = (uint32_t)(bytes / 16);
    if (n16 == 0 && !zero_counters && !zero_queue) return hipSuccess;
    const uint32_t blocks = n16 / 256u + 1u < 64u ? n16 / 256u + 1u : 64u;
    hipLaunchKernelGGL(frame_copy_kernel, dim3(blocks), dim3(256), 0, stream, static_cast<uint4 *>(dst),
                       static_cast<const uint4 *>(src), n16, zero_counters, zero_queue);
    return hipGetLastError();
}

}  // namespace rtamd
