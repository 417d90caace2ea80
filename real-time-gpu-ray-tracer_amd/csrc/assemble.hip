// assemble.hip — scatter gathered tile-compact RGBA8 slabs into a frame-layout framebuffer.
// This is the receive side of the multi-GPU screen-tile gather: rank r renders
// tiles t = r, r + N, r + 2N, ... (row-major tile order) into a compact slab; the slabs are
// gathered over RCCL and this kernel writes every in-frame pixel to its frame position.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.hpp"

namespace rtamd {

// One workgroup per gathered tile g (slab g / slab_tiles, its tile k = g % slab_tiles is frame tile
// t = rank + k * tile_count, tile_pixel's mapping): the tile's rows are copied 4 pixels (16 B) per
// thread, coalesced on both sides.  (A thread per pixel with 64-bit divisions per pixel took ~0.1 ms
// for a 1080p frame.)
__global__ __launch_bounds__(256) void assemble_kernel(const uint32_t *__restrict__ gathered, uint32_t slab_tiles,
                                                       uint32_t tile_w, uint32_t tile_h, uint32_t tile_count,
                                                       uint32_t width, uint32_t height, uint32_t *__restrict__ frame,
                                                       bool aligned16) {
    const uint32_t g = blockIdx.x;
    const uint32_t rank = g / slab_tiles, k = g - rank * slab_tiles;
    const uint32_t t = rank + k * tile_count;
    const uint32_t tiles_x = (width + tile_w - 1) / tile_w;
    if (t >= tiles_total(width, height, tile_w, tile_h)) return;            // padding of a short slab
    const uint32_t x0 = (t % tiles_x) * tile_w, y0 = (t / tiles_x) * tile_h;
    const uint32_t *src = gathered + (size_t)g * tile_w * tile_h;
    const uint32_t per = (tile_w & 3u) == 0 ? 4u : 1u;                    // pixels per thread step (a row piece)
    const bool vec = per == 4u && (width & 3u) == 0 && aligned16;   // 16 B loads / stores: both buffers 16 B-aligned
    for (uint32_t q = threadIdx.x; q < tile_w * tile_h / per; q += blockDim.x) {
        const uint32_t p = per * q, row = p / tile_w, col = p - row * tile_w;
        const uint32_t y = y0 + row, x = x0 + col;
        if (y >= height || x >= width) continue;
        uint32_t *dst = frame + (size_t)y * width + x;
        if (vec && x + 3u < width) {
            *reinterpret_cast<uint4 *>(dst) = *reinterpret_cast<const uint4 *>(src + p);
        } else {
            for (uint32_t j = 0; j < per && x + j < width; j++) dst[j] = src[p + j];
        }
    }
}

hipError_t launch_assemble(const void *gathered, uint32_t slab_tiles, uint32_t tile_w, uint32_t tile_h,
                           uint32_t tile_count, uint32_t width, uint32_t height, void *frame, hipStream_t stream) {
    const uint64_t blocks = (uint64_t)slab_tiles * tile_count;
    if (blocks == 0 || width == 0 || height == 0) return hipSuccess;
    if (tile_w == 0 || tile_h == 0 || blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    if (((reinterpret_cast<uintptr_t>(frame) | reinterpret_cast<uintptr_t>(gathered)) & 3u) != 0)
        return hipErrorInvalidValue;                                         // RGBA8 pixels are read as u32
    hipLaunchKernelGGL(assemble_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream,
                       static_cast<const uint32_t *>(gathered), slab_tiles, tile_w, tile_h, tile_count, width, height,
                       static_cast<uint32_t *>(frame),
                       ((reinterpret_cast<uintptr_t>(frame) | reinterpret_cast<uintptr_t>(gathered)) & 15u) == 0);
    return hipGetLastError();
}

}  // namespace rtamd
