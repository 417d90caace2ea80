// assemble.hip — scatter gathered tile-compact RGBA8 slabs into a frame-layout framebuffer.
// This is the receive side of the multi-GPU screen-tile gather: rank r renders
// tiles t = r, r + N, r + 2N, ... (row-major tile order) into a compact slab; the slabs are
// gathered over RCCL and this kernel writes every in-frame pixel to its frame position.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.hpp"

namespace rtamd {

__global__ __launch_bounds__(256) void assemble_kernel(const uint32_t *__restrict__ gathered, uint64_t slab_px,
                                                       uint32_t tile_w, uint32_t tile_h, uint32_t tile_count,
                                                       uint32_t width, uint32_t height, uint32_t *__restrict__ frame) {
    const uint64_t total = (uint64_t)tile_count * slab_px;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x, y;
        if (tile_pixel(width, height, tile_w, tile_h, (uint32_t)(i / slab_px), tile_count, i % slab_px, x, y))
            frame[(size_t)y * width + x] = gathered[i];
    }
}

hipError_t launch_assemble(const void *gathered, uint32_t slab_tiles, uint32_t tile_w, uint32_t tile_h,
                           uint32_t tile_count, uint32_t width, uint32_t height, void *frame, hipStream_t stream) {
    const uint64_t slab_px = (uint64_t)slab_tiles * tile_w * tile_h;
    const uint64_t total = (uint64_t)tile_count * slab_px;
    if (total == 0) return hipSuccess;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(assemble_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream,
                       static_cast<const uint32_t *>(gathered), slab_px, tile_w, tile_h, tile_count, width, height,
                       static_cast<uint32_t *>(frame));
    return hipGetLastError();
}

}  // namespace rtamd
