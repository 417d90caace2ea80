// assemble.hip — scatter gathered tile-compact RGBA8 slabs into a frame-layout framebuffer.
// This is the receive side of the multi-GPU screen-tile gather: rank r renders
// tiles t = r, r + N, r + 2N, ... (row-major tile order) into a compact slab; the slabs are
// gathered over RCCL and this kernel writes every in-frame pixel to its frame position.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtamd {

__global__ __launch_bounds__(256) void assemble_kernel(const uint32_t *__restrict__ gathered, uint32_t slab_tiles,
                                                       uint32_t tile_w, uint32_t tile_h, uint32_t tile_count,
                                                       uint32_t tiles_x, uint32_t tiles_total, uint32_t width,
                                                       uint32_t height, uint32_t *__restrict__ frame) {
    const uint64_t tile_px = (uint64_t)tile_w * tile_h;
    const uint64_t total = (uint64_t)tile_count * slab_tiles * tile_px;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t slab = i / (slab_tiles * tile_px);
        const uint64_t rem = i % (slab_tiles * tile_px);
        const uint32_t k = (uint32_t)(rem / tile_px);
        const uint32_t p = (uint32_t)(rem % tile_px);
        const uint32_t t = (uint32_t)slab + k * tile_count;
        if (t >= tiles_total) continue;
        const uint32_t x = (t % tiles_x) * tile_w + p % tile_w;
        const uint32_t y = (t / tiles_x) * tile_h + p / tile_w;
        if (x < width && y < height) frame[(size_t)y * width + x] = gathered[i];
    }
}

hipError_t launch_assemble(const void *gathered, uint32_t slab_tiles, uint32_t tile_w, uint32_t tile_h,
                           uint32_t tile_count, uint32_t width, uint32_t height, void *frame, hipStream_t stream) {
    const uint32_t tiles_x = (width + tile_w - 1) / tile_w;
    const uint32_t tiles_y = (height + tile_h - 1) / tile_h;
    const uint64_t total = (uint64_t)tile_count * slab_tiles * tile_w * tile_h;
    if (total == 0) return hipSuccess;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(assemble_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream,
                       static_cast<const uint32_t *>(gathered), slab_tiles, tile_w, tile_h, tile_count, tiles_x,
                       tiles_x * tiles_y, width, height, static_cast<uint32_t *>(frame));
    return hipGetLastError();
}

}  // namespace rtamd
