// write_cal.hip — calibrates rocprofv3 WRITE_SIZE for the framebuffer store patterns of the render kernel
// (verdict r2 "write amplification": WRITE_SIZE 15.1 MB per C2 launch against an 8.29 MB RGBA8 frame).
// Every kernel stores the same 1920x1080 RGBA8 frame once; only the store pattern differs:
//   linear16      16 B per lane, row-major (the guide's exact case)
//   linear4       4 B per lane, row-major
//   tile_block4   8x8-pixel tiles (one per wave, rows of 32 B), four horizontally adjacent tiles per
//                 256-thread workgroup: the four 32-B pieces of each 128-B line leave one CU
//   tile_wave_rr  one tile per 64-thread workgroup in row-major tile order: consecutive workgroups are
//                 dispatched round-robin over the 8 XCDs, so a line's four pieces leave four L2s
//   tile_perm     tiles in a fixed pseudo-random order (a heaviest-first claim order looks like this)
// Build: hipcc --offload-arch=gfx950 -O3 write_cal.hip -o write_cal ; run under rocprofv3 --pmc WRITE_SIZE
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int W = 1920, H = 1080, TX = W / 8, TY = H / 8 + 1;   // 1080 = 135 tiles of 8 rows exactly
constexpr int TILES = (W / 8) * (H / 8);

__device__ __forceinline__ uint32_t px(int x, int y, uint32_t salt) { return (uint32_t)(x * 2654435761u) ^ (uint32_t)y ^ salt; }

__global__ void linear16(uint4 *out, uint32_t salt) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= W * H / 4) return;
    const int p = 4 * i, x = p % W, y = p / W;
    out[i] = make_uint4(px(x, y, salt), px(x + 1, y, salt), px(x + 2, y, salt), px(x + 3, y, salt));
}
__global__ void linear4(uint32_t *out, uint32_t salt) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= W * H) return;
    out[i] = px(i % W, i / W, salt);
}
__device__ __forceinline__ void store_tile(uint32_t *out, int t, uint32_t salt) {
    const int lane = threadIdx.x & 63, tx = t % (W / 8), ty = t / (W / 8);
    const int x = tx * 8 + (lane & 7), y = ty * 8 + (lane >> 3);
    out[(size_t)y * W + x] = px(x, y, salt);
}
__global__ void tile_block4(uint32_t *out, uint32_t salt) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t < TILES) store_tile(out, t, salt);
}
__global__ void tile_wave_rr(uint32_t *out, uint32_t salt) {
    if ((int)blockIdx.x < TILES) store_tile(out, blockIdx.x, salt);
}
__global__ void tile_perm(uint32_t *out, const uint32_t *perm, uint32_t salt) {
    if ((int)blockIdx.x < TILES) store_tile(out, perm[blockIdx.x], salt);
}

int main() {
    uint32_t *out, *perm;
    CHECK(hipMalloc(&out, (size_t)W * H * 4));
    CHECK(hipMalloc(&perm, TILES * 4));
    uint32_t *hp = (uint32_t *)malloc(TILES * 4);
    for (int i = 0; i < TILES; i++) hp[i] = i;
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (int i = TILES - 1; i > 0; i--) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const int j = (int)(s % (uint64_t)(i + 1));
        const uint32_t tmp = hp[i]; hp[i] = hp[j]; hp[j] = tmp;
    }
    CHECK(hipMemcpy(perm, hp, TILES * 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 5; rep++) {
        const uint32_t salt = 77u * rep;
        hipLaunchKernelGGL(linear16, dim3((W * H / 4 + 255) / 256), dim3(256), 0, 0, (uint4 *)out, salt);
        hipLaunchKernelGGL(linear4, dim3((W * H + 255) / 256), dim3(256), 0, 0, out, salt);
        hipLaunchKernelGGL(tile_block4, dim3((TILES + 3) / 4), dim3(256), 0, 0, out, salt);
        hipLaunchKernelGGL(tile_wave_rr, dim3(TILES), dim3(64), 0, 0, out, salt);
        hipLaunchKernelGGL(tile_perm, dim3(TILES), dim3(64), 0, 0, out, perm, salt);
        CHECK(hipDeviceSynchronize());
    }
    CHECK(hipGetLastError());
    printf("frame bytes %d, tiles %d (TX %d TY %d)\n", W * H * 4, TILES, TX, TY);
    return 0;
}
