// sort_bench.hip — rocPRIM onesweep radix-sort configurations over the LBVH builder's sort (C5: one segment of
// ~10 M (30-bit Morton code, item) pairs).  The builder's default call sorts 8-bit digits (4 passes over 30 bits);
// 10- or 11-bit digits take 3.  Prints one line per configuration: mean ms per sort, and whether its output equals
// the default configuration's (keys and values: the radix sort is stable, so every configuration must agree).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/sort_bench.hip -o /tmp/sort_bench && /tmp/sort_bench [n]
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

static uint32_t expand10(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

template <class Config>
static double run(const char *name, uint32_t n, const uint32_t *k0, uint32_t *k1, const uint32_t *v0, uint32_t *v1,
                  const std::vector<uint32_t> *ref_k, const std::vector<uint32_t> *ref_v, std::vector<uint32_t> *out_k,
                  std::vector<uint32_t> *out_v) {
    size_t bytes = 0;
    CK(rocprim::radix_sort_pairs<Config>(nullptr, bytes, k0, k1, v0, v1, n, 0, 30, 0));
    void *tmp = nullptr;
    CK(hipMalloc(&tmp, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int w = 0; w < 3; w++) CK(rocprim::radix_sort_pairs<Config>(tmp, bytes, k0, k1, v0, v1, n, 0, 30, 0));
    const int reps = 20;
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; r++) CK(rocprim::radix_sort_pairs<Config>(tmp, bytes, k0, k1, v0, v1, n, 0, 30, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint32_t> hk(n), hv(n);
    CK(hipMemcpy(hk.data(), k1, 4ull * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hv.data(), v1, 4ull * n, hipMemcpyDeviceToHost));
    const bool same = !ref_k || (hk == *ref_k && hv == *ref_v);
    std::printf("%-34s %8.4f ms  tmp %7.1f MB  %s\n", name, ms / reps, bytes / 1e6, same ? "equal" : "DIFFERENT");
    if (out_k) { *out_k = hk; *out_v = hv; }
    CK(hipFree(tmp));
    return ms / reps;
}

using rocprim::kernel_config;
template <unsigned B, unsigned HB, unsigned HI, unsigned SB, unsigned SI>
using OS = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<kernel_config<HB, HI>, kernel_config<SB, SI>, B,
                                        rocprim::block_radix_rank_algorithm::match>>;

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 10000000u;
    // keys: Morton codes of clustered points (a particle soup: ~1000-point clusters in a unit cube), item order
    // = cluster order, as the builder's group segment holds them
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    std::normal_distribution<float> G(0.0f, 0.004f);
    std::vector<uint32_t> hk(n), hv(n);
    float cx = 0, cy = 0, cz = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (i % 1024 == 0) { cx = U(rng); cy = U(rng); cz = U(rng); }
        auto q = [](float c) { int v = (int)(c * 1024.0f); return (uint32_t)(v < 0 ? 0 : (v > 1023 ? 1023 : v)); };
        hk[i] = (expand10(q(cx + G(rng))) << 2) | (expand10(q(cy + G(rng))) << 1) | expand10(q(cz + G(rng)));
        hv[i] = i;
    }
    uint32_t *k0, *k1, *v0, *v1;
    CK(hipMalloc(&k0, 4ull * n)); CK(hipMalloc(&k1, 4ull * n)); CK(hipMalloc(&v0, 4ull * n)); CK(hipMalloc(&v1, 4ull * n));
    CK(hipMemcpy(k0, hk.data(), 4ull * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(v0, hv.data(), 4ull * n, hipMemcpyHostToDevice));
    std::vector<uint32_t> rk, rv;
    std::printf("n = %u pairs (%.1f MB in, 30-bit keys)\n", n, 8e-6 * n);
    run<rocprim::default_config>("default (8-bit digits)", n, k0, k1, v0, v1, nullptr, nullptr, &rk, &rv);
    run<OS<8, 1024, 16, 1024, 16>>("onesweep  8 sort1024x16", n, k0, k1, v0, v1, &rk, &rv, nullptr, nullptr);
    run<OS<8, 1024, 16, 1024, 24>>("onesweep  8 sort1024x24", n, k0, k1, v0, v1, &rk, &rv, nullptr, nullptr);
    run<OS<8, 1024, 16, 512, 24>>("onesweep  8 sort512x24", n, k0, k1, v0, v1, &rk, &rv, nullptr, nullptr);
    run<OS<9, 1024, 16, 1024, 16>>("onesweep  9 sort1024x16", n, k0, k1, v0, v1, &rk, &rv, nullptr, nullptr);
    run<OS<10, 1024, 16, 1024, 16>>("onesweep 10 sort1024x16", n, k0, k1, v0, v1, &rk, &rv, nullptr, nullptr);
    run<OS<10, 1024, 16, 1024, 12>>("onesweep 10 sort1024x12", n, k0, k1, v0, v1, &rk, &rv, nullptr, nullptr);
    run<OS<10, 1024, 16, 512, 16>>("onesweep 10 sort512x16", n, k0, k1, v0, v1, &rk, &rv, nullptr, nullptr);
    run<OS<10, 1024, 16, 1024, 24>>("onesweep 10 sort1024x24", n, k0, k1, v0, v1, &rk, &rv, nullptr, nullptr);
    run<OS<11, 1024, 16, 1024, 16>>("onesweep 11 sort1024x16", n, k0, k1, v0, v1, &rk, &rv, nullptr, nullptr);
    run<OS<11, 1024, 16, 1024, 24>>("onesweep 11 sort1024x24", n, k0, k1, v0, v1, &rk, &rv, nullptr, nullptr);
    run<OS<11, 1024, 16, 512, 24>>("onesweep 11 sort512x24", n, k0, k1, v0, v1, &rk, &rv, nullptr, nullptr);
    return 0;
}
