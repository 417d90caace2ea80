// scan_bench.hip — rocPRIM exclusive_scan configurations over the LBVH builder's pair-index scan (C5: ~10 M interior
// nodes, kept flags 0 / 1, about a third set).  Prints one line per configuration: mean ms per scan and whether the
// output equals the default configuration's.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/scan_bench.hip -o /tmp/scan_bench && /tmp/scan_bench [n]
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan.hpp>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

template <class Config>
static void run(const char *name, uint32_t n, const uint32_t *in, uint32_t *out, const std::vector<uint32_t> *ref,
                std::vector<uint32_t> *keep) {
    size_t bytes = 0;
    CK(rocprim::exclusive_scan<Config>(nullptr, bytes, in, out, 0u, n, rocprim::plus<uint32_t>(), 0));
    void *tmp = nullptr;
    CK(hipMalloc(&tmp, bytes ? bytes : 1));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int w = 0; w < 3; w++) CK(rocprim::exclusive_scan<Config>(tmp, bytes, in, out, 0u, n, rocprim::plus<uint32_t>(), 0));
    const int reps = 50;
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; r++) CK(rocprim::exclusive_scan<Config>(tmp, bytes, in, out, 0u, n, rocprim::plus<uint32_t>(), 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint32_t> h(n);
    CK(hipMemcpy(h.data(), out, 4ull * n, hipMemcpyDeviceToHost));
    std::printf("%-28s %8.4f ms  %s\n", name, ms / reps, (!ref || h == *ref) ? "equal" : "DIFFERENT");
    if (keep) *keep = h;
    CK(hipFree(tmp));
}

template <unsigned B, unsigned I>
using SC = rocprim::scan_config<B, I, rocprim::block_load_method::block_load_transpose,
                                rocprim::block_store_method::block_store_transpose, rocprim::block_scan_algorithm::using_warp_scan>;

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 10000000u;
    std::mt19937 rng(3);
    std::vector<uint32_t> h(n);
    for (auto &v : h) v = (rng() % 3) == 0;
    uint32_t *in, *out;
    CK(hipMalloc(&in, 4ull * n)); CK(hipMalloc(&out, 4ull * n));
    CK(hipMemcpy(in, h.data(), 4ull * n, hipMemcpyHostToDevice));
    std::vector<uint32_t> ref;
    std::printf("n = %u flags\n", n);
    run<rocprim::default_config>("default", n, in, out, nullptr, &ref);
    run<SC<256, 16>>("256 x 16", n, in, out, &ref, nullptr);
    run<SC<256, 32>>("256 x 32", n, in, out, &ref, nullptr);
    run<SC<256, 8>>("256 x 8", n, in, out, &ref, nullptr);
    run<SC<128, 32>>("128 x 32", n, in, out, &ref, nullptr);
    return 0;
}
