// Host check that build_sah_tree (presorted lists, csrc/bvh_build.hpp) builds the same tree as
// build_sah_tree_nodewise (per-node sorts): nodes (boxes, counts, child / slot indices) and leaf refs
// identical.  Inputs: random boxes, grid-snapped centroids (ties), flat axes, all-equal centroids.
// Prints one JSON line; built and run by tests/test_sah_presort.py (g++, CPU).
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>

#include "../../real-time-gpu-ray-tracer_amd/csrc/bvh_build.hpp"

using namespace rtamd;

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 258;
    const int kind = argc > 2 ? atoi(argv[2]) : 0;       // 0 random, 1 grid ties, 2 flat y, 3 all equal
    const uint32_t leaf = argc > 3 ? (uint32_t)atoi(argv[3]) : 1;
    std::mt19937 rng(n * 13 + kind * 7 + leaf);
    std::uniform_real_distribution<float> U(-10.0f, 10.0f), S(0.01f, 1.0f);
    std::vector<BuildItem> items(n);
    for (uint32_t i = 0; i < n; i++) {
        float x = U(rng), y = U(rng), z = U(rng);
        const float s = S(rng);
        if (kind == 1) { x = std::round(x); y = std::round(y * 0.3f); z = std::round(z); }
        if (kind == 2) y = 1.0f;
        if (kind == 3) { x = 1.0f; y = 2.0f; z = 3.0f; }
        items[i].box = hm::Box{{{x - s, x + s}, {y - s, y + s}, {z - s, z + s}}};
        items[i].centroid = hm::V3{x, y, z};
        items[i].index = i;                               // caller indices = positions
    }
    const auto t0 = std::chrono::steady_clock::now();
    const Tree a = build_sah_tree_nodewise(items, leaf);
    const auto t1 = std::chrono::steady_clock::now();
    const Tree b = build_sah_tree(items, leaf);
    const auto t2 = std::chrono::steady_clock::now();
    bool same = a.nodes.size() == b.nodes.size() && a.refs == b.refs;
    for (size_t k = 0; same && k < a.nodes.size(); k++)
        same = a.nodes[k].count == b.nodes[k].count && a.nodes[k].index == b.nodes[k].index &&
               std::memcmp(&a.nodes[k].box, &b.nodes[k].box, sizeof(hm::Box)) == 0;
    printf("{\"n\": %u, \"kind\": %d, \"leaf\": %u, \"nodes\": %zu, \"same\": %d, \"nodewise_ms\": %.3f, \"presort_ms\": %.3f}\n",
           n, kind, leaf, a.nodes.size(), same ? 1 : 0,
           std::chrono::duration<double, std::milli>(t1 - t0).count(), std::chrono::duration<double, std::milli>(t2 - t1).count());
    return 0;
}
