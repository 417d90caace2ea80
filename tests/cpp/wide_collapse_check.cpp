// Host check of flatten_tree_wide (csrc/bvh_build.hpp): the quad form of a binary tree covers exactly
// the binary tree's leaf slots (each once), its child boxes are binary node boxes, every quad holds two halves
// whose union boxes are binary node boxes too (a half = one binary child, layout.hpp NodeQuad), and an empty
// slot repeats its sibling's box.  Built and run by tests/test_wide_collapse.py (g++, CPU).
#include <algorithm>
#include <cstdio>
#include <map>
#include <random>
#include <set>

#include "../../real-time-gpu-ray-tracer_amd/csrc/bvh_build.hpp"

using namespace rtamd;

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000;
    const int sah = argc > 2 ? atoi(argv[2]) : 1;
    const bool halves = argc > 3 ? atoi(argv[3]) != 0 : true;        // two binary levels per quad, else greedy
    std::mt19937 rng(n * 7 + sah);
    std::uniform_real_distribution<float> U(-10.0f, 10.0f), S(0.01f, 1.0f);
    std::vector<BuildItem> items(n);
    for (uint32_t i = 0; i < n; i++) {
        const float x = U(rng), y = U(rng), z = U(rng), s = S(rng);
        items[i].box = hm::Box::from_ranges({x, x + s}, {y, y + s}, {z, z + s});
        items[i].centroid = hm::v3(x + s / 2, y + s / 2, z + s / 2);
        items[i].index = i;
    }
    const Tree t = sah ? build_sah_tree(items, 4) : build_median_tree(items, 4, 12345);
    const FlatTree f2 = flatten_tree(t, 0, 100, 2, true);
    const FlatWide f4 = flatten_tree_wide(t, 0, 100, 2, true, halves);
    // leaves and boxes reachable from each form
    std::multiset<uint32_t> leaves2, leaves4;
    std::set<std::vector<float>> boxes2, boxes4;
    std::vector<uint32_t> todo{f2.root_ref};
    while (!todo.empty()) {
        const uint32_t r = todo.back(); todo.pop_back();
        if (r & REF_LEAF) { for (uint32_t k = 0; k < ref_leaf_count(r); k++) leaves2.insert(ref_leaf_start(r) + k); continue; }
        const NodePair &p = f2.pairs[r & REF_INDEX_MASK];
        boxes2.insert(std::vector<float>(p.c0, p.c0 + 6)); boxes2.insert(std::vector<float>(p.c1, p.c1 + 6));
        todo.push_back(p.ref0); todo.push_back(p.ref1);
    }
    int bad = 0, quads = 0, children = 0, min_children = 4;
    todo = {f4.root_ref};
    while (!todo.empty()) {
        const uint32_t r = todo.back(); todo.pop_back();
        if (r & REF_LEAF) { for (uint32_t k = 0; k < ref_leaf_count(r); k++) leaves4.insert(ref_leaf_start(r) + k); continue; }
        const NodeQuad &q = f4.quads[r & REF_INDEX_MASK];
        quads++;
        int nc = 0;
        bad += q.ref[0] == REF_EMPTY || (halves && q.ref[2] == REF_EMPTY); // a half's first slot is always used
        for (int hh = 0; halves && hh < 2; hh++) {                         // the half's box: a binary node box
            const int a = 2 * hh, b = 2 * hh + 1;
            const float u[6] = {std::min(q.lo_x[a], q.lo_x[b]), std::max(q.hi_x[a], q.hi_x[b]),
                                std::min(q.lo_y[a], q.lo_y[b]), std::max(q.hi_y[a], q.hi_y[b]),
                                std::min(q.lo_z[a], q.lo_z[b]), std::max(q.hi_z[a], q.hi_z[b])};
            bad += boxes2.count(std::vector<float>(u, u + 6)) == 0;
        }
        for (int k = 0; k < 4; k++) {
            if (q.ref[k] == REF_EMPTY && !halves) {
                bad += !(q.lo_x[k] == INFINITY && q.hi_x[k] == INFINITY && q.lo_z[k] == INFINITY && q.hi_z[k] == INFINITY);
                continue;
            }
            if (q.ref[k] == REF_EMPTY) {
                const int s = k ^ 1;
                bad += !(q.lo_x[k] == q.lo_x[s] && q.hi_x[k] == q.hi_x[s] && q.lo_y[k] == q.lo_y[s] &&
                         q.hi_y[k] == q.hi_y[s] && q.lo_z[k] == q.lo_z[s] && q.hi_z[k] == q.hi_z[s]);
                continue;
            }
            nc++;
            const float b[6] = {q.lo_x[k], q.hi_x[k], q.lo_y[k], q.hi_y[k], q.lo_z[k], q.hi_z[k]};
            const std::vector<float> v(b, b + 6);
            bad += boxes2.count(v) == 0;          // every quad child box is a binary node box
            boxes4.insert(v);
            todo.push_back(q.ref[k]);
        }
        children += nc;
        min_children = nc < min_children ? nc : min_children;
    }
    printf("{\"n\": %u, \"sah\": %d, \"halves\": %d, \"slots_equal\": %d, \"bad_boxes\": %d, \"quads\": %d, \"pairs\": %zu, "
           "\"mean_children\": %.3f, \"min_children\": %d, \"height2\": %u, \"height4\": %u}\n",
           n, sah, (int)halves, (int)(leaves2 == leaves4), bad, quads, f2.pairs.size(), quads ? (double)children / quads : 0.0,
           min_children, f2.height, f4.height);
    return 0;
}
