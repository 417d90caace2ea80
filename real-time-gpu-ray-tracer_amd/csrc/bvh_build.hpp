// bvh_build.hpp — top-down median-split BVH builder (compat mode) and its flattening into
// the node-pair layout of layout.hpp.
//
// Restates BLAS::constructBLAS (src/AS/BLAS.cu:4-117) and TLAS::constructTLAS
// (src/AS/TLAS.cu:4-129): a task stack seeded with the root; a task with <= leaf_cap items
// becomes a leaf (its items appended to the index array in DFS order), otherwise two child
// nodes are allocated at the next free indices (left, left+1), the items are sorted by centroid
// on a pseudo-random axis and split at count/2, and the right task is pushed before the left.
// Node boxes are the union of the items' boxes (constructBoundingBoxForPrimitiveList).
// Deviations: the axis stream is a pinned function of the build seed instead of
// std::mt19937(random_device), and centroid ties are ordered by item index (std::sort leaves
// them unspecified).
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

#include "host_math.hpp"
#include "layout.hpp"

namespace rtamd {

struct BuildItem {
    hm::Box box;
    hm::V3 centroid;
    uint32_t index;      // caller's item index (primitive index / instance index)
};

struct TreeNode {        // BLASNode / TLASNode (BLAS.cuh:20-34, TLAS.cuh:24-39)
    hm::Box box;
    uint32_t count;      // > 0: leaf with `count` items starting at index-array slot `index`
    uint32_t index;      // interior: left child node index (right = index + 1)
};

struct Tree {
    std::vector<TreeNode> nodes;
    std::vector<uint32_t> refs;    // item index per leaf slot, DFS leaf order
};

inline Tree build_median_tree(std::vector<BuildItem> items, uint32_t leaf_cap, uint64_t axis_state) {
    Tree t;
    const uint32_t n = (uint32_t)items.size();
    t.nodes.resize(n ? 2 * (size_t)n - 1 : 0);
    t.refs.reserve(n);
    if (n == 0) return t;
    struct Task { uint32_t start, count, node; };
    std::vector<Task> stack;
    stack.push_back({0, n, 0});
    uint32_t node_count = 1;
    while (!stack.empty()) {
        const Task task = stack.back();
        stack.pop_back();
        TreeNode &node = t.nodes[task.node];
        hm::Box bb = items[task.start].box;
        for (uint32_t i = task.start + 1; i < task.start + task.count; i++) bb = hm::Box::merge(bb, items[i].box);
        node.box = bb;
        if (task.count <= leaf_cap) {
            node.count = task.count;
            node.index = (uint32_t)t.refs.size();
            for (uint32_t i = 0; i < task.count; i++) t.refs.push_back(items[task.start + i].index);
        } else {
            const uint32_t left = node_count++, right = node_count++;
            (void)right;
            const int axis = hm::draw_axis(axis_state);
            std::sort(items.begin() + task.start, items.begin() + task.start + task.count,
                      [axis](const BuildItem &a, const BuildItem &b) {
                          const float fa = a.centroid[axis], fb = b.centroid[axis];
                          if (fa < fb) return true;
                          if (fb < fa) return false;
                          return a.index < b.index;
                      });
            node.count = 0;
            node.index = left;
            const uint32_t mid = task.count / 2;
            stack.push_back({task.start + mid, task.count - mid, left + 1});
            stack.push_back({task.start, mid, left});
        }
    }
    t.nodes.resize(node_count);
    return t;
}

// Flattened form of one tree in the node-pair layout.
struct FlatTree {
    std::vector<NodePair> pairs;   // one per interior node
    uint32_t root_ref = 0;
    float root_box[6] = {0, 0, 0, 0, 0, 0};
    uint32_t leaves = 0;
};

// pair_base: index of this tree's first pair in the global pair array; slot_base: index of the
// tree's first leaf slot in the (leaf-ordered) item array; ptype: BLAS primitive type.
inline FlatTree flatten_tree(const Tree &t, uint32_t pair_base, uint32_t slot_base, uint32_t ptype, bool blas) {
    FlatTree f;
    const uint32_t n = (uint32_t)t.nodes.size();
    std::vector<uint32_t> pair_of(n, 0);
    uint32_t np = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (t.nodes[i].count == 0) pair_of[i] = np++;
        else f.leaves++;
    }
    auto ref_of = [&](uint32_t j) -> uint32_t {
        const TreeNode &nd = t.nodes[j];
        if (nd.count > 0) return make_leaf_ref(slot_base + nd.index, nd.count, ptype, blas);
        return make_interior_ref(pair_base + pair_of[j], blas);
    };
    f.pairs.resize(np);
    for (uint32_t i = 0; i < n; i++) {
        const TreeNode &nd = t.nodes[i];
        if (nd.count > 0) continue;
        NodePair &p = f.pairs[pair_of[i]];
        t.nodes[nd.index].box.store(p.c0);
        t.nodes[nd.index + 1].box.store(p.c1);
        p.ref0 = ref_of(nd.index);
        p.ref1 = ref_of(nd.index + 1);
        p.pad0 = p.pad1 = 0;
    }
    if (n) {
        f.root_ref = ref_of(0);
        t.nodes[0].box.store(f.root_box);
    }
    return f;
}

}  // namespace rtamd
