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
#include <limits>
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

// ---- SAH builder (RT_BUILD_SAH) ---------------------------------------------------------------
// Top-down surface-area-heuristic build: for each node, the split minimising
//   C = C_trav + (A_L / A) * N_L * C_isect + (A_R / A) * N_R * C_isect
// over the centroid-sorted sweeps of all three axes (exact sweep up to `sweep_max` items, 32 binned
// planes above that); a node becomes a leaf when it holds <= leaf_cap items and the leaf cost
// N * C_isect is not worse than the best split.  Output uses the same node convention as the
// median builder (children at index, index+1; leaves index a DFS-ordered item array), so the
// flattening and the kernels are unchanged.  Trees differ from the reference's, so results differ
// only where two surfaces tie within the 1e-6 window (FAST tolerance).
inline float half_area(const hm::Box &b) {
    const float dx = b.r[0].max - b.r[0].min, dy = b.r[1].max - b.r[1].min, dz = b.r[2].max - b.r[2].min;
    return dx * dy + dy * dz + dz * dx;
}

// Reference form: every node re-sorts its items along each axis (O(n log^2 n)); build_sah_tree below
// produces the same tree from lists presorted once.  Kept for lists above sweep_max (binned planes) and as
// the equivalence check's reference (tests/cpp/sah_presort_check.cpp).
inline Tree build_sah_tree_nodewise(std::vector<BuildItem> items, uint32_t leaf_cap, float c_trav = 1.0f,
                                    float c_isect = 1.0f, uint32_t sweep_max = 4096) {
    Tree t;
    const uint32_t n = (uint32_t)items.size();
    t.nodes.resize(n ? 2 * (size_t)n - 1 : 0);
    t.refs.reserve(n);
    if (n == 0) return t;
    struct Task { uint32_t start, count, node; };
    std::vector<Task> stack;
    stack.push_back({0, n, 0});
    uint32_t node_count = 1;
    std::vector<float> right_area(n + 1);
    while (!stack.empty()) {
        const Task task = stack.back();
        stack.pop_back();
        TreeNode &node = t.nodes[task.node];
        hm::Box bb = items[task.start].box;
        hm::Box cb{{{items[task.start].centroid.x, items[task.start].centroid.x},
                    {items[task.start].centroid.y, items[task.start].centroid.y},
                    {items[task.start].centroid.z, items[task.start].centroid.z}}};
        for (uint32_t i = task.start + 1; i < task.start + task.count; i++) {
            bb = hm::Box::merge(bb, items[i].box);
            for (int a = 0; a < 3; a++) {
                cb.r[a].min = std::min(cb.r[a].min, items[i].centroid[a]);
                cb.r[a].max = std::max(cb.r[a].max, items[i].centroid[a]);
            }
        }
        node.box = bb;
        const uint32_t cnt = task.count;
        const float parent_area = std::max(half_area(bb), 1e-30f);
        float best_cost = INFINITY;
        int best_axis = -1;
        uint32_t best_mid = 0;
        float best_plane = 0.0f;
        if (cnt > 1) {
            for (int axis = 0; axis < 3; axis++) {
                if (!(cb.r[axis].max > cb.r[axis].min)) continue;
                if (cnt <= sweep_max) {
                    std::sort(items.begin() + task.start, items.begin() + task.start + cnt,
                              [axis](const BuildItem &a, const BuildItem &b) {
                                  const float fa = a.centroid[axis], fb = b.centroid[axis];
                                  return fa < fb || (!(fb < fa) && a.index < b.index);
                              });
                    hm::Box acc = items[task.start + cnt - 1].box;
                    right_area[cnt - 1] = half_area(acc);
                    for (int64_t i = (int64_t)cnt - 2; i >= 1; i--) {
                        acc = hm::Box::merge(acc, items[task.start + i].box);
                        right_area[i] = half_area(acc);
                    }
                    acc = items[task.start].box;
                    for (uint32_t i = 1; i < cnt; i++) {          // left = [0, i), right = [i, cnt)
                        const float c = c_trav + (half_area(acc) * i + right_area[i] * (cnt - i)) * c_isect / parent_area;
                        if (c < best_cost) { best_cost = c; best_axis = axis; best_mid = i; }
                        acc = hm::Box::merge(acc, items[task.start + i].box);
                    }
                } else {
                    constexpr int NB = 32;
                    hm::Box bbox[NB];
                    uint32_t bcnt[NB] = {0};
                    const float lo = cb.r[axis].min, ext = cb.r[axis].max - cb.r[axis].min;
                    for (uint32_t i = task.start; i < task.start + cnt; i++) {
                        int b = (int)((items[i].centroid[axis] - lo) / ext * NB);
                        b = b < 0 ? 0 : (b >= NB ? NB - 1 : b);
                        bbox[b] = bcnt[b] ? hm::Box::merge(bbox[b], items[i].box) : items[i].box;
                        bcnt[b]++;
                    }
                    float ra[NB];
                    uint32_t rc[NB];
                    hm::Box acc{};
                    uint32_t accn = 0;
                    for (int b = NB - 1; b >= 1; b--) {
                        if (bcnt[b]) { acc = accn ? hm::Box::merge(acc, bbox[b]) : bbox[b]; accn += bcnt[b]; }
                        ra[b] = accn ? half_area(acc) : 0.0f;
                        rc[b] = accn;
                    }
                    accn = 0;
                    for (int b = 0; b < NB - 1; b++) {
                        if (bcnt[b]) { acc = accn ? hm::Box::merge(acc, bbox[b]) : bbox[b]; accn += bcnt[b]; }
                        if (accn == 0 || rc[b + 1] == 0) continue;
                        const float c = c_trav + (half_area(acc) * accn + ra[b + 1] * rc[b + 1]) * c_isect / parent_area;
                        if (c < best_cost) { best_cost = c; best_axis = axis; best_plane = lo + ext * (float)(b + 1) / NB; best_mid = accn; }
                    }
                }
            }
        }
        const float leaf_cost = c_isect * cnt;
        if (cnt <= leaf_cap && (best_axis < 0 || leaf_cost <= best_cost)) {
            node.count = cnt;
            node.index = (uint32_t)t.refs.size();
            for (uint32_t i = 0; i < cnt; i++) t.refs.push_back(items[task.start + i].index);
            continue;
        }
        uint32_t mid;
        if (best_axis < 0) {
            mid = cnt / 2;                                // all centroids equal: split the list
        } else if (cnt <= sweep_max) {
            const int axis = best_axis;
            std::sort(items.begin() + task.start, items.begin() + task.start + cnt,
                      [axis](const BuildItem &a, const BuildItem &b) {
                          const float fa = a.centroid[axis], fb = b.centroid[axis];
                          return fa < fb || (!(fb < fa) && a.index < b.index);
                      });
            mid = best_mid;
        } else {
            const int axis = best_axis;
            const float plane = best_plane;
            auto it = std::partition(items.begin() + task.start, items.begin() + task.start + cnt,
                                     [axis, plane](const BuildItem &a) { return a.centroid[axis] < plane; });
            mid = (uint32_t)(it - (items.begin() + task.start));
            if (mid == 0 || mid == cnt) mid = cnt / 2;
        }
        const uint32_t left = node_count++, right = node_count++;
        (void)right;
        node.count = 0;
        node.index = left;
        stack.push_back({task.start + mid, cnt - mid, left + 1});
        stack.push_back({task.start, mid, left});
    }
    t.nodes.resize(node_count);
    return t;
}

// The exact-sweep SAH build (n <= sweep_max) from three centroid-sorted index lists sorted once and
// split stably at every node, O(n log n): the per-frame SAH TLAS over C3's 258 instances took 0.29 ms
// with per-node sorting, which bounded a C4 rank's frame rate (scripts/host_overhead.py).  The tree is
// identical to build_sah_tree_nodewise's: the same (centroid, index) orders, the same cost arithmetic
// over the same boxes (min / max merges do not depend on merge order), the same tie rules, the same
// item order inside leaves and under "all centroids equal" splits, and the same DFS numbering.
inline Tree build_sah_tree(std::vector<BuildItem> items, uint32_t leaf_cap, float c_trav = 1.0f, float c_isect = 1.0f,
                           uint32_t sweep_max = 4096) {
    const uint32_t n = (uint32_t)items.size();
    if (n > sweep_max) return build_sah_tree_nodewise(std::move(items), leaf_cap, c_trav, c_isect, sweep_max);
    Tree t;
    t.nodes.resize(n ? 2 * (size_t)n - 1 : 0);
    t.refs.reserve(n);
    if (n == 0) return t;
    // ord[a]: item ids sorted by (centroid[a], index) inside every pending node's range; cur: the node's
    // incoming order (its parent's split order), which the nodewise builder leaves in place when no axis
    // of the node has centroid extent
    std::vector<uint32_t> ord[3], cur(n), tmp(n);
    std::vector<uint8_t> left_side(n);
    for (int a = 0; a < 3; a++) {
        ord[a].resize(n);
        for (uint32_t i = 0; i < n; i++) ord[a][i] = i;
        std::sort(ord[a].begin(), ord[a].end(), [&](uint32_t x, uint32_t y) {
            const float fa = items[x].centroid[a], fb = items[y].centroid[a];
            return fa < fb || (!(fb < fa) && items[x].index < items[y].index);
        });
    }
    for (uint32_t i = 0; i < n; i++) cur[i] = i;
    struct Task { uint32_t start, count, node; };
    std::vector<Task> stack;
    stack.push_back({0, n, 0});
    uint32_t node_count = 1;
    std::vector<float> right_area(n + 1);
    while (!stack.empty()) {
        const Task task = stack.back();
        stack.pop_back();
        TreeNode &node = t.nodes[task.node];
        const uint32_t s0 = task.start, cnt = task.count;
        const uint32_t *o0 = ord[0].data() + s0;
        hm::Box bb = items[o0[0]].box;
        hm::Box cb{{{items[o0[0]].centroid.x, items[o0[0]].centroid.x},
                    {items[o0[0]].centroid.y, items[o0[0]].centroid.y},
                    {items[o0[0]].centroid.z, items[o0[0]].centroid.z}}};
        for (uint32_t i = 1; i < cnt; i++) {
            const BuildItem &it = items[o0[i]];
            bb = hm::Box::merge(bb, it.box);
            for (int a = 0; a < 3; a++) {
                cb.r[a].min = std::min(cb.r[a].min, it.centroid[a]);
                cb.r[a].max = std::max(cb.r[a].max, it.centroid[a]);
            }
        }
        node.box = bb;
        const float parent_area = std::max(half_area(bb), 1e-30f);
        float best_cost = INFINITY;
        int best_axis = -1, last_axis = -1;
        uint32_t best_mid = 0;
        if (cnt > 1) {
            for (int axis = 0; axis < 3; axis++) {
                if (!(cb.r[axis].max > cb.r[axis].min)) continue;
                last_axis = axis;
                const uint32_t *o = ord[axis].data() + s0;
                hm::Box acc = items[o[cnt - 1]].box;
                right_area[cnt - 1] = half_area(acc);
                for (int64_t i = (int64_t)cnt - 2; i >= 1; i--) {
                    acc = hm::Box::merge(acc, items[o[i]].box);
                    right_area[i] = half_area(acc);
                }
                acc = items[o[0]].box;
                for (uint32_t i = 1; i < cnt; i++) {
                    const float c = c_trav + (half_area(acc) * i + right_area[i] * (cnt - i)) * c_isect / parent_area;
                    if (c < best_cost) { best_cost = c; best_axis = axis; best_mid = i; }
                    acc = hm::Box::merge(acc, items[o[i]].box);
                }
            }
        }
        const float leaf_cost = c_isect * cnt;
        if (cnt <= leaf_cap && (best_axis < 0 || leaf_cost <= best_cost)) {
            // the nodewise builder's item order here: its last axis sort, else the incoming order
            const uint32_t *o = last_axis >= 0 ? ord[last_axis].data() + s0 : cur.data() + s0;
            node.count = cnt;
            node.index = (uint32_t)t.refs.size();
            for (uint32_t i = 0; i < cnt; i++) t.refs.push_back(items[o[i]].index);
            continue;
        }
        // the split order: the best axis's; without a split plane (all centroids equal) the order in
        // place, cut in half
        const uint32_t mid = best_axis >= 0 ? best_mid : cnt / 2;
        const int split_axis = best_axis >= 0 ? best_axis : last_axis;
        uint32_t *split = split_axis >= 0 ? ord[split_axis].data() + s0 : cur.data() + s0;
        for (uint32_t i = 0; i < cnt; i++) left_side[split[i]] = i < mid ? 1 : 0;
        if (split_axis >= 0) std::copy(split, split + cnt, cur.begin() + s0);  // children's incoming order
        for (int a = 0; a < 3; a++) {                 // stable split of the other sorted lists
            if (a == split_axis) continue;
            uint32_t *o = ord[a].data() + s0;
            uint32_t l = 0, r = mid;
            for (uint32_t i = 0; i < cnt; i++) tmp[left_side[o[i]] ? l++ : r++] = o[i];
            std::copy(tmp.begin(), tmp.begin() + cnt, o);
        }
        const uint32_t left = node_count++, right = node_count++;
        (void)right;
        node.count = 0;
        node.index = left;
        stack.push_back({s0 + mid, cnt - mid, left + 1});
        stack.push_back({s0, mid, left});
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
    uint32_t height = 0;           // interior nodes on the longest root-to-leaf path
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
        std::vector<std::pair<uint32_t, uint32_t>> todo{{0u, 0u}};   // (node, interior nodes above it)
        while (!todo.empty()) {
            const auto [j, d] = todo.back();
            todo.pop_back();
            const TreeNode &nd = t.nodes[j];
            if (nd.count > 0) { f.height = std::max(f.height, d); continue; }
            todo.push_back({nd.index, d + 1});
            todo.push_back({nd.index + 1, d + 1});
        }
    }
    return f;
}

// Quad form of one tree (FAST kernel, option "wide").  The quad of a binary interior node holds its two
// binary levels below it as two halves (layout.hpp NodeQuad): slots 0, 1 = the left child's children,
// slots 2, 3 = the right child's, a leaf child in its half's first slot with the second empty; leaves keep
// their refs (same leaf-ordered slots), so the quad tree holds exactly the binary tree's leaves, and the
// kernel can visit them in the binary tree's order (BLAS.cu:186-202).
struct FlatWide {
    std::vector<NodeQuad> quads;
    uint32_t root_ref = 0;
    uint32_t height = 0;           // quad levels on the longest root-to-leaf path
};

// level_order: quads numbered level by level (breadth first), so the first k quads are the tree's top
// levels (the LDS-resident part of a group's BLAS); otherwise depth first
// halves = false (host SAH trees): the greedy BVH2 -> BVH4 collapse instead — a quad starts from a binary node's two
// children and repeatedly replaces its largest-area interior child by that child's two children until it holds 4
// (fewer quads per ray; the kernel visits such quads by entry t); empty slots have every bound = +inf.
inline FlatWide flatten_tree_wide(const Tree &t, uint32_t quad_base, uint32_t slot_base, uint32_t ptype, bool blas,
                                  bool halves = true, bool level_order = false) {
    FlatWide f;
    const uint32_t n = (uint32_t)t.nodes.size();
    if (n == 0) return f;
    // subtree item counts and first slots (children have larger indices than their parent)
    std::vector<uint32_t> items(n), first(n);
    for (uint32_t j = n; j-- > 0;) {
        const TreeNode &nd = t.nodes[j];
        if (nd.count > 0) { items[j] = nd.count; first[j] = nd.index; }
        else { items[j] = items[nd.index] + items[nd.index + 1]; first[j] = first[nd.index]; }
    }
    auto is_leaf = [&](uint32_t j) { return t.nodes[j].count > 0; };
    auto leaf_ref = [&](uint32_t j) { return make_leaf_ref(slot_base + first[j], items[j], ptype, blas); };
    if (is_leaf(0)) { f.root_ref = leaf_ref(0); return f; }
    struct Todo { uint32_t node, quad, depth; };
    std::vector<Todo> todo{{0u, 0u, 1u}};
    size_t head = 0;                               // level order: todo is a FIFO from `head`
    f.quads.emplace_back();
    while (todo.size() > head) {
        Todo w;
        if (level_order) {
            w = todo[head++];
        } else {
            w = todo.back();
            todo.pop_back();
        }
        f.height = std::max(f.height, w.depth);
        NodeQuad q;
        if (!halves) {
            uint32_t ch[4] = {t.nodes[w.node].index, t.nodes[w.node].index + 1, 0, 0};
            uint32_t nc = 2;
            while (nc < 4) {
                int best = -1;
                float area = -1.0f;
                for (uint32_t k = 0; k < nc; k++)
                    if (!is_leaf(ch[k]) && half_area(t.nodes[ch[k]].box) > area) {
                        area = half_area(t.nodes[ch[k]].box);
                        best = (int)k;
                    }
                if (best < 0) break;
                const uint32_t left = t.nodes[ch[best]].index;
                ch[best] = left;
                ch[nc++] = left + 1;
            }
            for (uint32_t k = 0; k < 4; k++) {
                float b[6];
                uint32_t ref = REF_EMPTY;
                if (k < nc) {
                    t.nodes[ch[k]].box.store(b);
                    if (is_leaf(ch[k])) {
                        ref = leaf_ref(ch[k]);
                    } else {
                        const uint32_t qi = (uint32_t)f.quads.size();
                        f.quads.emplace_back();
                        ref = make_interior_ref(quad_base + qi, blas);
                        todo.push_back({ch[k], qi, w.depth + 1});
                    }
                } else {
                    for (float &x : b) x = std::numeric_limits<float>::infinity();   // rejected by every slab test
                }
                quad_set_slot(q, k, b, ref);
            }
            f.quads[w.quad] = q;
            continue;
        }
        for (uint32_t h = 0; h < 2; h++) {
            const uint32_t c = t.nodes[w.node].index + h;
            float b[6];
            if (is_leaf(c)) {                          // a leaf half: the leaf, then an empty slot with its box
                t.nodes[c].box.store(b);
                quad_set_slot(q, 2 * h, b, leaf_ref(c));
                quad_set_slot(q, 2 * h + 1, b, REF_EMPTY);
                continue;
            }
            for (uint32_t j = 0; j < 2; j++) {
                const uint32_t g = t.nodes[c].index + j;
                t.nodes[g].box.store(b);
                uint32_t ref;
                if (is_leaf(g)) {
                    ref = leaf_ref(g);
                } else {
                    const uint32_t qi = (uint32_t)f.quads.size();
                    f.quads.emplace_back();
                    ref = make_interior_ref(quad_base + qi, blas);
                    todo.push_back({g, qi, w.depth + 1});
                }
                quad_set_slot(q, 2 * h + j, b, ref);
            }
        }
        f.quads[w.quad] = q;
    }
    f.root_ref = make_interior_ref(quad_base, blas);
    return f;
}

}  // namespace rtamd
