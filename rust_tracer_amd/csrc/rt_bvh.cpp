// rt_bvh.cpp -- binned-SAH build of the culling hierarchy (see rt_bvh.hpp).
#include "rt_bvh.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <limits>

namespace rtbvh {
namespace {

constexpr int BINS = 16;
// SAH cost of one visited node and the largest leaf.  The node cost is not the child-box
// test's ~30 VALU: a visit is a dependent scalar load, ballots, a branch and an LDS stack
// operation for the whole wave, while leaf tests are straight-line packed arithmetic.
// Measured (config 3, 1080p, ms/frame): node cost 40 / leaves <= 8: 7.88; 80: 7.20;
// 120 / 16: 6.98; 200 / 16: 6.76; 200 / 32: 6.73; 300 / 32: 6.78; 500 / 64: 7.09.
// Retuned with light buffers and the own-shape shadow tests (the walk now serves mostly
// trace rays): 100 / 32: 5.07; 200 / 32: 4.76; 400 / 32: 4.65; 600 / 32: 4.68;
// 400 / 64: 4.65; 800 / 64: 4.89.
// Tune::bvh_cnode / bvh_maxleaf override them (A/B measurements).

struct Box {
    double lo[3], hi[3];
    Box() {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::numeric_limits<double>::infinity();
            hi[k] = -std::numeric_limits<double>::infinity();
        }
    }
    void grow(const double* l, const double* h) {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], l[k]);
            hi[k] = std::max(hi[k], h[k]);
        }
    }
    void grow(const Box& b) { grow(b.lo, b.hi); }
    bool empty() const { return !(lo[0] <= hi[0]); }
    double area() const {
        if (empty()) return 0.0;
        double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
        return 2.0 * (x * y + y * z + z * x);
    }
};

// leaf cost with pair packing: diag spheres and triangles are tested two at a time
struct Cost {
    double n[4] = {0, 0, 0, 0}, c[4] = {0, 0, 0, 0};
    void add(const Prim& p) {
        n[p.kind] += 1;
        c[p.kind] += p.cost;
    }
    void add(const Cost& o) {
        for (int k = 0; k < 4; k++) {
            n[k] += o.n[k];
            c[k] += o.c[k];
        }
    }
    double value() const {
        double v = c[P_GSPH] + c[P_CUBE];
        for (int k : {(int)P_DSPH, (int)P_TRI})
            if (n[k] > 0) v += c[k] * (2.0 * std::ceil(n[k] / 2.0) / n[k]);
        return v;
    }
};

struct Builder {
    const double C_NODE_V;
    const size_t MAX_LEAF_V;
    const std::vector<Prim>& P;
    Tree& T;
    std::vector<double> cen;  // 3 per prim

    Builder(const std::vector<Prim>& p, Tree& t, double c_node, size_t max_leaf)
        : C_NODE_V(c_node), MAX_LEAF_V(max_leaf), P(p), T(t), cen(3 * p.size()) {
        for (size_t i = 0; i < p.size(); i++)
            for (int k = 0; k < 3; k++) cen[3 * i + k] = 0.5 * (p[i].lo[k] + p[i].hi[k]);
    }

    Box bounds(const std::vector<uint32_t>& idx) const {
        Box b;
        for (uint32_t i : idx) b.grow(P[i].lo, P[i].hi);
        return b;
    }

    uint32_t make_leaf(std::vector<uint32_t>&& idx) {
        T.leaves.push_back(std::move(idx));
        return LEAF | (uint32_t)(T.leaves.size() - 1);
    }

    // returns the child pointer of the subtree over idx
    uint32_t rec(std::vector<uint32_t> idx, int depth, Box& box_out) {
        box_out = bounds(idx);
        T.depth = std::max(T.depth, depth);
        Cost lcost;
        for (uint32_t i : idx) lcost.add(P[i]);
        double leaf_cost = lcost.value();
        if (idx.size() <= 1) return make_leaf(std::move(idx));
        Box cb;
        for (uint32_t i : idx) cb.grow(&cen[3 * i], &cen[3 * i]);
        double best = std::numeric_limits<double>::infinity();
        int best_axis = -1, best_bin = -1;
        double parea = box_out.area();
        for (int ax = 0; ax < 3; ax++) {
            double ext = cb.hi[ax] - cb.lo[ax];
            if (!(ext > 0)) continue;
            Box bb[BINS];
            Cost bc[BINS];
            for (uint32_t i : idx) {
                int b = std::min(BINS - 1, (int)((cen[3 * i + ax] - cb.lo[ax]) / ext * BINS));
                bb[b].grow(P[i].lo, P[i].hi);
                bc[b].add(P[i]);
            }
            Box right[BINS];
            double rc[BINS];
            Box acc;
            Cost c;
            for (int b = BINS - 1; b >= 1; b--) {
                acc.grow(bb[b]);
                c.add(bc[b]);
                right[b] = acc;
                rc[b] = c.value();
            }
            Box left;
            Cost lc;
            for (int b = 0; b < BINS - 1; b++) {
                left.grow(bb[b]);
                lc.add(bc[b]);
                if (left.empty() || right[b + 1].empty()) continue;
                double cost = C_NODE_V + (left.area() * lc.value() + right[b + 1].area() * rc[b + 1]) / parea;
                if (cost < best) {
                    best = cost;
                    best_axis = ax;
                    best_bin = b;
                }
            }
        }
        if (depth >= MAX_DEPTH) return make_leaf(std::move(idx));  // depth cap: one big leaf
        bool force = idx.size() > MAX_LEAF_V;
        if (!force && !(best < leaf_cost)) return make_leaf(std::move(idx));
        std::vector<uint32_t> L, R;
        int axis = best_axis;
        if (best_axis >= 0) {
            double ext = cb.hi[axis] - cb.lo[axis];
            for (uint32_t i : idx) {
                int b = std::min(BINS - 1, (int)((cen[3 * i + axis] - cb.lo[axis]) / ext * BINS));
                (b <= best_bin ? L : R).push_back(i);
            }
        } else {  // coincident centroids or depth cap: median split on the widest axis
            axis = 0;
            for (int k = 1; k < 3; k++)
                if (box_out.hi[k] - box_out.lo[k] > box_out.hi[axis] - box_out.lo[axis]) axis = k;
            std::vector<uint32_t> s = idx;
            std::stable_sort(s.begin(), s.end(),
                             [&](uint32_t a, uint32_t b) { return cen[3 * a + axis] < cen[3 * b + axis]; });
            L.assign(s.begin(), s.begin() + s.size() / 2);
            R.assign(s.begin() + s.size() / 2, s.end());
        }
        if (L.empty() || R.empty()) return make_leaf(std::move(idx));
        uint32_t me = (uint32_t)T.nodes.size();
        T.nodes.push_back(Node{});
        Box bl, br;
        uint32_t cl = rec(std::move(L), depth + 1, bl);
        uint32_t cr = rec(std::move(R), depth + 1, br);
        Node& n = T.nodes[me];
        for (int k = 0; k < 3; k++) {
            n.lo[0][k] = bl.lo[k];
            n.hi[0][k] = bl.hi[k];
            n.lo[1][k] = br.lo[k];
            n.hi[1][k] = br.hi[k];
        }
        n.child[0] = cl;
        n.child[1] = cr;
        n.axis = (uint32_t)axis;
        return me;
    }
};

}  // namespace

Tree build(const std::vector<Prim>& prims, double c_node, size_t max_leaf) {
    Tree T;
    if (prims.empty()) return T;
    Builder b(prims, T, c_node, max_leaf);
    std::vector<uint32_t> idx(prims.size());
    for (size_t i = 0; i < idx.size(); i++) idx[i] = (uint32_t)i;
    Box root;
    T.root = b.rec(std::move(idx), 0, root);
    for (int k = 0; k < 3; k++) {
        T.lo[k] = root.lo[k];
        T.hi[k] = root.hi[k];
    }
    return T;
}

}  // namespace rtbvh
