// rt_bvh.hpp -- host-side bounding-volume hierarchy over the scene's spheres, cubes and
// loose triangles (planes are unbounded and stay in the linear pass).
//
// The hierarchy only ever *skips* work: the device walks it with boxes inflated by a
// per-ray bound on the reference's f32 error (DESIGN.md "Exact culling"), so every
// primitive the reference could report for a ray is still tested with the reference's
// own arithmetic, and the nearest hit -- including ties, broken by the shape key in
// insertion order -- is the one Scene::intersect (scene/mod.rs:98-116) returns.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace rtbvh {

enum PrimKind : int { P_DSPH = 0, P_GSPH = 1, P_TRI = 2, P_CUBE = 3 };

struct Prim {
    int kind;        // PrimKind
    uint32_t id;     // index into the caller's per-kind list
    double lo[3], hi[3];  // conservative world-space box
    double cost;     // expected per-lane test cost (VALU ops)
};

struct Node {        // binary node: both children's boxes, tested together (2-wide)
    double lo[2][3], hi[2][3];
    uint32_t child[2];   // node index, or LEAF | leaf index
    uint32_t axis;       // split axis: child 0 holds the lower centroids
};

constexpr uint32_t LEAF = 0x80000000u;
constexpr int MAX_DEPTH = 30;   // the device stack holds 32 entries

struct Tree {
    std::vector<Node> nodes;
    std::vector<std::vector<uint32_t>> leaves;  // prim indices per leaf
    uint32_t root = LEAF;                        // child pointer of the root
    double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
    int depth = 0;
};

// Binned SAH (16 bins per axis) with cost model c_node + sum(area fraction * cost), leaves of
// at most max_leaf primitives (Tune::bvh_cnode / bvh_maxleaf).
Tree build(const std::vector<Prim>& prims, double c_node, std::size_t max_leaf);

}  // namespace rtbvh
