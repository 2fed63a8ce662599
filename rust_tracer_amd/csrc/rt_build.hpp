// rt_build.hpp -- the host half of rt_scene_create (rt_build.cpp): the reference's scene-build
// arithmetic, the culling hierarchy, grazing masks, light and shape buffers, and the section
// table of the one device allocation.  No HIP call: rt_scene_layout_digest runs it alone.
// Internal to the library (not part of the C ABI).
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_device.hpp"
#include "rt_tune.hpp"

namespace rthost {

struct HostScene;  // rt_build.cpp
struct HostSceneDeleter {
    void operator()(HostScene* h) const;
};
using HostScenePtr = std::unique_ptr<HostScene, HostSceneDeleter>;

// Builds every array of the device scene from the description (scene build of the
// reference's constructors and set_transform: matrix.rs:99-153, plane.rs:22-42,
// triangle.rs:16-39, cube.rs:21-77) plus the acceleration data.
rt_status host_scene_build(const rt_scene_desc* d, const Tune& tn, HostScenePtr& out);
// Bytes of the device allocation.
size_t host_scene_bytes(const HostScene& H);
// The host pieces of the allocation: (offset, source, bytes); the padding between them is zero.
struct UploadPiece {
    size_t off;
    const void* src;
    size_t bytes;
};
void host_scene_pieces(const HostScene& H, std::vector<UploadPiece>& out);
// What the handle keeps besides the device scene.
struct SceneFacts {
    uint64_t flops_per_scan;  // SURVEY.md §8(d) F_alg of one linear scan (bench roofline)
    uint32_t n_point_lights;
    double normal_max;        // largest hit-normal length (dark_zero of an edited material)
};
// The DevScene of an allocation at `dmem` holding host_scene_pieces().
void host_scene_bind(const HostScene& H, const void* dmem, const rt_scene_desc* d, const Tune& tn, rtdev::DevScene& S,
                     SceneFacts& facts);
// A material's device record (rt_scene_set_material): RT_ERR_INVALID_ARG for a bad one.
rt_status material_record(const rt_material& m, rtdev::MatRec& M, double normal_max);

}  // namespace rthost
