// rt_device.hpp -- device-side scene layout shared by the host builder (rt_api.cpp) and
// the HIP kernels (rt_kernels.hip).
//
// The scene lives in ONE device allocation, cut into per-type runs so the hot
// nearest-hit scan walks each run with wave-uniform indices (the loads become scalar
// SMEM loads: every lane tests the same primitive against its own ray).
//
//   run      record (float4s)                              bytes   used by
//   dsph     {s0 s1 s2 key} {o0 o1 o2 -}                   32      scan: spheres whose inverse has a
//                                                                  zero 3x3 off-diagonal (translate*scale)
//   gsph     {inv row0} {inv row1} {inv row2} {key - - -}  64      scan: all other spheres
//   tri      {v0 key} {e1 -} {e2 -}                        48      scan: loose triangles (world space)
//   cube     {inv row0} {inv row1} {inv row2} {key - - -}  64      scan: cube instances (12 object tris)
//   plane    {inv r0} {inv r1} {inv r2} {n key} {origin -} 80      scan: planes
//   cubetri  12 x {v0 -} {e1 -} {e2 -} {n -}               768     unit-cube triangles (cube.rs:21-77)
//   shapes   ShapeRec per shape, insertion order            128     attributes of the nearest hit
//   mats     MatRec                                         80      shading
//   lights   LightRec                                       32      shading
//
// `key` = (shape index << 4) | cube triangle index, stored as the float's bits; the
// nearest-hit tie-break compares (t, key) lexicographically, which reproduces
// Scene::intersect's strict `<` over insertion order (scene/mod.rs:98-116) and the
// cube's inner scene order (cube.rs:58-69).
#pragma once
#include <stdint.h>

namespace rtdev {

struct ShapeRec {
    int32_t kind, mat, pad0, pad1;
    float inv[12];   // rows 0..2 of the inverse transform (row 3 is never read)
    float a[16];     // plane: n(3) origin(3) Tn(3) u(3) v(3); triangle: v0 e1 e2 normal
};

struct TexRec {
    int32_t kind;
    float r, g, b;
};

struct MatRec {
    int32_t kind, pad;
    float power, reflectivity;
    float refraction_index, pad1, pad2, pad3;
    TexRec ambient, diffuse, specular;
};

struct LightRec {
    int32_t kind;
    float px, py, pz;
    float r, g, b, pad;
};

// Kernel-argument view of an uploaded scene (pointers into the one allocation).
struct DevScene {
    const float4* dsph;
    const float4* gsph;
    const float4* tri;
    const float4* cube;
    const float4* plane;
    const float4* cubetri;
    const ShapeRec* shapes;
    const MatRec* mats;
    const LightRec* lights;
    int32_t n_dsph, n_gsph, n_tri, n_cube, n_plane, n_shapes, n_lights, n_mats;
    float amb_r, amb_g, amb_b;
};

// Everything one launch needs.
struct RenderParams {
    DevScene S;
    float cam_ox, cam_oy, cam_oz;
    float x_min, y_max, x_delta, y_delta;   // render.rs:178-185, deltas computed on the host
    uint32_t width, height;                 // full frame
    uint32_t depth;
    uint32_t band_rows, rank, world, rows_local;  // this launch's rows: see rt_render_bands_async
    uint32_t tiles_x, total_items;          // 8x8 pixel tiles over (width x rows_local)
    float* out;                             // rows_local * width * 3 floats
    unsigned long long* ray_counters;       // [node, shadow, pixels], added to
    uint32_t* work_counter;                 // zeroed before the launch
};

}  // namespace rtdev
