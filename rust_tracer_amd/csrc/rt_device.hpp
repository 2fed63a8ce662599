// rt_device.hpp -- device-side scene layout shared by the host builder (rt_build.cpp) and
// the HIP kernels (rt_wavefront.hip, rt_order.hip, rt_frame.hip).
//
// The scene lives in ONE device allocation, cut into per-type runs so the hot
// nearest-hit scan walks each run with wave-uniform indices (the loads become scalar
// SMEM loads: every lane tests the same primitive against its own ray).
//
//   run      record (float4s)                              bytes   used by
//   dsph     PAIRS of spheres whose inverse has a zero 3x3   64      scan (2-wide packed)
//            off-diagonal: {sxA sxB syA syB} {szA szB oxA oxB} {oyA oyB ozA ozB} {keyA keyB - -}
//   gsph     {inv row0} {inv row1} {inv row2} {key - - -}  64      scan: other spheres (+ odd tail)
//   tri      PAIRS of loose triangles (world space):        96      scan (2-wide packed)
//            {v0xA v0xB v0yA v0yB} {v0zA v0zB e1xA e1xB} {e1yA e1yB e1zA e1zB}
//            {e2xA e2xB e2yA e2yB} {e2zA e2zB keyA keyB} {- - - -}   (odd tail: degenerate pad)
//   cube     {inv row0} {inv row1} {inv row2} {key - - -}  64      scan: cube instances (12 object tris,
//                                                                  compile-time, rt_scan.hpp)
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
    int32_t kind, mat;
    uint32_t center_key;  // sphere / cube: 15-bit Morton code of its centre (rt_wavefront.hip task_key)
    int32_t pad1;         // sphere: its shape buffer's leaf + 1 (0: none; rt_build.cpp build_shape_buffers)
    float inv[12];   // rows 0..2 of the inverse transform (row 3 is never read)
    float a[16];     // plane: n(3) origin(3) Tn(3) u(3) v(3); triangle: v0 e1 e2 normal;
                     // sphere with a shape buffer: its bounding ball's centre (3) and radius
};

struct TexRec {
    int32_t kind;
    float r, g, b;
};

struct MatRec {
    int32_t kind;
    int32_t dark_zero;   // 1: an unlit point light's term is exactly +-0 for this material (rt_build.cpp mat_rec)
    float power, reflectivity;
    float refraction_index, pad1, pad2, pad3;
    TexRec ambient, diffuse, specular;
};

struct LightRec {
    int32_t kind;
    float px, py, pz;
    float r, g, b;
    uint32_t lb_base;  // light buffer: first cell (a bvh_leaves index) in bits 0-27, tier count in bits 28-30; ~0: none
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
    int32_t n_dsph, n_gsph, n_tri, n_cube, n_plane, n_shapes, n_lights, n_mats;  // dsph/tri: pairs
    float amb_r, amb_g, amb_b;
    // ---- culling hierarchy (rt_bvh.hpp; DESIGN.md "Exact culling").  The first
    // n_*_bvh records of each run are the hierarchy's primitives in leaf order; the rest
    // (ill-conditioned shapes, or everything when the hierarchy is off) are scanned
    // linearly for every ray.
    const float4* bvh_nodes;   // 4 float4 per node: both child boxes + child pointers
    const uint4* bvh_leaves;   // 2 uint4 per leaf: [dsph b,e gsph b,e] [tri b,e cube b,e]
    const float4* graze_blk;   // grazing pass: 8 float4 per block of 8 triangles (cone + normals)
    const float4* graze_tri;   // ... and the block's triangles as 4 pairs
    int32_t n_graze_blk;
    uint32_t bvh_root;         // child pointer (BVH_LEAF bit: a leaf)
    int32_t n_bvh_nodes;
    int32_t use_bvh;
    int32_t n_dsph_bvh, n_gsph_bvh, n_tri_bvh, n_cube_bvh;
    // per ray, D = |o - c| + r: box inflation h(D) = (g2 D + g1) D + g0 and t-margin
    // m(D) = m1 D + m0 (distance units), see rt_scan.hpp
    float bvh_cx, bvh_cy, bvh_cz, bvh_r, bvh_g2, bvh_g1, bvh_g0, bvh_m1, bvh_m0;
    float walk_lin_h;          // shadow walks: a wave whose nearest walking origin has h(D) >= this
                               // tests every hierarchy primitive in order (rt_scan.hpp hier_linear)
    float graze_s2;            // 1.0201: (d.n')^2 < graze_s2 |d|^2 with n' = n / sin(phi_T): the ray grazes
    const float4* graze_pn;    // per graze pair: {nAx nBx nAy nBy} {nAz nBz - -} (n / sin(phi_T))
    const uint32_t* graze_mask;  // per direction cell: graze_words words of pair bits
    uint32_t graze_res, graze_words;  // 0: the cone path (rt_scan.hpp graze_pass)
    uint32_t graze_lane;       // 1: each lane tests its own cell's pairs first (per-lane grazing sets)
    unsigned long long* scan_ops;  // RT_OPS_* lane-weighted test counts
    // light buffers (shadow rays; rt_build.cpp build_light_buffers): per point light
    // 6 x lb_res x lb_res cells, each a leaf of bvh_leaves (LightRec::lb_base + cell)
    uint32_t lb_res;           // 0: no light buffers
    float lb_dmax;             // tier t of a light's buffer holds origins with D <= lb_dmax 2^t
    uint32_t lb_tiers;         // the most tiers of any light (each light's own count: LightRec::lb_base bits 28-30)
    int32_t dark_skip;         // 1: every hit normal is finite with |n| <= 1e3 (shadowed-light skip, light_sum)
};
#define RT_LB_LMAX 45.f        // ... and so do origins farther than this from the light

#define BVH_LEAF 0x80000000u
// lane-weighted counters of the scan's tests (each += active lanes)
enum : int {
    RT_OPS_NODE = 0,    // 2-wide child-box tests
    RT_OPS_DSPH = 1,    // diag sphere pairs
    RT_OPS_GSPH = 2,    // general spheres
    RT_OPS_TRI = 3,     // loose triangle pairs
    RT_OPS_CUBE_BOX = 4,  // object-space cube box tests
    RT_OPS_CUBE = 5,    // full cubes (12 triangles)
    RT_OPS_GRAZE = 6,   // grazing cone tests (blocks of 8 triangles)
    RT_OPS_PLANE = 7,   // planes
    RT_OPS_GRAZE_N = 8, // grazing normal tests (blocks of 8 whose cone some lane meets)
    // instrumented kernels only: shader-clock cycles (s_memtime) per wave spent in
    RT_OPS_CYC_NODE = 9,   // ... child-box tests and their stack / branch bookkeeping
    RT_OPS_CYC_LEAF = 10,  // ... leaf primitive tests
    RT_OPS_CYC_GRAZE = 11, // ... the grazing pass
    RT_OPS_CYC_SCAN = 12,  // ... whole scans (planes, walk, grazing pass, linear rest)
    RT_OPS_CYC_LOAD = 13,  // trace kernel: fetching / generating the ray (task gather)
    RT_OPS_CYC_POST = 14,  // trace kernel: after the scan (attributes, node record, children,
                           // shadow entries), the own-shape shadow tests excluded
    RT_OPS_CYC_SELF = 15,  // trace kernel: the own-shape shadow tests
    RT_OPS_N = 16,
    // scan_ops is RT_OPS_SLOTS x RT_OPS_STRIDE u64: block b adds to slot b % RT_OPS_SLOTS
    // (same-address global atomics from every block would serialise in L2)
    RT_OPS_SLOTS = 64,
    RT_OPS_STRIDE = 16
};

// The level table: (offset, count) per level, the shadow-queue count, then one work
// counter per level and one for the shadow pass: waves take their next 64 tasks from it
// (dynamic scheduling: a launch ends when the work does, not when its slowest static
// share does).
#define RT_LEVEL_WORDS (2 * (RT_MAX_DEPTH + 2))
#define RT_WORK_WORD(k) (RT_LEVEL_WORDS + (k))  // k: level, or RT_MAX_DEPTH + 1: shadow pass
#define RT_LEVEL_TABLE_WORDS (RT_LEVEL_WORDS + RT_MAX_DEPTH + 2)


// ---- level-synchronous ("wavefront") pipeline, rt_wavefront.hip ----------------------
// A ray task of tree level k >= 1 (level-0 tasks are the pixels themselves).
struct Task {
    float ox, oy, oz, dx, dy, dz;
    uint32_t parent;   // (node index << 1) | slot  (slot 0 = reflected, 1 = refracted)
    uint32_t pixel;    // y * width + x of the tree's pixel (ray forest)
};

// One traced tree node, in structure-of-arrays form (index n = the node's slot in its
// level's queue, so a wave's accesses to one array are one contiguous 1 KB run):
//   node_flags[n]  NODE_HIT / NODE_MISS / NODE_NONE | F_HAS_R / F_HAS_T (a reflected /
//                  refracted child was queued) | F_ENTER | material index << F_MAT_SHIFT
//   node_ps[n]     {shadow-ray origin p + 0.0002 n (render.rs:147), texture u}
//   node_n[n]      {hit normal, texture v}
//   node_d[n]      {the ray's direction, parent = (parent node << 1) | slot}
//   node_lit[n]    bit l: point light l is NOT shadowed (lights 32 and up: node_lit_hi)
//   node_ec[2n+s]  colour the node's child in slot s (0 reflected, 1 refracted) reports
// That is 52 B written per hit node.  Everything else render.rs:57-100 needs (eye_dir,
// n1 / n2, the material's textures at (u, v), the reflected direction, Schlick weights,
// (m.h)^power, the refracted direction) is a pure function of these and the material,
// and the combine pass re-evaluates it with the trace kernel's own expressions
// (rt_common.hpp node_weights), bit for bit.  The shadow pass reads node_ps at random
// (16 B per entry).  Ray forest (render_tree.rs): node_dc[2n+s] holds the direction the
// child reports (render_tree.rs:252), node_key / node_pixel the shape id and pixel.
enum : uint32_t {
    NODE_HIT = 1u << 8, NODE_MISS = 1u << 9, NODE_NONE = 1u << 10,
    F_HAS_R = 1u << 11, F_HAS_T = 1u << 12, F_ENTER = 1u << 13,
    F_MAT_SHIFT = 14u   // material index: up to 2^18 materials
};
#define RT_MAX_MATERIALS (1u << 18)

// frame batches (rt_render_bands_batch_async): up to RT_MAX_FRAMES frames of one
// resolution in one pipeline pass; a task carries its frame in Task.pixel's top bits
#ifndef RT_MAX_FRAMES
#define RT_MAX_FRAMES 32  // 5 frame bits: Task.pixel bits 27-31 (frames of < 2^27 pixels)
#endif
#if RT_MAX_FRAMES > 32
#error "RT_MAX_FRAMES: at most 32 (5 frame bits in Task.pixel)"
#elif RT_MAX_FRAMES > 16
#define RT_FRAME_SHIFT 27
#else
#define RT_FRAME_SHIFT 28  // -DRT_MAX_FRAMES=16: 4 frame bits, bits 28-31
#endif
struct FrameCam {
    float ox, oy, oz, x_min, y_max, x_delta, y_delta, pad;
};
struct WaveParams {
    DevScene S;
    uint32_t frames;                   // frames in this pass (1: rt_render_bands_async)
    uint32_t frame_items;              // level-0 items per frame (total_items / frames)
    uint32_t task_frame_shift;         // task key |= frame << this (frames > 1)
    uint32_t task_fine;                // key mode 7 with 5 more origin bits (a batch's 3 radix passes have room)
    uint32_t shadow_frame_shift;       // shadow key |= frame << this (frames > 1)
    size_t frame_floats;               // output floats per frame (rows_local x width x 3; direct: height x width x 3)
    uint32_t direct;                   // out / out8 are whole frames: pixel (u, v) at v x width + u, padding never written
    FrameCam cams[RT_MAX_FRAMES];      // frames > 1: each frame's camera (render.rs:155-186)
    uint32_t width, height, depth;
    uint32_t band_rows, rank, world, rows_local;
    uint32_t tiles_x, total_items;     // level-0 tasks (8x8 tiles over width x rows_local)
    uint32_t capacity;                 // node / task slots
    uint32_t shadow_capacity;          // shadow-queue slots
    Task* tasks;                       // [capacity]
    uint32_t* node_flags;              // [capacity] (node layout above)
    float4* node_ps;                   // [capacity]
    float4* node_n;                    // [capacity]
    float4* node_d;                    // [capacity]
    uint32_t* node_lit;                // [capacity]: unshadowed-light bits of lights 0-31
    uint32_t* node_lit_hi;             // [(lit_words - 1) x capacity]: lights 32 and up, word w of
                                       // node n at (lit_words - 1) n + w - 1 (bit l % 32: light l)
    uint32_t lit_words;                // ceil(lights / 32), at least 1
    float4* node_ec;                   // [2 x capacity]: children's colours
    uint32_t* shadow;                  // [shadow_capacity]: (node << light_bits) | light; wide: the node
    uint32_t light_bits;               // bits of the light index in a shadow entry (wide: 0)
    // scenes of more than 256 lights ("wide" entries, 8 B): the light index of slot s in
    // shadow_light[s]; the shadow kernel then reads SLOTS through shadow_in (the sort's values
    // are the slots; unsorted: shadow_in is null and entry t is slot t)
    uint32_t* shadow_light;            // [shadow_capacity] or null (packed entries)
    uint32_t* levels;                  // [RT_LEVEL_TABLE_WORDS]: offset, count per level;
                                       // levels[2 * (RT_MAX_DEPTH + 1)] = shadow-queue count;
                                       // then the work counters (RT_WORK_WORD)
    uint32_t* overflow;                // set when an append would exceed a capacity (this pass)
    uint32_t* overflow_sticky;         // ORed with `overflow` at the end of every pass (rt_scene_sync_status)
    float* out;
    uint8_t* out8;                     // optional: Color::as_u8 of `out`, written by the level-0 combine
    unsigned long long* ray_counters;  // [node, shadow, pixels], added to
    // ray-queue ordering (rt_order.hip): the producer writes a 16-bit key per task /
    // shadow entry; the sort writes the order; the consumer reads through `perm` (tasks)
    // or `shadow_in` (shadow entries).  Null keys: no ordering.
    uint32_t* task_keys;               // [capacity]
    const uint32_t* perm;              // [capacity] or null: level-k slot -> task slot
    uint32_t* shadow_keys;             // [shadow_capacity]
    const uint32_t* shadow_in;         // the shadow entries the shadow kernel reads
    uint32_t key_mode;                 // task key variant (A/B)
    float key_ahead;                   // modes 5 / 6: the key's point lies key_ahead x (scene radius) ahead
    uint32_t shadow_fine;              // 18 / 19 / 21: bits below the light index (3 sort passes); 0: 16-bit key
    uint32_t shadow_cell;              // light | light-buffer cell (1), x 3-bit (2) / 4-bit (3, shadow_fine 19)
                                       // distance from the light; rays that walk: light | flag | Morton
    // cell keys: key = light << shadow_li_shift | low, low = shadow_walk_flag | Morton for rays that
    // walk, shadow_lb_flag | cell... for the others (Tune::walk_first: the flag above the light
    // bits on the buffered rays -- walking rays first; else on the walking rays, below the light)
    uint32_t shadow_li_shift, shadow_walk_flag, shadow_lb_flag;
    uint32_t light_shift;              // shadow key = (light << light_shift) | (Morton >> (15 - light_shift))
    uint32_t count_mask;               // bit 0: trace kernels add to scan_ops, bit 1: shadow kernel
    // ray forest (render_tree.rs; set only when building an rt_forest): per node
    float4* node_dc;                   // [2 x capacity]: directions the children report
    uint32_t* node_key;                // shape id as the reference records it (cube: inner triangle)
    uint32_t* node_pixel;              // y * width + x of the tree's pixel
    const uint8_t* dirty;              // forest shade: per-pixel mask (null: every pixel)
    // supersampling (rt_render_spp): this pipeline run traces sample `sample` of `spp`;
    // level 0 jitters the primary ray (spp > 1) and the level-0 combine accumulates
    uint32_t spp, sample, seed;
    // sample batches (rt_render.cpp launch_bands_wave): this pass's `frames` are samples
    // sample + f of one camera; the level-0 combine writes each sample's raw colour to its
    // own buffer (out + f x frame_floats) and spp_accumulate_kernel sums them in sample order
    uint32_t spp_batch;
    uint32_t frame_keys;               // frames > 1: the frame index sits above the queue keys' bits
    uint32_t l0_interleave;            // frames > 1: level-0 tiles dealt to the frames in turn (default; RT_L0_INTERLEAVE=0 off)
    uint32_t self_shadow;              // trace decides shadow rays its own shape settles (A/B: RT_SELF_SHADOW=0)
    uint32_t inline_levels;            // trace levels < this trace their own shadow rays (RT_INLINE_SHADOW)
    uint32_t sched;                    // trace kernels' work distribution (Tune::sched, rt_wavefront.hip sched_base)
    uint32_t task_w_min;               // narrowest trace task (rays per wave iteration; 64 = never narrowed)
    float task_w_fill;                 // trace tasks are narrowed while a level has fewer than fill x wave slots of them
    // host-side launch choices (Tune, rt_wavefront.hip's launchers): walk records staged in LDS
    // (bit 0 trace kernels, bit 1 shadow kernel), the deep-level trace instantiation, grids
    // per instantiation's own occupancy
    uint32_t lds_mask, deep_kernel, occ_each;
};

// 15-bit Morton code of a point in the 32^3 grid over [c - r, c + r]^3 (clamped)
#define RT_MORTON_BITS 15

}  // namespace rtdev
