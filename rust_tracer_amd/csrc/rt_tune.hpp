// rt_tune.hpp -- the render path's tunables, per scene handle.
//
// Every field's default is the measured optimum (DESIGN.md records each A/B).  None of them
// changes a pixel: every alternative is exact by construction (the GPU suite checks the
// ones a test needs bit for bit against the default and the oracle), they move only where
// time goes.  A handle gets its tuning at creation -- the defaults, then the environment's
// RT_TUNE="key=value,..." (the A/B harness; the library's only environment read), then the
// `tuning` string of rt_scene_create_tuned -- and rt_scene_set_tuning changes the pass-time
// keys later.  Clones (frames in flight, band shares, devices) copy their source's tuning.
//
// Result-changing measurement knobs (scaled culling bounds, no grazing pass, ...) do not
// exist in the product library; diagnostic builds add them (-DRT_DIAG=1,
// tools/build_variant.sh).
#pragma once
#include <cstdint>

struct Tune {
    // ---- scene build (fixed for the handle's life)
    int bvh = 1;              // culling hierarchy (0: every shape in the linear pass)
    double graze_k = 5e-4;    // grazing threshold sin(phi_T) = k / sin(alpha) (1e-3 until round 5; with 6-primitive
                              // leaves 3e-4 / 5e-4 / 7e-4 +0.8% / +0.6 - 0.9% / +1.0% at K = 20, 2e-3 -1.4%, profiles/r5ab/)
    int graze_res = 64;       // grazing direction cells per cube-map face side (0: cone path)
    int graze_lane = 1;       // per-lane grazing sets (0: the wave-union path)
    int lb_res = 48;          // light-buffer cells per face side (0: no light buffers)
    int lb_reach = 1;         // light-buffer runs cut at the undecided lanes' reach
    double lb_dmax_k = 3.0;   // light-buffer tier 0 serves origins with D <= lb_dmax_k R
    int lb_near_all = 1;      // light-buffer tiers past the first: records near the light in every cell (no tier limit)
    int lb_tiers = 5;         // light-buffer tiers (at most, per light): tier t serves origins with D <= 3 R 2^t
                              // (1 until round 4; K = 20: 1 / 3 / 4 / 5 tiers 1097 / 1200 / 1212 / 1212 without
                              // lb_near_all; with it 4 / 5 / 6 tiers 1245 / 1258 / 1250 vs 1240)
    int shape_buf = 1;        // shape buffers for rays inside spheres
    int bvh_tris = 1;         // loose triangles in the hierarchy (0: linear)
    int dark_skip = 1;        // shadowed lights skipped in the combine where exact
    double bvh_cnode = 400.0; // SAH node cost
    int bvh_maxleaf = 6;      // primitives per leaf at most (32 until round 4: K = 20 +0.9%, K = 64 flat; 16 in
                              // round 4; round 5, profiles/r5ab/: 6 vs 16 +1.9% at K = 20, +2.2% at K = 64;
                              // 4 / 8 / 12: -1.5% / +1.6% / +0.9% at K = 20)
    int force_rccl = 0;       // rt_scene_create_multi with one device: a one-rank communicator
    int build_threads = 0;    // host threads of the scene build (0: the CPUs the process may use, at most 32)
    // ---- per pass
    int sort_tasks = 1;       // order the trace queues spatially
    int sort_shadow = 1;      // order the shadow queue
    int task_key = 7;         // task key mode (rt_wavefront.hip task_key / inside_key)
    int self_shadow = 1;      // own-shape shadow pre-test in the trace kernel
    int inline_shadow = 1;    // levels whose shadow rays the trace kernel scans inline
    int task_w = 32;          // narrowest trace task (64 / 32 / 16 rays)
    int sched = 0;            // trace kernels' work distribution: 0 grid-stride, 1 dynamic, 2 block-contiguous
    double task_fill = 0.5;   // tasks per wave slot below which a level's tasks are narrowed
    int shadow_key = 2;       // shadow queue key: 2 cell2, 1 cell, 16 / 18 / 21 light | Morton bits
    double walk_linear = 1.0; // shadow walks: linear hierarchy scan from h(D) >= this x scene radius (0: off)
    int walk_first = 1;       // cell keys: the shadow rays that walk the hierarchy sort first (0: last)
    int task_fine = 1;        // frame batches: 21-bit task keys
    int shadow_fine = 1;      // frame batches: a 4th shadow-distance bit
    int key24 = 1;            // frame batches without frame bits: 24-bit keys
    int spp_keys = 1;         // sample batches' keys: 0 mix, 1 mixfine, 2 frame
    int frame_keys = 1;       // frame batches' keys: 0 mix, 1 mixfine, 2 frame
    int l0_interleave = 1;    // level-0 tiles dealt to a pass's frames in turn
    int spp_batch = 0;        // samples per pass (0: as many as spp_batch_items allow)
    uint64_t spp_batch_items = 1ull << 25;
    int node_factor = 6;      // node slots per level-0 item
    double shadow_factor = 2.0;  // shadow-queue slots per node slot
    uint64_t node_cap = 0;    // test knob: pin the node pool (0: sized from node_factor)
    int grid_pct = 0;         // trace grids' share of the chip (0: rt_scene_set_grid_share's)
    int grid_pct_shadow = 100;
    int grid_pct_combine = 100;
    int lds_nodes = 3;        // walk records staged in LDS: bit 0 trace kernel, bit 1 shadow kernel
    int deep_kernel = 1;      // the deep-level trace instantiation
    int occ_each = 0;         // grids per trace instantiation's own occupancy
    int count = 3;            // counting frames: bit 0 trace tests, bit 1 shadow tests
    int dup = 0;              // measurement: launch stages twice (bit 0 sorts, 1 shadow, 2 combine)
    int seam_split = 2;       // rt_render / rt_render_frame_async: band shares side by side
    int seam_band_rows = 0;   // pin the shares' meeting row (0: adapted)
    int seam_adapt = 1;       // meeting row: 1 copy-aware, 2 device finish times, 0 even split
    int seam_grid_pct = 80;   // the shares' grids' share of the chip
    int frame_fork = 0;       // rt_render_frame_async: 1 = share 0 on the caller's stream
};

// Applies "key=value" pairs (separated by ',' or whitespace) to t.  build_keys: whether
// scene-build keys are accepted.  Returns false (t partly updated) on an unknown key, a bad
// value, or a scene-build key when !build_keys.
bool tune_apply(Tune& t, const char* spec, bool build_keys);
