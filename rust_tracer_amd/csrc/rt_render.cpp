// rt_render.cpp -- the render driver behind the C ABI: render() (render.rs:31-38) and its
// stream-ordered band renders run the level-synchronous pipeline of rt_wavefront.hip (trace /
// shadow / combine) with the queue sorts of rt_order.hip, in the handle's workspace; rt_render
// splits one frame into two band shares side by side; overflowing queues grow the pool (never
// a truncated frame).  There is no CPU fallback anywhere in this library.
#include "rt_scene.hpp"

using namespace rtdev;
using namespace rthost;

namespace rthost {

rt_status ensure_ws(rt_scene* s, size_t out_floats, size_t out8_bytes) {
    Workspace& w = s->ws;
    if (!w.counters) {
        HIP_TRY(hipMalloc(&w.counters, 4 * sizeof(unsigned long long)));
        HIP_TRY(hipMalloc(&w.work, 64));
        HIP_TRY(hipMalloc(&w.ctr_save, 64));
    }
    if (out_floats > w.out_floats) {
        if (w.out) (void)hipFree(w.out);
        w.out = nullptr;
        w.out_floats = 0;
        HIP_TRY(hipMalloc(&w.out, out_floats * sizeof(float)));
        w.out_floats = out_floats;
    }
    if (out8_bytes > w.out8_bytes) {
        if (w.out8) (void)hipFree(w.out8);
        w.out8 = nullptr;
        w.out8_bytes = 0;
        HIP_TRY(hipMalloc(&w.out8, out8_bytes));
        w.out8_bytes = out8_bytes;
    }
    return RT_OK;
}

// (Re)allocates every per-node array with `cap` slots: tasks, the node arrays
// (rt_device.hpp).  The per-node sort buffers follow lazily (sort_capacity < capacity),
// the shadow queue from capacity * point lights.
rt_status grow_node_pool(Workspace& w, uint32_t cap) {
    for (void** b : {(void**)&w.tasks, (void**)&w.node_flags, (void**)&w.node_ps, (void**)&w.node_n,
                     (void**)&w.node_d, (void**)&w.node_lit, (void**)&w.node_lit_hi, (void**)&w.node_ec, (void**)&w.node_dc,
                     (void**)&w.node_key, (void**)&w.node_pixel}) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
    w.capacity = 0;
    HIP_TRY(hipMalloc(&w.tasks, (size_t)cap * sizeof(Task)));
    HIP_TRY(hipMalloc(&w.node_flags, (size_t)cap * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&w.node_ps, (size_t)cap * sizeof(float4)));
    HIP_TRY(hipMalloc(&w.node_n, (size_t)cap * sizeof(float4)));
    HIP_TRY(hipMalloc(&w.node_d, (size_t)cap * sizeof(float4)));
    HIP_TRY(hipMalloc(&w.node_lit, (size_t)cap * sizeof(uint32_t)));
    if (w.lit_words > 1) HIP_TRY(hipMalloc(&w.node_lit_hi, (size_t)(w.lit_words - 1) * cap * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&w.node_ec, 2 * (size_t)cap * sizeof(float4)));
    if (w.forest) {
        HIP_TRY(hipMalloc(&w.node_dc, 2 * (size_t)cap * sizeof(float4)));
        HIP_TRY(hipMalloc(&w.node_key, (size_t)cap * sizeof(uint32_t)));
        HIP_TRY(hipMalloc(&w.node_pixel, (size_t)cap * sizeof(uint32_t)));
    }
    w.capacity = cap;
    return RT_OK;
}

// Frees every device / pinned buffer of a workspace.
void free_workspace(Workspace& w) {
    for (void* b : {(void*)w.out, (void*)w.out8, (void*)w.counters, (void*)w.work, (void*)w.tasks, (void*)w.shadow,
                    (void*)w.shadow_light,
                    (void*)w.node_flags, (void*)w.levels, (void*)w.overflow, (void*)w.node_ps, (void*)w.node_n,
                    (void*)w.node_d, (void*)w.node_lit, (void*)w.node_lit_hi, (void*)w.node_ec, (void*)w.task_keys, (void*)w.perm,
                    (void*)w.shadow_keys, (void*)w.shadow_sorted, (void*)w.sort_tmp, (void*)w.node_dc,
                    (void*)w.node_key, (void*)w.node_pixel, (void*)w.spp_buf, (void*)w.ctr_save})
        if (b) (void)hipFree(b);
    w = Workspace();
}

}  // namespace rthost

// (the rt_render_bands_* entry points below keep the C linkage of their rt_api.h declarations)
static rt_status launch_bands_wave(rt_scene* s, const rt_camera* cam, uint32_t depth, uint32_t spp, uint32_t seed,
                                   uint32_t band_rows, uint32_t rank, uint32_t world, const PassOut& o,
                                   hipStream_t stream);

static rt_status launch_bands(rt_scene* s, const rt_camera* cam, uint32_t depth, uint32_t spp, uint32_t seed,
                              uint32_t band_rows, uint32_t rank, uint32_t world, const PassOut& o,
                              hipStream_t stream) {
    if (!s || !cam || (!o.rgb && !o.rgb8) || band_rows == 0 || world == 0 || rank >= world) return RT_ERR_INVALID_ARG;
    if (spp == 0) return RT_ERR_INVALID_ARG;
    if (cam->x_res == 0 || cam->y_res == 0) return RT_ERR_INVALID_ARG;
    if (depth > RT_MAX_DEPTH) return RT_ERR_UNSUPPORTED;
    if ((uint64_t)cam->x_res * cam->y_res * 3 >= (1ull << 32)) return RT_ERR_UNSUPPORTED;
    rt_status st = ensure_ws(s, 0, 0);
    if (st != RT_OK) return st;
    return launch_bands_wave(s, cam, depth, spp, seed, band_rows, rank, world, o, stream);
}

// Level-synchronous pipeline: trace(0..L-1), then combine(L-1..0), all on `stream`.
// The level-synchronous pipeline into workspace `w`.  Forest builds (w.forest) write the
// per-node shade inputs, always read the level sizes on the host, skip the combine pass
// and leave the parameters (with the device level table) in *forest_params.
// (wave_pipeline: declared in rt_scene.hpp)

// Samples per pipeline pass for spp > 1: Tune::spp_batch, else as many (<= RT_MAX_FRAMES) as
// keep a pass within Tune::spp_batch_items level-0 items (default 2^25: 4 x 3840x2160 or
// 8 x 1920x1080; the pass's workspace grows with its items).
static uint32_t spp_batch_size(const Tune& tn, uint32_t spp, uint64_t frame_items) {
    if (tn.spp_batch > 0) return (uint32_t)std::max(1, std::min(tn.spp_batch, (int)RT_MAX_FRAMES));
    const uint64_t cap = tn.spp_batch_items;
    uint32_t b = 1;
    while (b < RT_MAX_FRAMES && b < spp && (uint64_t)(b + 1) * frame_items <= cap) b++;
    return b;
}

// spp samples in sample order.  Batched (the default): B samples per pipeline pass, each a
// "frame" of the pass with the same camera and its own jitter (sample index = base + frame),
// its raw colour written to its own buffer; spp_accumulate_kernel then folds the batch into
// the running sum in sample order and the last batch divides -- the same f32 operations as
// one pass per sample, where the level-0 combine adds sample k's colour to the running sum
// of samples 0..k-1 and the last one divides (RT_SPP_BATCH=1).
static rt_status launch_bands_wave(rt_scene* s, const rt_camera* cam, uint32_t depth, uint32_t spp, uint32_t seed,
                                   uint32_t band_rows, uint32_t rank, uint32_t world, const PassOut& o,
                                   hipStream_t stream) {
    const uint32_t rows_local = rt_band_rows_per_rank(cam->y_res, band_rows, world);
    const uint64_t frame_items = (uint64_t)((cam->x_res + 7) / 8) * ((rows_local + 7) / 8) * 64u;
    const uint32_t sb = spp > 1 && o.rgb && (uint64_t)cam->x_res * cam->y_res < (1ull << RT_FRAME_SHIFT)
                            ? spp_batch_size(s->tune, spp, frame_items) : 1u;
    if (sb > 1) {
        Workspace& w = s->ws;
        const size_t frame_floats = (size_t)rows_local * cam->x_res * 3u;
        if (w.spp_buf_floats < sb * frame_floats) {
            if (w.spp_buf) (void)hipFree(w.spp_buf);
            w.spp_buf = nullptr;
            w.spp_buf_floats = 0;
            HIP_TRY(hipMalloc(&w.spp_buf, sb * frame_floats * sizeof(float)));
            w.spp_buf_floats = sb * frame_floats;
        }
        rt_camera cams[RT_MAX_FRAMES];
        for (uint32_t f = 0; f < sb; f++) cams[f] = *cam;
        const PassOut ob{w.spp_buf, nullptr, o.counters, o.latch, o.may_sync};
        for (uint32_t k = 0; k < spp; k += sb) {
            const uint32_t b = std::min(sb, spp - k);
            rt_status st = wave_pipeline(s, w, cam, depth, band_rows, rank, world, ob, stream, nullptr, nullptr, spp, k,
                                         seed, b, cams, true);
            if (st != RT_OK) return st;
            HIP_TRY(launch_spp_accumulate(w.spp_buf, b, frame_floats, k, spp, o.rgb, o.rgb8, stream));
        }
        return RT_OK;
    }
    for (uint32_t k = 0; k < spp; k++) {
        rt_status st = wave_pipeline(s, s->ws, cam, depth, band_rows, rank, world, o, stream, nullptr, nullptr, spp, k,
                                     seed);
        if (st != RT_OK) return st;
    }
    return RT_OK;
}

rt_status rthost::wave_pipeline(rt_scene* s, Workspace& w, const rt_camera* cam, uint32_t depth, uint32_t band_rows,
                               uint32_t rank, uint32_t world, const PassOut& o, hipStream_t stream,
                               WaveParams* forest_params, uint32_t* forest_levels, uint32_t spp, uint32_t sample,
                               uint32_t seed, uint32_t frames, const rt_camera* cams, bool spp_batch,
                               hipEvent_t forest_done) {
    if (frames == 0 || frames > RT_MAX_FRAMES || (frames > 1 && (!cams || forest_params))) return RT_ERR_INVALID_ARG;
    WaveParams p;
    std::memset(&p, 0, sizeof(p));
    p.spp = spp;
    p.spp_batch = spp_batch ? 1u : 0u;
    // queue keys of a sample batch: "mix" -- no sample index in the keys, the samples of one
    // place share waves; "mixfine" (default) -- the same with a frame batch's finer 21-bit
    // task / 4-bit-distance shadow keys; "frame" -- the sample index above the key bits like
    // a frame batch (Tune::spp_keys, A/B)
    // (frame batches: Tune::frame_keys, default "mixfine" as well)
    // measured (config 5, 4 passes of 4K x 64 samples in batches of 4): mix 1021, mixfine
    // 1058, frame 1023 Msamples/s; one pass per sample 788.  Frame batches (config 3, 4 passes
    // of 5 frames): frame 944 / 945, mix 1023 / 1018, mixfine 1073 / 1076 Mpixels/s with one
    // camera for every frame; with a camera per frame (an animation) frame 948, mixfine 1025
    const Tune& tn = s->tune;
    const int spp_keys = spp_batch ? tn.spp_keys : tn.frame_keys;
    p.frame_keys = spp_keys == 2 ? 1u : 0u;
    {
        // level-0 tiles dealt to a pass's frames in turn (default since the 16-frame passes:
        // 1124 - 1133 vs 1116 - 1122 Mpixels/s in 7 alternating pairs, tools/r3_ab23.sh /
        // r3_ab24.sh; at 5-frame passes it was noise); l0_interleave=0: frame-major (A/B)
        p.l0_interleave = tn.l0_interleave ? 1u : 0u;
    }
    p.sample = sample;
    p.seed = seed;
    p.S = s->S;
    // shadow waves whose walk cannot cull (its box growth h(D) at least walk_linear scene radii:
    // origins on the far floor) scan the hierarchy's primitives linearly (exact either way)
    p.S.walk_lin_h = tn.walk_linear > 0.0 ? (float)tn.walk_linear * s->S.bvh_r : __builtin_huge_valf();
    p.width = cam->x_res;
    p.height = cam->y_res;
    p.depth = depth;
    p.band_rows = band_rows;
    p.rank = rank;
    p.world = world;
    p.rows_local = rt_band_rows_per_rank(cam->y_res, band_rows, world);
    p.tiles_x = (cam->x_res + 7) / 8;
    uint64_t total = (uint64_t)p.tiles_x * ((p.rows_local + 7) / 8) * 64u;
    p.frames = frames;
    p.frame_items = (uint32_t)total;
    p.frame_floats = (size_t)p.rows_local * p.width * 3u;
    if (o.direct) {
        if (spp_batch || forest_params) return RT_ERR_INVALID_ARG;
        p.direct = 1u;
        p.frame_floats = (size_t)p.height * p.width * 3u;
    }
    if (frames > 1 && (uint64_t)cam->x_res * cam->y_res >= (1ull << RT_FRAME_SHIFT)) return RT_ERR_UNSUPPORTED;
    {
        // level 0 reads every frame's camera from cams[] (frames == 1: cams[0] = cam)
        if (frames == 1) cams = cam;
        for (uint32_t f = 0; f < frames; f++) {
            if (cams[f].x_res != cam->x_res || cams[f].y_res != cam->y_res) return RT_ERR_INVALID_ARG;
            FrameCam& c = p.cams[f];
            c.ox = cams[f].origin[0];
            c.oy = cams[f].origin[1];
            c.oz = cams[f].origin[2];
            c.x_min = cams[f].x_min;
            c.y_max = cams[f].y_max;
            c.x_delta = (cams[f].x_max - cams[f].x_min) / (float)cams[f].x_res;  // render.rs:179-180
            c.y_delta = (cams[f].y_max - cams[f].y_min) / (float)cams[f].y_res;
            c.pad = 0.f;
        }
    }
    total *= frames;
    if (total >= (1ull << 30)) return RT_ERR_UNSUPPORTED;
    p.total_items = (uint32_t)total;
    // node / task pool: Tune::node_factor (default 6) nodes per level-0 item -- config 3
    // traces 3.66 node rays per pixel, config 4 the same scene at 4K; an overflow is
    // reported, never silently truncated, and the next pass gets twice the pool (rt_render
    // retries by itself).  A shadow entry packs (node << light_bits) | light, so nodes stay
    // below 2^(32 - light_bits).
    p.light_bits = light_bits(s);
    const uint64_t max_cap = pool_cap_limit(s);
    if (total >= max_cap) return RT_ERR_UNSUPPORTED;
    uint64_t want = std::max<uint64_t>(total * (uint64_t)tn.node_factor, 1u << 20);
    if (tn.node_cap) want = std::max<uint64_t>(total + 1, tn.node_cap);  // test knob
    if (&w == &s->ws) want = std::max<uint64_t>(want, s->pool_floor);
    if (want > max_cap) want = max_cap;
    const uint32_t lit_words = ((uint32_t)s->S.n_lights + 31u) / 32u > 1u ? ((uint32_t)s->S.n_lights + 31u) / 32u : 1u;
    if (w.capacity < want || w.lit_words != lit_words) {  // grows only (rt_render may have grown it after an overflow)
        w.lit_words = lit_words;
        rt_status st = grow_node_pool(w, (uint32_t)std::max<uint64_t>(want, w.capacity));
        if (st != RT_OK) return st;
    }
    if (!w.levels) {
        HIP_TRY(hipMalloc(&w.levels, RT_LEVEL_TABLE_WORDS * sizeof(uint32_t)));
        HIP_TRY(hipMalloc(&w.overflow, 64));
        // stream-ordered on the pass's own stream: a hipMemset on the null stream is not
        // ordered with the caller's non-blocking stream and could land after this pass had
        // latched an overflow (profiles/r3y: a missed RT_ERR_CAPACITY that depended on which
        // hardware queue the null stream shared with another slot's pass)
        HIP_TRY(hipMemsetAsync(w.overflow, 0, 64, stream));
    }
    // shadow queue: at most one entry per point light per hit node; Tune::shadow_factor
    // (default 2) entries per node slot, at most the point lights (config 3 queues 2.0 per
    // traced node: the trace kernel decides the rest; overflow reported like the node pool's)
    // Scenes of more than 32 point lights: lights 32 and up are never decided by the trace
    // kernel, so a hit queues about one entry per point light -- the queue is sized for that
    const double sh_per_node = s->n_point_lights > 32u ? (double)s->n_point_lights
                                                        : std::min<double>(tn.shadow_factor, (double)s->n_point_lights);
    uint64_t want_sh = std::min<uint64_t>((uint64_t)((double)w.capacity * sh_per_node), 0x7FFFFFFFu);
    if (want_sh == 0) want_sh = 1;
    const bool wide = wide_entries(s);
    if (w.shadow_capacity < want_sh || wide != (w.shadow_light != nullptr)) {
        for (uint32_t** b : {&w.shadow, &w.shadow_light}) {
            if (*b) (void)hipFree(*b);
            *b = nullptr;
        }
        want_sh = std::max<uint64_t>(want_sh, w.shadow_capacity);
        w.shadow_capacity = 0;
        HIP_TRY(hipMalloc(&w.shadow, want_sh * sizeof(uint32_t)));
        if (wide) HIP_TRY(hipMalloc(&w.shadow_light, want_sh * sizeof(uint32_t)));
        w.shadow_capacity = (uint32_t)want_sh;
    }
    const bool sort_tasks = s->S.use_bvh && tn.sort_tasks;
    const bool sort_shadow = s->S.use_bvh && tn.sort_shadow;
    p.key_mode = (uint32_t)tn.task_key;
    p.key_ahead = p.key_mode == 5 ? 0.5f : 0.25f;
    p.self_shadow = tn.self_shadow ? 1u : 0u;
    // trace levels run in queue order, grid-stride (Tune::sched: a dynamic per-wave work counter
    // measured 6.7 vs 4.9 ms; tracing a level's sorted queue from its end 939 / 947 vs 944 / 945
    // Mpixels/s, removed)
    p.sched = (uint32_t)tn.sched;
    // primary hits are coherent (8x8 tiles): their shadow rays are traced inline by the
    // trace kernel (config 3: -2%); deeper levels' hit points are scattered and go
    // through the sorted shadow queue (inlining levels 0-1: +20%, all: x2.4)
    p.inline_levels = (uint32_t)tn.inline_shadow;
    // narrowest trace task width (64: fixed 64-ray tasks) and the tasks per wave slot below
    // which a level's tasks are narrowed.  A level with fewer 64-ray tasks than half the wave
    // slots (a world-8 share's deep levels: 1.3 - 1.8 K tasks for 5120 waves) runs one task per
    // wave and lasts as long as its slowest task (p50 25 us, max 140 us: tools/trace_tail.py);
    // 32-ray tasks there: world-8 share 1.764 -> 1.584 ms (16: 1.594; 32 from a full level
    // down, task_fill 1: 1.630, and the seam's half frames lose), frames in flight and the
    // seam unchanged (profiles/r6ab/r6ah_task_width.log)
    p.task_w_min = (uint32_t)tn.task_w;
    p.task_w_fill = (float)tn.task_fill;
    // instrumented kernels (counting frames): Tune::count selects the kernels that count
    p.count_mask = s->count_ops ? (uint32_t)tn.count : 0u;
    p.lds_mask = (uint32_t)tn.lds_nodes;
    p.deep_kernel = (uint32_t)tn.deep_kernel;
    p.occ_each = (uint32_t)tn.occ_each;
    // 16-bit keys: task = direction cell | coarse origin Morton (task_key); shadow =
    // light index | the Morton bits that fit (all 15 above 16 lights' worth of bits)
    uint32_t lbits = 0;
    while ((1u << lbits) < s->S.n_lights) lbits++;
    p.light_shift = lbits <= 1 ? 15u : (16u - lbits > 15u ? 15u : 16u - lbits);
    uint32_t task_bits = (p.key_mode == 3 || p.key_mode == 4) ? 24u : 16u, shadow_bits = 16u;
    {
        // light | light-buffer cell | 3-bit distance from the light by default ("cell2": a wave
        // holds rays that test one cell's records, at similar reach; rays that walk the
        // hierarchy: light | flag | 17-bit Morton): 790 / 789 Mpixels/s vs 784 / 775 for the
        // cell alone ("cell") and 752 / 763 for light | 18-bit Morton ("18", round 1's
        // default; round 1: 4.80 ms vs 4.93 with the 16-bit key "16"); Tune::shadow_key (A/B)
        const uint32_t cell = tn.shadow_key == 1 ? 1u : (tn.shadow_key == 2 ? 2u : 0u);
        const int v = cell ? 18 : tn.shadow_key;
        p.shadow_fine = (p.key_mode == 3 || p.key_mode == 4 || v == 18) ? 18u : (v == 21 ? 21u : 0u);
        if (p.shadow_fine && p.shadow_fine + lbits > 32u) p.shadow_fine = 0u;
        // cell keys: the light-buffer cell index (x 8 distance buckets for cell2) must fit
        // below the flag bit
        const uint64_t cells = 6ull * s->S.lb_res * s->S.lb_res * (cell == 2u ? 8u : 1u);
        p.shadow_cell = (cell && p.shadow_fine == 18u && s->S.lb_res && cells < (1u << 17)) ? cell : 0u;
    }
    if (p.shadow_fine) shadow_bits = p.shadow_fine + lbits;
    // (one frame with a batch's finer keys -- 21-bit task keys, 4-bit shadow distance --
    // measured 4.08 vs 4.11 ms, split 3.88 vs 3.76: not kept)
    if (frames > 1 && spp_keys != 0) {  // the frame index above every key bit: frames are contiguous in sorted queues (ordering only)
        uint32_t fbits = 0;
        while ((1u << fbits) < frames) fbits++;
        if (!p.frame_keys) fbits = 0;  // "mixfine": the finer keys without the sample index
        // a batch's task keys take 3 radix passes of 8 bits anyway: key mode 7 fills them with
        // 5 more origin bits (task_fine=0: off, A/B)
        if (tn.task_fine && p.key_mode == 7 && task_bits == 16u && fbits <= 3) {
            p.task_fine = 1u;
            task_bits = 21u;
        }
        // ... and the shadow keys a fourth distance bit when 3 passes still hold them
        // (shadow_fine=0: off, A/B)
        if (tn.shadow_fine && p.shadow_cell == 2u && p.shadow_fine == 18u && shadow_bits + 1u + fbits <= 24u &&
            6ull * s->S.lb_res * s->S.lb_res * 16u < (1u << 18)) {
            p.shadow_cell = 3u;
            p.shadow_fine = 19u;
            shadow_bits += 1u;
        }
        // without frame bits a batch's 3 radix passes hold 24 key bits: 18-bit Morton task keys
        // and a 7-bit shadow distance (1035 / 1039 vs 1027 / 1031 Mpixels/s with the 21-bit
        // keys; key24=0: off, A/B; 4x4 direction cells | 16-bit Morton instead: no gain)
        if (tn.key24 && fbits == 0) {
            if (p.task_fine == 1u) {
                p.task_fine = 2u;
                task_bits = 24u;
            }
            if (p.shadow_cell == 3u && 6ull * s->S.lb_res * s->S.lb_res * 128u < (1u << 21) && lbits + 22u <= 24u) {
                p.shadow_cell = 4u;
                p.shadow_fine = 22u;
                shadow_bits = 22u + lbits;
            }
        }
        p.task_frame_shift = task_bits;
        p.shadow_frame_shift = shadow_bits;
        task_bits += fbits;
        shadow_bits += fbits;
        if (shadow_bits > 32u) return RT_ERR_UNSUPPORTED;
    }
    // Cell keys put the shadow rays that walk the hierarchy (origins beyond every light-buffer
    // tier: the far floor) first instead of after each light's cells: such a task takes ~20x
    // a buffered one (300 - 430 us against ~12, tools/shadow_tail.py), and at the end of the
    // queue it started last and set the shadow kernel's end.  Same key bits, ordering only.
    // World-8 share 0.469 -> 0.337 ms of shadow kernel, the seam's one frame 3.35 - 3.40 ->
    // 3.16 - 3.20 ms (profiles/r6ab/r6z_shadow_tail.log).  Measured without gain: the buffered
    // rays after them in tier order, farthest first (2 more key bits: world 1 better, world 8
    // 0.48 ms -- the far tiers' records crowd the walkers' out of the caches); consecutive
    // tasks on the waves of consecutive blocks (other CUs) instead of one block's 4 waves: flat.
    const bool walk_first = tn.walk_first && p.shadow_cell && p.shadow_fine;
    p.shadow_li_shift = walk_first ? p.shadow_fine - 1u : p.shadow_fine;
    p.shadow_walk_flag = walk_first ? 0u : (p.shadow_fine ? 1u << (p.shadow_fine - 1u) : 0u);
    p.shadow_lb_flag = walk_first ? 1u << (p.shadow_fine - 1u + lbits) : 0u;
    if (sort_tasks && w.sort_capacity < w.capacity) {
        for (uint32_t** b : {&w.task_keys, &w.perm}) {
            if (*b) (void)hipFree(*b);
            *b = nullptr;
        }
        w.sort_capacity = 0;
        for (uint32_t** b : {&w.task_keys, &w.perm}) HIP_TRY(hipMalloc(b, (size_t)w.capacity * sizeof(uint32_t)));
        w.sort_capacity = w.capacity;
    }
    if (sort_shadow && w.sort_shadow_capacity < w.shadow_capacity) {
        for (uint32_t** b : {&w.shadow_keys, &w.shadow_sorted}) {
            if (*b) (void)hipFree(*b);
            *b = nullptr;
        }
        w.sort_shadow_capacity = 0;
        for (uint32_t** b : {&w.shadow_keys, &w.shadow_sorted})
            HIP_TRY(hipMalloc(b, (size_t)w.shadow_capacity * sizeof(uint32_t)));
        w.sort_shadow_capacity = w.shadow_capacity;
    }
    // sort scratch: keys + values for the larger queue, its tile counts, digit totals
    const uint32_t sort_cap = std::max(w.capacity, w.shadow_capacity);
    const size_t sort_words =
        4 * (size_t)sort_cap + (size_t)sort_max_digits() * sort_max_tiles(sort_cap) + sort_max_digits();
    if ((sort_tasks || sort_shadow) && w.sort_tmp_words < sort_words) {
        if (w.sort_tmp) (void)hipFree(w.sort_tmp);
        w.sort_tmp = nullptr;
        w.sort_tmp_words = 0;
        HIP_TRY(hipMalloc(&w.sort_tmp, sort_words * sizeof(uint32_t)));
        w.sort_tmp_words = sort_words;
    }
    uint32_t* sort_scratch = w.sort_tmp;
    uint32_t* tile_counts = w.sort_tmp ? w.sort_tmp + 4 * (size_t)sort_cap : nullptr;
    uint32_t* digit_totals = w.sort_tmp ? tile_counts + (size_t)sort_max_digits() * sort_max_tiles(sort_cap) : nullptr;
    // radix digits of up to RT_SORT_DIGIT (8..11) bits, the fewest passes for the key: 8 by
    // default (byte digits: 3 passes for the 17-bit task keys of a 2-frame batch and the
    // 21-bit shadow keys).  At 4 passes x 2 frames in flight: 9 (task keys in 2 passes)
    // 788 / 795 vs 791 / 790 Mpixels/s, 11 (every key in 2 passes) 751 / 750 vs 789 / 785 --
    // a wider digit's ranking and tile counts cost more than the pass it saves
    const uint32_t sort_digit = 8u;
    p.task_keys = sort_tasks ? w.task_keys : nullptr;
    p.perm = nullptr;
    p.shadow_keys = sort_shadow ? w.shadow_keys : nullptr;
    // packed entries are read straight from the queue; wide ones by slot (null: slot t)
    p.shadow_in = wide ? nullptr : w.shadow;
    p.shadow_light = w.shadow_light;
    p.capacity = w.capacity;
    p.shadow_capacity = w.shadow_capacity;
    p.shadow = w.shadow;
    p.tasks = w.tasks;
    p.node_flags = w.node_flags;
    p.node_ps = w.node_ps;
    p.node_n = w.node_n;
    p.node_d = w.node_d;
    p.node_lit = w.node_lit;
    p.node_lit_hi = w.node_lit_hi;
    p.lit_words = w.lit_words;
    p.node_ec = w.node_ec;
    p.levels = w.levels;
    p.overflow = w.overflow;
    p.overflow_sticky = o.latch ? w.overflow + 1 : nullptr;
    p.out = o.rgb;
    p.out8 = o.rgb8;
    p.ray_counters = o.counters;
    if (w.forest) {
        p.node_dc = w.node_dc;
        p.node_key = w.node_key;
        p.node_pixel = w.node_pixel;
    }
    if (s->occ_trace == 0) {
        int a = 0, b = 0, c = 0;
        HIP_TRY(wave_occupancy(p, &a, &b, &c, s->occ_trace_each));
        s->occ_trace = a > 0 ? a : 1;
        s->occ_shadow = b > 0 ? b : 1;
        s->occ_combine = c > 0 ? c : 1;
    }
    int tb = s->num_cus * s->occ_trace;
    int sb = s->num_cus * s->occ_shadow;
    int cb = s->num_cus * s->occ_combine;
    {
        // the persistent trace grids at grid_pct % of a full chip (rt_scene_set_grid_share;
        // Tune::grid_pct overrides it, A/B)
        const int pct = tn.grid_pct ? tn.grid_pct : s->grid_pct;
        // the shadow pass keeps the whole chip (measured: 937 vs 927 Mpixels/s at 75%);
        // Tune::grid_pct_shadow sets its own share (A/B)
        const int spct = tn.grid_pct_shadow;
        if (pct > 0 && pct < 100) tb = std::max(1, tb * pct / 100);
        if (spct > 0 && spct < 100) sb = std::max(1, sb * spct / 100);
        // the combine grids too (50% / 25%: 928 / 918, 889 / 896 vs 936 / 940 Mpixels/s);
        // Tune::grid_pct_combine (A/B)
        const int cpct = tn.grid_pct_combine;
        if (cpct > 0 && cpct < 100) cb = std::max(1, cb * cpct / 100);
    }
    uint32_t levels = depth > 0 ? depth : 1;
    // measurement (Tune::dup, letters s / h / c): launch every queue sort / the shadow pass /
    // every combine twice -- each is idempotent -- to measure a stage's marginal cost in place
    const int dup_sort = (tn.dup & 1) ? 2 : 1, dup_shadow = (tn.dup & 2) ? 2 : 1, dup_comb = (tn.dup & 4) ? 2 : 1;
    // Every launch sizes itself from the device-side level counts: the whole frame is
    // enqueued without a host round trip (levels past the deepest non-empty one are no-ops).
    HIP_TRY(launch_wave_init(w.levels, RT_LEVEL_TABLE_WORDS, p.total_items, sample == 0 ? w.overflow : nullptr,
                             stream));
    if (w.lit_words > 1)  // lights 32 and up: their bits start at 0 (the trace kernel stores word 0 only)
        HIP_TRY(hipMemsetAsync(w.node_lit_hi, 0, (size_t)(w.lit_words - 1) * w.capacity * sizeof(uint32_t), stream));
    {
        KSpan k0(s, stream, RT_KT_TRACE);
        HIP_TRY(launch_wave_trace(p, 0, tb, stream, s->occ_trace_each, s->occ_trace));
    }
    // every level's queue is sorted (leaving any level unsorted lost: DESIGN.md)
    const uint64_t sort_levels = ~0ull;
    for (uint32_t k = 1; k < levels; k++) {
        if (o.may_sync && levels > 16 && (k & 7u) == 0) {
            // a deep pass the caller waits for anyway: stop at the first empty level (the
            // levels after it would be no-op launches; the ray trees have ended)
            uint32_t next = 0;
            HIP_TRY(hipMemcpyAsync(&next, w.levels + 2 * k + 1, sizeof(next), hipMemcpyDeviceToHost, stream));
            HIP_TRY(hipStreamSynchronize(stream));
            if (next == 0) {
                levels = k;
                break;
            }
        }
        p.perm = nullptr;  // production order unless this level is sorted
        if (sort_tasks && ((sort_levels >> (k < 64 ? k : 63)) & 1ull)) {
            KSpan ks(s, stream, RT_KT_SORT_TASKS);
            for (int r = 0; r < dup_sort; r++)
                HIP_TRY(launch_sort(w.levels, (int32_t)k, w.capacity, task_bits, w.task_keys, nullptr, sort_scratch,
                                    w.perm, tile_counts, digit_totals, 4 * s->num_cus, stream, sort_digit));
            p.perm = w.perm;
        }
        KSpan kt(s, stream, RT_KT_TRACE);
        HIP_TRY(launch_wave_trace(p, k, tb, stream, s->occ_trace_each, s->occ_trace));
    }
    if (sort_shadow) {
        KSpan ks(s, stream, RT_KT_SORT_SHADOW);
        for (int r = 0; r < dup_sort; r++)
            HIP_TRY(launch_sort(w.levels, -1, w.shadow_capacity, shadow_bits, w.shadow_keys, wide ? nullptr : w.shadow,
                                sort_scratch, w.shadow_sorted, tile_counts, digit_totals, 4 * s->num_cus, stream,
                                sort_digit));  // (wide entries: the values are the slots)
        p.shadow_in = w.shadow_sorted;
    }
    {
        KSpan ksh(s, stream, RT_KT_SHADOW);
        for (int r = 0; r < dup_shadow; r++) HIP_TRY(launch_wave_shadow(p, sb, stream));
    }
    if (w.forest) {  // no combine: the forest is shaded later, any number of times
        if (forest_done) HIP_TRY(hipEventRecord(forest_done, stream));
        HIP_TRY(hipMemcpyAsync(forest_levels, w.levels, 2 * (RT_MAX_DEPTH + 1) * sizeof(uint32_t),
                               hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        uint32_t used = 1;  // levels that hold nodes
        for (uint32_t k = 1; k < levels; k++) {
            uint32_t off = forest_levels[2 * k], cnt = forest_levels[2 * k + 1];
            if (off >= w.capacity || std::min(cnt, w.capacity - off) == 0) break;
            used = k + 1;
        }
        p.perm = nullptr;
        *forest_params = p;
        forest_levels[2 * (RT_MAX_DEPTH + 1)] = used;
        return RT_OK;
    }
    for (uint32_t k = levels; k-- > 0;) {
        KSpan kc(s, stream, RT_KT_COMBINE);
        for (int r = 0; r < dup_comb; r++) HIP_TRY(launch_wave_combine(p, k, cb, stream));
    }
    return RT_OK;
}

static rt_status render_bands_impl(const rt_scene* scene, const rt_camera* cams, uint32_t n_frames, uint32_t depth,
                                   uint32_t spp, uint32_t seed, uint32_t band_rows, uint32_t rank, uint32_t world,
                                   float* d_rgb, uint8_t* d_rgb8, uint64_t* d_counters, void* stream, bool direct) {
    rt_scene* s = const_cast<rt_scene*>(scene);
    if (!s || !cams || n_frames == 0 || n_frames > RT_MAX_FRAMES || spp == 0) return RT_ERR_INVALID_ARG;
    if (!d_rgb && (!d_rgb8 || spp > 1)) return RT_ERR_INVALID_ARG;  // spp > 1 accumulates in d_rgb
    if (n_frames > 1 && spp != 1) return RT_ERR_INVALID_ARG;
    const rt_camera* cam = cams;
    if (band_rows == 0 || world == 0 || rank >= world) return RT_ERR_INVALID_ARG;
    if (cam->x_res == 0 || cam->y_res == 0) return RT_ERR_INVALID_ARG;
    if (depth > RT_MAX_DEPTH) return RT_ERR_UNSUPPORTED;
    if ((uint64_t)cam->x_res * cam->y_res * 3 >= (1ull << 32)) return RT_ERR_UNSUPPORTED;
    HIP_TRY(hipSetDevice(s->device));
    rt_status st = ensure_ws(s, 0, 0);
    if (st != RT_OK) return st;
    hipStream_t hs = (hipStream_t)stream;
    const PassOut o{d_rgb, d_rgb8, reinterpret_cast<unsigned long long*>(d_counters), true, false, direct};
    // A pass larger (level-0 items) or deeper than any this handle has completed is checked
    // before the call returns: the pool is sized from node_factor, which suits config-3-like
    // trees, and a mirror- or glass-heavy scene needs more.  The call waits for that pass, and
    // if a queue overflowed it grows the pool and renders it again (the caller's counters
    // restored first), as rt_render does -- so a new scene or frame size costs one
    // synchronisation, not an incomplete frame.  Passes no larger than a checked one stay
    // asynchronous: an overflow there (trees that grew with the camera) is latched and
    // reported by rt_scene_sync_status, and the next pass gets twice the pool.  The node_cap
    // test knob pins the pools and skips the check.
    const uint64_t rows_local = rt_band_rows_per_rank(cam->y_res, band_rows, world);
    const uint64_t items = (uint64_t)((cam->x_res + 7u) / 8u) * ((rows_local + 7u) / 8u) * 64u * n_frames *
                           std::min<uint32_t>(spp, RT_MAX_FRAMES);
    const bool checked = !s->tune.node_cap && (items > s->checked_items || depth > s->checked_depth);
    if (checked) {
        // the check waits on the host: never inside a stream capture (rt_api.h "HOST WAIT")
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        HIP_TRY(hipStreamIsCapturing(hs, &cap));
        if (cap != hipStreamCaptureStatusNone) return RT_ERR_UNSUPPORTED;
        HIP_TRY(hipStreamSynchronize(hs));
        for (auto& se : s->ev_streams) HIP_TRY(hipEventSynchronize(se.second));
        if (s->ws.overflow) {  // an earlier pass's unreported overflow stays reported
            uint32_t v = 0;
            HIP_TRY(hipMemcpyAsync(&v, s->ws.overflow + 1, sizeof(v), hipMemcpyDeviceToHost, hs));
            HIP_TRY(hipStreamSynchronize(hs));
            if (v) {
                s->ovf_pending = true;
                HIP_TRY(hipMemsetAsync(s->ws.overflow + 1, 0, sizeof(v), hs));
            }
        }
        if (d_counters) HIP_TRY(hipMemcpyAsync(s->ws.ctr_save, d_counters, 3 * sizeof(uint64_t), hipMemcpyDeviceToDevice, hs));
    }
    for (int attempt = 0;; attempt++) {
        if (n_frames == 1) {
            st = launch_bands(s, cam, depth, spp, seed, band_rows, rank, world, o, hs);
        } else {
            st = wave_pipeline(s, s->ws, cam, depth, band_rows, rank, world, o, hs, nullptr, nullptr, 1, 0, 0,
                               n_frames, cams);
        }
        if (st != RT_OK || !checked) break;
        uint32_t ovf = 0;
        HIP_TRY(hipMemcpyAsync(&ovf, s->ws.overflow, sizeof(ovf), hipMemcpyDeviceToHost, hs));
        HIP_TRY(hipStreamSynchronize(hs));
        if (!ovf) {
            s->checked_items = std::max(s->checked_items, items);
            s->checked_depth = std::max(s->checked_depth, depth);
            break;
        }
        const uint64_t lim = pool_cap_limit(s);
        if (attempt >= 8 || s->ws.capacity >= lim) break;  // latched: rt_scene_sync_status reports it
        HIP_TRY(hipMemsetAsync(s->ws.overflow + 1, 0, sizeof(uint32_t), hs));  // rendered again
        s->pool_floor = (uint32_t)std::min<uint64_t>(2ull * s->ws.capacity, lim);
        if (d_counters)
            HIP_TRY(hipMemcpyAsync(d_counters, s->ws.ctr_save, 3 * sizeof(uint64_t), hipMemcpyDeviceToDevice, hs));
    }
    if (st != RT_OK) return st;
    hipEvent_t ev = nullptr;
    for (size_t i = 0; i < s->ev_streams.size();) {  // drop completed renders of other streams
        auto& se = s->ev_streams[i];
        if (se.first != hs && hipEventQuery(se.second) == hipSuccess) {
            (void)hipEventDestroy(se.second);
            se = s->ev_streams.back();
            s->ev_streams.pop_back();
            continue;
        }
        if (se.first == hs) ev = se.second;
        i++;
    }
    if (!ev) {
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        s->ev_streams.emplace_back(hs, ev);
    }
    HIP_TRY(hipEventRecord(ev, hs));
    return RT_OK;
}

rt_status rt_render_bands_ex_async(const rt_scene* scene, const rt_camera* cams, uint32_t n_frames, uint32_t depth,
                                   uint32_t spp, uint32_t seed, uint32_t band_rows, uint32_t rank, uint32_t world,
                                   float* d_rgb, uint8_t* d_rgb8, uint64_t* d_counters, void* stream) {
    return render_bands_impl(scene, cams, n_frames, depth, spp, seed, band_rows, rank, world, d_rgb, d_rgb8, d_counters,
                             stream, false);
}

// This rank's rows of n_frames whole frames, written in place (include/rt_api.h): several
// band shares of one device fill the same frames side by side with no assembly step
rt_status rt_render_bands_direct_async(const rt_scene* scene, const rt_camera* cams, uint32_t n_frames,
                                       uint32_t depth, uint32_t band_rows, uint32_t rank, uint32_t world,
                                       float* d_frames, uint8_t* d_frames8, uint64_t* d_counters, void* stream) {
    return render_bands_impl(scene, cams, n_frames, depth, 1, 0, band_rows, rank, world, d_frames, d_frames8,
                             d_counters, stream, true);
}

rt_status rt_render_bands_spp_async(const rt_scene* scene, const rt_camera* cam, uint32_t depth, uint32_t spp,
                                    uint32_t seed, uint32_t band_rows, uint32_t rank, uint32_t world, float* d_rgb,
                                    uint64_t* d_counters, void* stream) {
    if (!d_rgb) return RT_ERR_INVALID_ARG;
    return rt_render_bands_ex_async(scene, cam, 1, depth, spp, seed, band_rows, rank, world, d_rgb, nullptr,
                                    d_counters, stream);
}

rt_status rt_render_bands_batch_async(const rt_scene* scene, const rt_camera* cams, uint32_t n_frames,
                                      uint32_t depth, uint32_t band_rows, uint32_t rank, uint32_t world,
                                      float* d_rgb, uint64_t* d_counters, void* stream) {
    if (!d_rgb) return RT_ERR_INVALID_ARG;
    return rt_render_bands_ex_async(scene, cams, n_frames, depth, 1, 0, band_rows, rank, world, d_rgb, nullptr,
                                    d_counters, stream);
}

rt_status rt_render_bands_async(const rt_scene* scene, const rt_camera* cam, uint32_t depth,
                                uint32_t band_rows, uint32_t rank, uint32_t world, float* d_rgb,
                                uint64_t* d_counters, void* stream) {
    return rt_render_bands_spp_async(scene, cam, depth, 1, 0, band_rows, rank, world, d_rgb, d_counters, stream);
}

// rt_render's band shares on this device: s->split with n ranks (s itself and n - 1 clones,
// each rank its own stream); built on first use, rebuilt when n changes

extern "C" {

static rt_status ensure_split(rt_scene* s, int n) {
    if (s->split_n == n && s->split) return RT_OK;
    if (s->split) rt_multi_free(s->split);
    s->split = nullptr;
    s->split_n = 0;
    s->split_dev_pending = false;
    std::vector<int32_t> devs((size_t)n, s->device);
    rt_status st = rt_multi_build(s, devs.data(), (uint32_t)n, false, &s->split);
    if (st != RT_OK) return st;
    const bool count = s->count_ops;
    (void)rt_multi_each(s->split, [&](rt_scene* c) { return rt_scene_set_scan_counting(c, count); });
    s->split_n = n;
    s->split_dev_y = 0;
    return RT_OK;
}

// rt_render's seam split in stream order (rt_multi.cpp rt_multi_render_frame_async): the
// frame's top rows [0, rows) and the rest render side by side as two band shares of this
// device -- rt_render's shares (s->split: this handle and one clone, each share on the
// state's own stream; the same two streams as rt_render, since streams created later may
// share a hardware queue: 5.4 vs 3.4 ms for a frame when they did) -- forked from and
// joined back into `stream`.  The meeting row starts at the
// even split and, whenever the previous call's share spans have already completed when the
// next call is enqueued, moves 8 rows toward the share that finished first (within [half,
// 3/4] of the frame); the shares' persistent grids take Tune::seam_grid_pct (default 80) % of
// the chip, or the scene's own share if smaller.  seam_split=1 (or frames under 32 rows):
// one pass on `stream`.  No pixel depends on any of it.
rt_status rt_render_frame_async(const rt_scene* scene, const rt_camera* cam, uint32_t depth, float* d_rgb,
                                uint8_t* d_rgb8, uint64_t* d_counters, void* stream) {
    rt_scene* s = const_cast<rt_scene*>(scene);
    if (!s || !cam || !d_rgb || cam->x_res == 0 || cam->y_res == 0) return RT_ERR_INVALID_ARG;
    if (s->multi) return RT_ERR_UNSUPPORTED;  // a multi-device scene renders through rt_render
    if (depth > RT_MAX_DEPTH) return RT_ERR_UNSUPPORTED;
    if ((uint64_t)cam->x_res * cam->y_res * 3 >= (1ull << 32)) return RT_ERR_UNSUPPORTED;
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t hs = (hipStream_t)stream;
    const uint32_t y = cam->y_res;
    if (s->tune.seam_split != 2 || y < 32u) {
        // one pass: one band of 8-row tiles holding every row, padded to a multiple of 8
        const size_t n = (size_t)cam->x_res * y * 3;
        const size_t n_pad = (size_t)cam->x_res * rt_band_rows_per_rank(y, 8, 1) * 3;
        if (n_pad == n)
            return rt_render_bands_ex_async(s, cam, 1, depth, 1, 0, 8, 0, 1, d_rgb, d_rgb8, d_counters, stream);
        rt_status st = ensure_ws(s, n_pad, d_rgb8 ? n_pad : 0);
        if (st != RT_OK) return st;
        st = rt_render_bands_ex_async(s, cam, 1, depth, 1, 0, 8, 0, 1, s->ws.out, d_rgb8 ? s->ws.out8 : nullptr,
                                      d_counters, stream);
        if (st != RT_OK) return st;
        HIP_TRY(hipMemcpyAsync(d_rgb, s->ws.out, n * sizeof(float), hipMemcpyDeviceToDevice, hs));
        if (d_rgb8) HIP_TRY(hipMemcpyAsync(d_rgb8, s->ws.out8, n, hipMemcpyDeviceToDevice, hs));
        return RT_OK;
    }
    rt_status st0 = ensure_split(s, 2);
    if (st0 != RT_OK) return st0;
    const uint32_t even = ((y + 1u) / 2u + 7u) / 8u * 8u;
    const uint32_t hi = std::max(even, (y * 3u / 4u) / 8u * 8u);
    if (s->split_dev_y != y || s->split_dev_rows < even || s->split_dev_rows > hi) {
        s->split_dev_rows = even;
        s->split_dev_y = y;
        // both shares' node pools sized once for the largest share they can get (unless the
        // node_cap test knob pins them)
        const uint64_t floor = std::min<uint64_t>((uint64_t)hi * cam->x_res * (uint64_t)s->tune.node_factor,
                                                  pool_cap_limit(s));
        if (!s->tune.node_cap)
            (void)rt_multi_each_rank(s->split, [&](rt_scene* c) {
                c->pool_floor = std::max<uint32_t>(c->pool_floor, (uint32_t)floor);
                return RT_OK;
            });
    } else {
        float t[2] = {0.f, 0.f};
        if (rt_multi_async_share_ms(s->split, t, 2) == RT_OK && t[0] > 0.f && t[1] > 0.f) {
            const float late = t[1] - t[0], band = 0.03f * t[1];  // > 0: share 0 can take more rows
            if (late > band && s->split_dev_rows + 8u <= hi)
                s->split_dev_rows += 8u;
            else if (late < -band && s->split_dev_rows >= even + 8u)
                s->split_dev_rows -= 8u;
        }
    }
    const int pct = std::min(s->grid_pct, s->tune.seam_grid_pct);
    const int saved = s->grid_pct;  // read when the passes are enqueued: restored right after
    auto set_pct = [&](int v) {
        s->grid_pct = v;
        (void)rt_multi_each(s->split, [&](rt_scene* c) {
            c->grid_pct = v;
            return RT_OK;
        });
    };
    set_pct(pct);
    rt_status st = rt_multi_render_frame_async(s->split, cam, depth, s->split_dev_rows, d_rgb, d_rgb8, d_counters, hs);
    set_pct(saved);
    if (st != RT_OK) return st;
    s->split_dev_pending = true;
    return RT_OK;
}

rt_status rt_scene_sync_status(rt_scene* s) {
    if (!s) return RT_ERR_INVALID_ARG;
    rt_status st = rt_scene_sync_own(s);
    if (st != RT_OK && st != RT_ERR_CAPACITY) return st;
    bool ovf = st == RT_ERR_CAPACITY || s->split_dev_overflow;
    s->split_dev_overflow = false;
    if (s->split && s->split_dev_pending) {  // rt_render_frame_async's other share
        s->split_dev_pending = false;
        rt_status e = rt_multi_each(s->split, [&](rt_scene* c) -> rt_status {
            rt_status r = rt_scene_sync_own(c);
            if (r == RT_ERR_CAPACITY) {
                ovf = true;
                return RT_OK;
            }
            return r;
        });
        if (e != RT_OK) return e;
    }
    return ovf ? RT_ERR_CAPACITY : RT_OK;
}

rt_status rt_scene_sync_own(rt_scene* s) {
    if (!s) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(s->device));
    // every stream-ordered render of this handle is complete after this loop, so the events
    // are released (one per caller stream would otherwise accumulate for the process's life)
    for (auto& se : s->ev_streams) HIP_TRY(hipEventSynchronize(se.second));
    for (auto& se : s->ev_streams) (void)hipEventDestroy(se.second);
    s->ev_streams.clear();
    // an overflow a checked pass found latched before it rendered (rt_render_bands_ex_async)
    bool ovf = s->ovf_pending;
    s->ovf_pending = false;
    if (s->ws.overflow) {
        // read and clear the sticky word on the handle's own stream, waited for here: no
        // null-stream operation (unordered with the callers' non-blocking streams) touches it
        uint32_t v = 0;
        HIP_TRY(hipMemcpyAsync(&v, s->ws.overflow + 1, sizeof(v), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
        if (v) {
            HIP_TRY(hipMemsetAsync(s->ws.overflow + 1, 0, sizeof(v), s->stream));
            HIP_TRY(hipStreamSynchronize(s->stream));
            ovf = true;
        }
    }
    if (!ovf) return RT_OK;
    // the next pass on this scene gets a pool twice as large (up to the index limit)
    s->pool_floor = (uint32_t)std::min<uint64_t>(2ull * s->ws.capacity, pool_cap_limit(s));
    return RT_ERR_CAPACITY;
}

rt_status rt_unpermute_bands_async(const float* d_gathered, uint32_t x_res, uint32_t y_res,
                                   uint32_t band_rows, uint32_t world, float* d_frame, void* stream) {
    if (!d_gathered || !d_frame || band_rows == 0 || world == 0 || x_res == 0 || y_res == 0)
        return RT_ERR_INVALID_ARG;
    uint32_t rpr = rt_band_rows_per_rank(y_res, band_rows, world);
    HIP_TRY(launch_unpermute(d_gathered, x_res, y_res, band_rows, world, rpr, d_frame, (hipStream_t)stream));
    return RT_OK;
}

rt_status rt_unpermute_bands_u8_async(const uint8_t* d_gathered, uint32_t x_res, uint32_t y_res,
                                      uint32_t band_rows, uint32_t world, uint8_t* d_frame, void* stream) {
    if (!d_gathered || !d_frame || band_rows == 0 || world == 0 || x_res == 0 || y_res == 0)
        return RT_ERR_INVALID_ARG;
    uint32_t rpr = rt_band_rows_per_rank(y_res, band_rows, world);
    HIP_TRY(launch_unpermute_u8(d_gathered, x_res, y_res, band_rows, world, rpr, d_frame, (hipStream_t)stream));
    return RT_OK;
}

rt_status rt_unpermute_bands_batch_async(const float* d_gathered, uint32_t x_res, uint32_t y_res,
                                         uint32_t band_rows, uint32_t world, uint32_t n_frames,
                                         uint32_t stride_frames, float* d_frames, void* stream) {
    if (!d_gathered || !d_frames || band_rows == 0 || world == 0 || x_res == 0 || y_res == 0 || n_frames == 0 ||
        stride_frames < n_frames || n_frames > 65535u)
        return RT_ERR_INVALID_ARG;
    const uint32_t rpr = rt_band_rows_per_rank(y_res, band_rows, world);
    HIP_TRY(launch_unpermute(d_gathered, x_res, y_res, band_rows, world, rpr, d_frames, (hipStream_t)stream, n_frames,
                             stride_frames * rpr));
    return RT_OK;
}

rt_status rt_unpermute_bands_batch_u8_async(const uint8_t* d_gathered, uint32_t x_res, uint32_t y_res,
                                            uint32_t band_rows, uint32_t world, uint32_t n_frames,
                                            uint32_t stride_frames, uint8_t* d_frames, void* stream) {
    if (!d_gathered || !d_frames || band_rows == 0 || world == 0 || x_res == 0 || y_res == 0 || n_frames == 0 ||
        stride_frames < n_frames || n_frames > 65535u)
        return RT_ERR_INVALID_ARG;
    const uint32_t rpr = rt_band_rows_per_rank(y_res, band_rows, world);
    HIP_TRY(launch_unpermute_u8(d_gathered, x_res, y_res, band_rows, world, rpr, d_frames, (hipStream_t)stream,
                                n_frames, stride_frames * rpr));
    return RT_OK;
}

rt_status rt_quantize_u8_async(const float* d_rgb, size_t n, uint8_t* d_rgb8, void* stream) {
    if (!d_rgb || !d_rgb8) return RT_ERR_INVALID_ARG;
    if (n == 0) return RT_OK;
    HIP_TRY(launch_quantize(d_rgb, n, d_rgb8, (hipStream_t)stream));
    return RT_OK;
}

rt_status rt_render(const rt_scene* scene, const rt_camera* cam, uint32_t depth, const rt_render_opts* opts,
                    float* rgb, uint8_t* rgb8) {
    return rt_render_spp(scene, cam, depth, 1, 0, opts, rgb, rgb8);
}

rt_status rt_render_spp(const rt_scene* scene, const rt_camera* cam, uint32_t depth, uint32_t spp, uint32_t seed,
                        const rt_render_opts* opts, float* rgb, uint8_t* rgb8) {
    rt_scene* s = const_cast<rt_scene*>(scene);
    if (!s || !cam || !rgb || spp == 0) return RT_ERR_INVALID_ARG;
    if (opts && opts->device >= 0 && opts->device != s->device) return RT_ERR_INVALID_ARG;
    if (s->multi) return rt_multi_render(s, cam, depth, spp, seed, opts, rgb, rgb8);
    // One frame as S band shares of this device, rendered side by side on S streams (each
    // its own scene clone and workspace), exchanged by device copies and un-permuted: the
    // latency-bound tails of one share's levels overlap the other's work.  Tune::seam_split
    // (default 2; 1 = one pass), seam_band_rows (default: contiguous shares).  Config 3,
    // 1080p, one MI355X: 3.47 ms of device time against 4.09 for one pass (8-row bands: 3.69;
    // 3 shares: 3.80, 4: 5.08).
    const int split = s->tune.seam_split;
    if (split > 1 && cam->y_res >= 16u * (uint32_t)split) {
        if (s->split_dev_pending) {
            // a stream-ordered rt_render_frame_async on these shares is not reported yet: keep
            // its overflow for the caller's rt_scene_sync_status (this render's own status
            // checks below would otherwise consume it)
            rt_status ps = rt_scene_sync_status(s);
            if (ps == RT_ERR_CAPACITY)
                s->split_dev_overflow = true;
            else if (ps != RT_OK)
                return ps;
        }
        rt_status es = ensure_split(s, split);
        if (es != RT_OK) return es;
        // contiguous shares by default (top / bottom halves: 3.47 ms against 3.69 with 8-row
        // bands dealt in turn -- shares of different content fall out of step, so one share's
        // level tails meet the other's work)
        const uint32_t br = (uint32_t)s->tune.seam_band_rows;
        const uint32_t even = ((cam->y_res + (uint32_t)split - 1u) / (uint32_t)split + 7u) / 8u * 8u;
        // Two shares meet where share 1 finishes as share 0's rows reach the caller (share 0's
        // copy then runs under share 1's tail): after each render the row moves 8 rows toward
        // the share that is late on that mark (within [half, 3/4] of the frame: share 0 holds
        // one band only down to half the rows).  Config 3: share 0 (the top) is the cheaper
        // half; fixed rows 544 / 576 / 608 measured 3.38 / 3.35 / 3.37 ms of device time
        // (seam_band_rows pins the row, seam_adapt=0 keeps the even split, seam_adapt=device
        // balances the finish times alone)
        const bool adapt = !br && split == 2 && s->tune.seam_adapt != 0;
        const bool adapt_copy = s->tune.seam_adapt != 2;
        const uint32_t hi = std::max(even, (cam->y_res * 3u / 4u) / 8u * 8u);
        if (s->seam_y != cam->y_res || s->seam_rows < even || s->seam_rows > hi) {
            s->seam_rows = even;
            s->seam_y = cam->y_res;
            if (adapt && !s->tune.node_cap) {  // every share's node pool sized once for the largest
                                                // share it can get (unless the node_cap test knob
                                                // pins the pools)
                const uint64_t floor = std::min<uint64_t>((uint64_t)hi * cam->x_res * (uint64_t)s->tune.node_factor,
                                                          pool_cap_limit(s));
                auto raise = [&](rt_scene* c) {
                    c->pool_floor = std::max<uint32_t>(c->pool_floor, (uint32_t)floor);
                    return RT_OK;
                };
                (void)raise(s);
                (void)rt_multi_each(s->split, raise);
            }
        }
        const uint32_t rows = br ? br : (adapt ? s->seam_rows : even);
        rt_multi_set_band_rows(s->split, rows);
        // the shares' persistent grids at Tune::seam_grid_pct % of the chip (default 80: two
        // concurrent full-chip grids leave more blocks waiting for a slot; 100 / 90 / 80 at
        // the 576-row meeting: 3.35 / 3.31 - 3.34 / 3.30 - 3.31 ms), or the scene's own
        // share if that is smaller; restored afterwards
        const int pct = std::min(s->grid_pct, s->tune.seam_grid_pct);
        const int saved = s->grid_pct;
        auto set_pct = [&](int v) {
            s->grid_pct = v;
            (void)rt_multi_each(s->split, [&](rt_scene* c) {
                c->grid_pct = v;
                return RT_OK;
            });
        };
        set_pct(pct);
        rt_status st = rt_multi_render_state(s->split, cam, depth, spp, seed, opts, rgb, rgb8);
        set_pct(saved);
        if (st == RT_OK && adapt) {
            float t[2] = {0.f, 0.f}, c[2] = {0.f, 0.f};
            if (rt_multi_share_ms(s->split, t, 2) == RT_OK && t[0] > 0.f && t[1] > 0.f &&
                (!adapt_copy || rt_multi_copy_ms(s->split, c, 2) == RT_OK)) {
                // > 0: share 1 ends after share 0's rows are out -- share 0 can take more rows
                const float late = t[1] - (t[0] + c[0]), band = 0.03f * t[1];
                if (late > band && s->seam_rows + 8u <= hi)
                    s->seam_rows += 8u;
                else if (late < -band && s->seam_rows >= even + 8u)
                    s->seam_rows -= 8u;
            }
        }
        return st;
    }
    HIP_TRY(hipSetDevice(s->device));
    size_t n = (size_t)cam->x_res * cam->y_res * 3;
    // one band share holding every row: its buffer has the padded row count (the pass
    // zero-fills rows y_res .. rows_local - 1); the first y_res rows are the frame
    const size_t n_pad = (size_t)cam->x_res * rt_band_rows_per_rank(cam->y_res, 8, 1) * 3;
    rt_status st = ensure_ws(s, n_pad, rgb8 ? n_pad : 0);
    if (st != RT_OK) return st;
    hipStream_t stream = s->stream;
    for (int attempt = 0;; attempt++) {
        HIP_TRY(hipMemsetAsync(s->ws.counters, 0, 4 * sizeof(unsigned long long), stream));
        HIP_TRY(hipEventRecord(s->ev0, stream));
        // single device: one "band" holding every row; as_u8 fused into the level-0 combine
        const PassOut o{s->ws.out, rgb8 ? s->ws.out8 : nullptr, s->ws.counters, false, true};
        st = launch_bands(s, cam, depth, spp, seed, 8, 0, 1, o, stream);
        if (st != RT_OK) return st;
        HIP_TRY(hipEventRecord(s->ev1, stream));
        if (!s->ws.overflow) break;
        uint32_t ovf = 0;
        HIP_TRY(hipMemcpyAsync(&ovf, s->ws.overflow, sizeof(ovf), hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        if (!ovf) break;
        // node pool too small for this scene's ray trees: grow it and render again
        const uint64_t lim = pool_cap_limit(s);
        if (attempt >= 8 || s->ws.capacity >= lim) return RT_ERR_CAPACITY;
        rt_status g = grow_node_pool(s->ws, (uint32_t)std::min<uint64_t>(2ull * s->ws.capacity, lim));
        if (g != RT_OK) return g;
    }
    HIP_TRY(hipMemcpyAsync(rgb, s->ws.out, n * sizeof(float), hipMemcpyDeviceToHost, stream));
    if (rgb8) HIP_TRY(hipMemcpyAsync(rgb8, s->ws.out8, n, hipMemcpyDeviceToHost, stream));
    unsigned long long cnt[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(cnt, s->ws.counters, sizeof(cnt), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    if (opts && opts->counters) {
        opts->counters->node_rays = cnt[0];
        opts->counters->shadow_rays = cnt[1];
        opts->counters->pixels = cnt[2];
        opts->counters->wave_iterations = cnt[3];
    }
    if (opts && opts->kernel_ms) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, s->ev0, s->ev1));
        *opts->kernel_ms = ms;
    }
    return RT_OK;
}

}  // extern "C"

// debug (tests/test_gpu_sort.py): the ray-queue radix sort on its own.  Sorts n device keys
// (their low `bits` bits) with digits of up to max_digit bits, stably; the values (d_vals, or
// the indices 0..n-1 when null) land in d_vals_out in key order.  Runs on the current device
// and synchronises it.
extern "C" int rt_debug_sort(const uint32_t* d_keys, const uint32_t* d_vals, uint32_t n, uint32_t bits,
                             uint32_t max_digit, uint32_t* d_vals_out) {
    if (!d_keys || !d_vals_out || bits == 0 || bits > 32) return RT_ERR_INVALID_ARG;
    if (n == 0) return RT_OK;
    uint32_t* levels = nullptr;
    uint32_t* tmp = nullptr;
    int rc = RT_OK;
    const size_t words = 4 * (size_t)n + (size_t)sort_max_digits() * sort_max_tiles(n) + sort_max_digits();
    if (hipMalloc(&levels, RT_LEVEL_TABLE_WORDS * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&tmp, words * sizeof(uint32_t)) != hipSuccess) {
        rc = RT_ERR_HIP;
    } else {
        // the shadow queue's slot: count at levels[2 (RT_MAX_DEPTH + 1)], offset 0
        std::vector<uint32_t> lv(RT_LEVEL_TABLE_WORDS, 0u);
        lv[2 * (RT_MAX_DEPTH + 1)] = n;
        uint32_t* tiles = tmp + 4 * (size_t)n;
        uint32_t* totals = tiles + (size_t)sort_max_digits() * sort_max_tiles(n);
        int cus = 0, dev = 0;
        if (hipMemcpy(levels, lv.data(), lv.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess ||
            hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            rc = RT_ERR_HIP;
        else if (launch_sort(levels, -1, n, bits, d_keys, d_vals, tmp, d_vals_out, tiles, totals, 4 * cus, 0,
                             max_digit) != hipSuccess ||
                 hipDeviceSynchronize() != hipSuccess)  // d_vals == null: the values are the indices
            rc = RT_ERR_HIP;
    }
    if (levels) (void)hipFree(levels);
    if (tmp) (void)hipFree(tmp);
    return rc;
}
