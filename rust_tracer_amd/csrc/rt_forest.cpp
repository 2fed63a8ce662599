// rt_forest.cpp -- the ray-forest path of the C ABI (src/render_tree.rs).
// ---------------------------------------------------------------- ray forest
// render_tree.rs: generate_ray_forest (:147-164) keeps every intersection of every
// pixel's ray tree; render_forest (:121-127) shades the whole forest; render_forest_filter
// (:129-145) re-shades only trees that hold a mutated shape.  On the device the forest is
// the level-synchronous pipeline's node pool, kept after the trace + shadow passes, plus
// per node: material index, texture coordinates, `entering`, the shape id and the pixel.
#include "rt_scene.hpp"

using namespace rtdev;
using namespace rthost;

struct rt_forest {
    rt_scene* s = nullptr;
    uint64_t generation = 0;    // the scene's rt_scene::generation at creation
    rt_camera cam{};
    uint32_t depth = 0;
    Workspace ws;
    WaveParams p{};
    uint32_t levels[2 * (RT_MAX_DEPTH + 1) + 1] = {};  // (offset, count) per level, then levels used
    uint32_t n_nodes = 0;
    float* frame = nullptr;     // [y_res * x_res * 3] the last shade
    uint8_t* mark = nullptr;    // [pixels] dirty / tree-holds-id marks
    uint8_t* key_mask = nullptr;
    uint32_t n_keys = 0;
    uint32_t* sizes = nullptr;  // [pixels]
    unsigned long long* counters = nullptr;  // node, shadow, pixels of the build
    // device time of the build's last pass and of the last shade (rt_forest_timings)
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    bool shaded = false;
};

namespace {

size_t forest_pixels(const rt_forest* f) { return (size_t)f->cam.x_res * f->cam.y_res; }

rt_status forest_shade(rt_forest* f, const uint8_t* dirty) {
    WaveParams p = f->p;
    p.S = f->s->S;  // current material table
    p.dirty = dirty;
    int cb = f->s->num_cus * (f->s->occ_combine > 0 ? f->s->occ_combine : 1);
    uint32_t used = f->levels[2 * (RT_MAX_DEPTH + 1)];
    for (uint32_t k = used; k-- > 0;) HIP_TRY(launch_forest_shade(p, k, cb, f->frame, f->s->stream));
    HIP_TRY(hipEventRecord(f->ev[3], f->s->stream));
    f->shaded = true;
    return RT_OK;
}
// a rebuild since the forest was made: its nodes' material indices and lit words describe
// the old scene, which the handle no longer holds (rt_api.h rt_scene_update)
bool forest_stale(const rt_forest* f) { return f->generation != f->s->generation; }

// mark[pixel] = tree holds one of `ids` (or sizes per pixel when ids == nullptr)
rt_status forest_mark(rt_forest* f, const int32_t* ids, uint32_t n_ids, bool sizes, hipEvent_t start = nullptr) {
    hipStream_t st = f->s->stream;
    size_t px = forest_pixels(f);
    const uint8_t* mask = nullptr;
    if (ids) {
        std::vector<uint8_t> h(f->n_keys, 0);
        for (uint32_t i = 0; i < n_ids; i++)
            if (ids[i] >= 0 && (uint32_t)ids[i] < f->n_keys) h[ids[i]] = 1;
        HIP_TRY(hipMemcpyAsync(f->key_mask, h.data(), f->n_keys, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemsetAsync(f->mark, 0, px, st));
        HIP_TRY(hipStreamSynchronize(st));  // h goes out of scope
        mask = f->key_mask;
    }
    if (sizes) HIP_TRY(hipMemsetAsync(f->sizes, 0, px * sizeof(uint32_t), st));
    if (start) HIP_TRY(hipEventRecord(start, st));
    HIP_TRY(launch_forest_mark(f->ws.node_key, f->ws.node_pixel, f->ws.node_flags, f->n_nodes, mask, f->n_keys, f->mark,
                               sizes ? f->sizes : nullptr, st));
    return RT_OK;
}

}  // namespace

extern "C" {

rt_status rt_forest_create(rt_scene* s, const rt_camera* cam, uint32_t depth, rt_forest** out) {
    if (!s || !cam || !out) return RT_ERR_INVALID_ARG;
    if (cam->x_res == 0 || cam->y_res == 0) return RT_ERR_INVALID_ARG;
    if (depth > RT_MAX_DEPTH) return RT_ERR_UNSUPPORTED;
    if ((uint64_t)cam->x_res * cam->y_res * 3 >= (1ull << 32)) return RT_ERR_UNSUPPORTED;
    HIP_TRY(hipSetDevice(s->device));
    std::unique_ptr<rt_forest> f(new (std::nothrow) rt_forest());
    if (!f) return RT_ERR_OUT_OF_MEMORY;
    f->s = s;
    f->generation = s->generation;
    f->cam = *cam;
    f->depth = depth;
    f->ws.forest = true;
    size_t px = forest_pixels(f.get());
    f->n_keys = std::max<uint32_t>((uint32_t)s->S.n_shapes, 12u);  // cube hits report ids 0..11
    struct Guard {  // frees everything if creation fails half way
        rt_forest* f;
        ~Guard() {
            if (!f) return;
            free_workspace(f->ws);
            for (void* b : {(void*)f->frame, (void*)f->mark, (void*)f->key_mask, (void*)f->sizes, (void*)f->counters})
                if (b) (void)hipFree(b);
            for (hipEvent_t e : f->ev)
                if (e) (void)hipEventDestroy(e);
        }
    } guard{f.get()};
    for (hipEvent_t& e : f->ev) HIP_TRY(hipEventCreate(&e));
    HIP_TRY(hipMalloc(&f->frame, px * 3 * sizeof(float)));
    HIP_TRY(hipMalloc(&f->mark, px));
    HIP_TRY(hipMalloc(&f->key_mask, f->n_keys));
    HIP_TRY(hipMalloc(&f->sizes, px * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&f->counters, 4 * sizeof(unsigned long long)));
    hipStream_t st = s->stream;
    const uint32_t band_rows = 8;
    for (int attempt = 0;; attempt++) {
        HIP_TRY(hipMemsetAsync(f->counters, 0, 4 * sizeof(unsigned long long), st));
        const PassOut o{nullptr, nullptr, f->counters, false, true};
        HIP_TRY(hipEventRecord(f->ev[0], st));
        rt_status r = wave_pipeline(s, f->ws, cam, depth, band_rows, 0, 1, o, st, &f->p, f->levels, 1, 0, 0, 1,
                                    nullptr, false, f->ev[1]);
        if (r != RT_OK) return r;
        uint32_t ovf = 0;
        HIP_TRY(hipMemcpyAsync(&ovf, f->ws.overflow, sizeof(ovf), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (!ovf) break;
        const uint64_t lim = pool_cap_limit(s);
        if (attempt >= 8 || f->ws.capacity >= lim) return RT_ERR_CAPACITY;
        rt_status g = grow_node_pool(f->ws, (uint32_t)std::min<uint64_t>(2ull * f->ws.capacity, lim));
        if (g != RT_OK) return g;
    }
    uint32_t used = f->levels[2 * (RT_MAX_DEPTH + 1)];
    f->n_nodes = used ? f->levels[2 * (used - 1)] + f->levels[2 * (used - 1) + 1] : 0;
    guard.f = nullptr;
    *out = f.release();
    return RT_OK;
}

rt_status rt_forest_destroy(rt_forest* f) {
    if (!f) return RT_ERR_INVALID_ARG;
    (void)hipSetDevice(f->s->device);
    (void)hipStreamSynchronize(f->s->stream);
    free_workspace(f->ws);
    for (void* b : {(void*)f->frame, (void*)f->mark, (void*)f->key_mask, (void*)f->sizes, (void*)f->counters})
        if (b) (void)hipFree(b);
    for (hipEvent_t e : f->ev)
        if (e) (void)hipEventDestroy(e);
    delete f;
    return RT_OK;
}

rt_status rt_forest_timings(const rt_forest* f, float* build_ms, float* shade_ms) {
    if (!f) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(f->s->device));
    if (build_ms) HIP_TRY(hipEventElapsedTime(build_ms, f->ev[0], f->ev[1]));
    if (shade_ms) {
        *shade_ms = 0.f;
        if (f->shaded) HIP_TRY(hipEventElapsedTime(shade_ms, f->ev[2], f->ev[3]));
    }
    return RT_OK;
}

rt_status rt_forest_render(rt_forest* f, float* rgb) {
    if (!f || !rgb) return RT_ERR_INVALID_ARG;
    if (forest_stale(f)) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(f->s->device));
    HIP_TRY(hipEventRecord(f->ev[2], f->s->stream));
    rt_status r = forest_shade(f, nullptr);
    if (r != RT_OK) return r;
    HIP_TRY(hipMemcpyAsync(rgb, f->frame, forest_pixels(f) * 3 * sizeof(float), hipMemcpyDeviceToHost,
                           f->s->stream));
    HIP_TRY(hipStreamSynchronize(f->s->stream));
    return RT_OK;
}

rt_status rt_forest_render_filter(rt_forest* f, const int32_t* mutated_ids, uint32_t n_ids, float* rgb) {
    if (!f || !rgb || (n_ids && !mutated_ids)) return RT_ERR_INVALID_ARG;
    if (forest_stale(f)) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(f->s->device));
    hipStream_t st = f->s->stream;
    size_t bytes = forest_pixels(f) * 3 * sizeof(float);
    HIP_TRY(hipMemcpyAsync(f->frame, rgb, bytes, hipMemcpyHostToDevice, st));  // untouched pixels keep these
    rt_status r = forest_mark(f, mutated_ids, n_ids, false, f->ev[2]);
    if (r != RT_OK) return r;
    r = forest_shade(f, f->mark);
    if (r != RT_OK) return r;
    HIP_TRY(hipMemcpyAsync(rgb, f->frame, bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return RT_OK;
}

rt_status rt_forest_tree_sizes(rt_forest* f, uint32_t* sizes) {
    if (!f || !sizes) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(f->s->device));
    rt_status r = forest_mark(f, nullptr, 0, true);
    if (r != RT_OK) return r;
    HIP_TRY(hipMemcpyAsync(sizes, f->sizes, forest_pixels(f) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           f->s->stream));
    HIP_TRY(hipStreamSynchronize(f->s->stream));
    return RT_OK;
}

rt_status rt_forest_trees_with(rt_forest* f, int32_t shape_id, uint64_t* count) {
    if (!f || !count) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(f->s->device));
    rt_status r = forest_mark(f, &shape_id, 1, false);
    if (r != RT_OK) return r;
    std::vector<uint8_t> m(forest_pixels(f));
    HIP_TRY(hipMemcpyAsync(m.data(), f->mark, m.size(), hipMemcpyDeviceToHost, f->s->stream));
    HIP_TRY(hipStreamSynchronize(f->s->stream));
    uint64_t n = 0;
    for (uint8_t v : m) n += v;
    *count = n;
    return RT_OK;
}

rt_status rt_forest_counters(const rt_forest* f, rt_counters* out) {
    if (!f || !out) return RT_ERR_INVALID_ARG;
    unsigned long long h[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpy(h, f->counters, sizeof(h), hipMemcpyDeviceToHost));
    out->node_rays = h[0];
    out->shadow_rays = h[1];
    out->pixels = h[2];
    out->wave_iterations = 0;
    return RT_OK;
}

}  // extern "C"
