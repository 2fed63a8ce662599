// rt_scene.hpp -- the scene handle behind the C ABI (struct rt_scene), its render workspace and
// the helpers the library's translation units share: rt_scene.cpp (handle life cycle, updates,
// tuning), rt_render.cpp (the render driver), rt_forest.cpp (ray forests), rt_build.cpp (the
// host scene build).  Internal (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_device.hpp"
#include "rt_internal.hpp"
#include "rt_tune.hpp"

namespace rtdev {
hipError_t launch_unpermute(const float* in, uint32_t x_res, uint32_t y_res, uint32_t band_rows,
                            uint32_t world, uint32_t rows_per_rank, float* out, hipStream_t stream,
                            uint32_t frames = 1, uint32_t rank_rows = 0);
hipError_t launch_quantize(const float* in, size_t n, uint8_t* out, hipStream_t stream);
hipError_t launch_unpermute_u8(const uint8_t* in, uint32_t x_res, uint32_t y_res, uint32_t band_rows,
                               uint32_t world, uint32_t rows_per_rank, uint8_t* out, hipStream_t stream,
                               uint32_t frames = 1, uint32_t rank_rows = 0);
bool rt_cube_table_check(const float* table);
hipError_t wave_occupancy(const WaveParams& p, int* trace_blocks, int* shadow_blocks, int* combine_blocks,
                          int* trace_each);
hipError_t launch_wave_shadow(const WaveParams& p, int blocks, hipStream_t stream);
hipError_t launch_wave_init(uint32_t* levels, uint32_t n_words, uint32_t total_items, uint32_t* overflow,
                            hipStream_t stream);
hipError_t launch_wave_trace(const WaveParams& p, uint32_t level, int blocks, hipStream_t stream,
                             const int* occ_each = nullptr, int occ_min = 0);
hipError_t launch_wave_combine(const WaveParams& p, uint32_t level, int blocks, hipStream_t stream);
hipError_t launch_forest_shade(const WaveParams& p, uint32_t level, int blocks, float* frame, hipStream_t stream);
hipError_t launch_forest_mark(const uint32_t* node_key, const uint32_t* node_pixel, const uint32_t* node_flags,
                              uint32_t n_nodes, const uint8_t* key_mask, uint32_t n_keys, uint8_t* mark,
                              uint32_t* sizes, hipStream_t stream);
hipError_t launch_sort(const uint32_t* levels, int32_t level, uint32_t cap, uint32_t bits, const uint32_t* keys,
                       const uint32_t* vals, uint32_t* tmp, uint32_t* vals_out,
                         uint32_t* tile_counts, uint32_t* digit_totals, int blocks, hipStream_t stream,
                         uint32_t max_digit);
uint32_t sort_max_tiles(uint32_t cap);
uint32_t sort_max_digits();
hipError_t launch_spp_accumulate(const float* samples, uint32_t n, size_t frame_floats, uint32_t first, uint32_t spp,
                                 float* out, uint8_t* out8, hipStream_t stream);
}  // namespace rtdev

using namespace rtdev;

namespace rthost {

struct Workspace {
    float* out = nullptr;            // device frame (rt_render)
    size_t out_floats = 0;
    uint8_t* out8 = nullptr;
    size_t out8_bytes = 0;
    unsigned long long* counters = nullptr;  // [node, shadow, pixels, wave iterations]
    uint32_t* work = nullptr;        // persistent-kernel work counter
    // level-synchronous pipeline: the node arrays of rt_device.hpp
    Task* tasks = nullptr;
    uint32_t* node_flags = nullptr;  // [capacity]
    float4* node_ps = nullptr;       // [capacity] shadow-ray origins, texture u
    float4* node_n = nullptr;        // [capacity] normals, texture v
    float4* node_d = nullptr;        // [capacity] ray directions, parents
    uint32_t* node_lit = nullptr;    // [capacity] unshadowed-light bits (lights 0-31)
    uint32_t* node_lit_hi = nullptr; // [(lit_words - 1) x capacity] lights 32 and up
    uint32_t lit_words = 1;          // ceil(lights / 32) (rt_device.hpp WaveParams::lit_words)
    float4* node_ec = nullptr;       // [2 x capacity] children's colours
    uint32_t capacity = 0;
    uint32_t* shadow = nullptr;      // shadow queue
    uint32_t* shadow_light = nullptr;  // wide entries (> 256 lights): each entry's light
    uint32_t shadow_capacity = 0;
    uint32_t* levels = nullptr;      // RT_LEVEL_TABLE_WORDS words
    uint32_t* overflow = nullptr;    // [0] this pass's queue overflows, [1] sticky (rt_scene_sync_status)
    uint64_t* ctr_save = nullptr;    // a checked pass's caller counters before it (rt_render_bands_ex_async)
    // queue ordering (rt_order.hip)
    uint32_t* task_keys = nullptr;   // [capacity] x2 buffers
    uint32_t* perm = nullptr;
    uint32_t sort_capacity = 0;
    uint32_t* shadow_keys = nullptr; // [shadow_capacity] x2 buffers
    uint32_t* shadow_sorted = nullptr;
    uint32_t sort_shadow_capacity = 0;
    uint32_t* sort_tmp = nullptr;    // scratch keys + values, 256 x tiles counts, 256 digit totals
    size_t sort_tmp_words = 0;
    // ray forest only (rt_forest): per-node shade inputs, grown with the pool
    bool forest = false;
    float4* node_dc = nullptr;       // [2 x capacity] children's directions
    uint32_t* node_key = nullptr;
    uint32_t* node_pixel = nullptr;
    // sample batches: one band buffer per sample of a batch (launch_bands_wave)
    float* spp_buf = nullptr;
    size_t spp_buf_floats = 0;
};

// Task ordering key (rt_wavefront.hip task_key / inside_key; Tune::task_key): 7 (default) =
// a ray inside a sphere or cube (the refracted child of an entering hit, the reflected child
// of a hit from inside) is keyed by that shape's centre (1 | 15-bit Morton of the centre), so
// a wave holds the rays trapped in one or two shapes; every other ray by face x 2x2
// direction cells | 10-bit Morton code of a point 0.25 x (scene radius) ahead on the ray
// (mode 6 with one bit less).  Measured alternatives (config 3, 1080p): 1 = face
// x 2x2 cells | 11-bit Morton origin 4.90 ms, 6 at 0.10 - 0.35 ahead 4.81 - 4.94, 5 (0.5
// ahead) +1.5%, 3 / 4 (24-bit keys) 6.13 / 6.42 vs 5.78 for mode 1.
int g_num_cus(int device);

}  // namespace rthost

struct rt_scene {
    int device = 0;
    void* dmem = nullptr;
    size_t dbytes = 0;
    DevScene S;
    uint64_t flops_per_scan = 0;
    uint32_t n_point_lights = 0;
    int num_cus = 256;
    int occ_trace = 0, occ_shadow = 0, occ_combine = 0;
    int occ_trace_each[3] = {0, 0, 0};  // generic / level-0 / deep trace instantiations
    bool count_ops = false;  // rt_scene_set_scan_counting
    int grid_pct = 100;      // rt_scene_set_grid_share: % of a full chip for persistent grids
    Tune tune;               // rt_tune.hpp: fixed scene-build keys, pass keys (rt_scene_set_tuning)
    rthost::Workspace ws;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // one event per stream a stream-ordered render ran on, recorded after each such render:
    // rt_scene_sync_status and rt_scene_destroy wait for every one of them
    std::vector<std::pair<hipStream_t, hipEvent_t>> ev_streams;
    uint32_t pool_floor = 0;       // node-pool size the next pass grows to (after a reported overflow)
    double normal_max = 1.0;       // largest hit-normal length (dark_zero of an edited material)
    rt_multi_state* multi = nullptr;  // rt_scene_create_multi: the other devices' clones (rt_multi.cpp)
    rt_multi_state* split = nullptr;  // rt_render's band shares on this one device (seam_split)
    int split_n = 0;
    uint32_t seam_rows = 0, seam_y = 0;  // the two shares' meeting row (adapted per render) for y_res seam_y
    // rt_render_frame_async (on `split`, rt_render's shares): its meeting row for y_res
    // split_dev_y, whether a render awaits rt_scene_sync_status, and an overflow of such a
    // render that rt_render's own status check found first (reported by the next
    // rt_scene_sync_status)
    uint32_t split_dev_rows = 0, split_dev_y = 0;
    bool split_dev_pending = false, split_dev_overflow = false;
    // rt_render_bands_ex_async: the largest pass (level-0 items, depth) checked for overflow on
    // this handle, and an overflow of an earlier pass that such a check found latched
    // (reported by sync_status)
    uint64_t checked_items = 0;
    uint32_t checked_depth = 0;
    bool ovf_pending = false;
    // the description the device scene was built from (rt_scene_update compares against it)
    std::vector<rt_material> d_mats;
    std::vector<rt_shape> d_shapes;
    std::vector<rt_light> d_lights;
    rt_color d_ambient{0.f, 0.f, 0.f};
    // bumped by every rebuild rt_scene_update adopts: a forest made before it refuses to shade
    // (its trees hold the old scene's material indices and light count)
    uint64_t generation = 0;
    // rt_scene_set_kernel_timing: HIP events around every launch of this handle's passes, by
    // kernel kind (RT_KT_*), summed by rt_scene_kernel_times
    bool ktime = false;
    std::vector<hipEvent_t> kt_events;        // pool, reused
    std::vector<std::pair<int, size_t>> kt_spans;  // (kind, index of the start event; end = +1)
    size_t kt_used = 0;
};

namespace rthost {

// Brackets one launch of kind `kind` with a pair of events when the handle times its kernels.
struct KSpan {
    rt_scene* s;
    hipStream_t st;
    size_t at = 0;
    bool on = false;
    KSpan(rt_scene* sc, hipStream_t stream, int kind) : s(sc), st(stream) {
        if (!s->ktime) return;
        if (s->kt_used + 2 > s->kt_events.size()) {
            for (int i = 0; i < 64; i++) {
                hipEvent_t e = nullptr;
                if (hipEventCreate(&e) != hipSuccess) return;
                s->kt_events.push_back(e);
            }
        }
        at = s->kt_used;
        s->kt_used += 2;
        on = hipEventRecord(s->kt_events[at], st) == hipSuccess;
        if (on) s->kt_spans.emplace_back(kind, at);
    }
    ~KSpan() {
        if (on) (void)hipEventRecord(s->kt_events[at + 1], st);
    }
};

inline rt_status hip_status(hipError_t e) {
    if (e == hipSuccess) return RT_OK;
    if (e == hipErrorOutOfMemory) return RT_ERR_OUT_OF_MEMORY;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return RT_ERR_NO_DEVICE;
    return RT_ERR_HIP;
}
// a failing HIP call is reported on stderr (expression, line, HIP's message)
#define HIP_TRY(x)                                                                                   \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            std::fprintf(stderr, "%s:%d: %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));\
            return hip_status(e_);                                                                   \
        }                                                                                            \
    } while (0)

inline rt_status select_device(int32_t device, int* resolved) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return RT_ERR_NO_DEVICE;
    int d = device;
    if (d < 0) HIP_TRY(hipGetDevice(&d));
    if (d >= n) return RT_ERR_NO_DEVICE;
    HIP_TRY(hipSetDevice(d));
    *resolved = d;
    return RT_OK;
}

// Shadow entries: packed (node << bits) | light in 4 B for scenes of up to 256 lights (8 bits);
// "wide" above that -- the node in shadow[], its light in shadow_light[] (rt_device.hpp), so that
// a scene of many lights keeps the full node pool (RT_MAX_LIGHTS).
constexpr uint32_t PACKED_LIGHT_BITS = 8;
inline uint32_t light_index_bits(const rt_scene* s) {
    uint32_t b = 1;
    while ((1u << b) < (uint32_t)s->S.n_lights) b++;
    return b;
}
inline bool wide_entries(const rt_scene* s) { return light_index_bits(s) > PACKED_LIGHT_BITS; }
inline uint32_t light_bits(const rt_scene* s) { return wide_entries(s) ? 0u : light_index_bits(s); }
// Largest node pool: node indices must fit a packed shadow entry beside the light index (and
// (node << 1) | slot a parent reference).
inline uint64_t pool_cap_limit(const rt_scene* s) { return std::min<uint64_t>(1ull << (32 - light_bits(s)), 1ull << 30); }

// rt_render.cpp: the workspace's device buffers
rt_status ensure_ws(rt_scene* s, size_t out_floats, size_t out8_bytes);
rt_status grow_node_pool(Workspace& w, uint32_t cap);
void free_workspace(Workspace& w);

// Where one render pass's results go: the float frame (or band buffer), optionally its
// Color::as_u8 bytes (fused into the level-0 combine), ray counters, and whether queue
// overflows are latched into the scene's sticky status (the stream-ordered entry points;
// rt_render retries instead).
struct PassOut {
    float* rgb;
    uint8_t* rgb8;
    unsigned long long* counters;
    bool latch;
    bool may_sync;  // the caller waits anyway (rt_render, forests): deep passes stop at the first empty level
    bool direct = false;  // rgb / rgb8 are whole frames: this rank's rows land in place (row-major)
};

// The level-synchronous pipeline into workspace `w` (rt_render.cpp): trace(0..L-1), the shadow
// pass, then combine(L-1..0), all on `stream`.  Forest builds (w.forest) write the per-node
// shade inputs, always read the level sizes on the host, skip the combine pass and leave the
// parameters (with the device level table) in *forest_params (forest_done recorded after the
// last launch).
rt_status wave_pipeline(rt_scene* s, Workspace& w, const rt_camera* cam, uint32_t depth, uint32_t band_rows,
                        uint32_t rank, uint32_t world, const PassOut& o, hipStream_t stream,
                        WaveParams* forest_params, uint32_t* forest_levels, uint32_t spp = 1,
                        uint32_t sample = 0, uint32_t seed = 0, uint32_t frames = 1,
                        const rt_camera* cams = nullptr, bool spp_batch = false,
                        hipEvent_t forest_done = nullptr);

// rt_scene.cpp: a new handle of `d` on `device` with tuning `tn`
rt_status create_handle(const rt_scene_desc* d, int32_t device, const Tune& tn, rt_scene** out);

}  // namespace rthost
