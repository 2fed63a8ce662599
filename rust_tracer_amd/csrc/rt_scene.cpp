// rt_scene.cpp -- the C ABI's scene handles (include/rt_api.h): creation (the host build of
// rt_build.cpp uploaded as one allocation), clones, destruction, tuning and queries, and the
// updates a drop-in render() binding makes between frames (rt_scene_update, rt_scene_set_material:
// the reference's Scene edited in place, my_scene.rs / gui.rs:221-236).
#include "rt_scene.hpp"

#include "rt_build.hpp"

using namespace rtdev;
using namespace rthost;

rt_multi_state*& rt_scene_multi(rt_scene* s) { return s->multi; }
int rt_scene_device_of(const rt_scene* s) { return s->device; }
const Tune& rt_scene_tune(const rt_scene* s) { return s->tune; }

int rthost::g_num_cus(int device) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 256;
    return prop.multiProcessorCount;
}

extern "C" {

int32_t rt_api_version(void) { return RT_API_VERSION; }
uint32_t rt_max_frames(void) { return RT_MAX_FRAMES; }

const char* rt_status_str(rt_status s) {
    switch (s) {
        case RT_OK: return "RT_OK";
        case RT_ERR_INVALID_ARG: return "RT_ERR_INVALID_ARG";
        case RT_ERR_SINGULAR_MATRIX: return "RT_ERR_SINGULAR_MATRIX";
        case RT_ERR_UNSUPPORTED: return "RT_ERR_UNSUPPORTED";
        case RT_ERR_NO_DEVICE: return "RT_ERR_NO_DEVICE";
        case RT_ERR_HIP: return "RT_ERR_HIP";
        case RT_ERR_OUT_OF_MEMORY: return "RT_ERR_OUT_OF_MEMORY";
        case RT_ERR_BAD_MATERIAL: return "RT_ERR_BAD_MATERIAL";
        case RT_ERR_CAPACITY: return "RT_ERR_CAPACITY";
        default: return "RT_ERR_UNKNOWN";
    }
}

uint32_t rt_band_rows_per_rank(uint32_t y_res, uint32_t band_rows, uint32_t world) {
    if (band_rows == 0 || world == 0) return 0;
    uint32_t n_bands = (y_res + band_rows - 1) / band_rows;
    uint32_t per_rank = (n_bands + world - 1) / world;
    return per_rank * band_rows;
}

rt_status rt_scene_create(const rt_scene_desc* d, int32_t device, rt_scene** out) {
    return rt_scene_create_tuned(d, device, nullptr, out);
}

rt_status rt_scene_create_tuned(const rt_scene_desc* d, int32_t device, const char* tuning, rt_scene** out) {
    if (!d || !out) return RT_ERR_INVALID_ARG;
    // the handle's tuning: defaults, the environment's RT_TUNE (A/B harness), then `tuning`
    Tune tn;
    if (!tune_apply(tn, std::getenv("RT_TUNE"), true) || !tune_apply(tn, tuning, true)) return RT_ERR_INVALID_ARG;
    return rthost::create_handle(d, device, tn, out);
}
}  // extern "C"

namespace rthost {

rt_status create_handle(const rt_scene_desc* d, int32_t device, const Tune& tn, rt_scene** out) {
    HostScenePtr H;
    rt_status pst = host_scene_build(d, tn, H);
    if (pst != RT_OK) return pst;
    std::unique_ptr<rt_scene> sc(new (std::nothrow) rt_scene());
    if (!sc) return RT_ERR_OUT_OF_MEMORY;
    rt_status st = select_device(device, &sc->device);
    if (st != RT_OK) return st;
    HIP_TRY(hipStreamCreateWithFlags(&sc->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&sc->ev0));
    HIP_TRY(hipEventCreate(&sc->ev1));
    const size_t total = host_scene_bytes(*H);
    HIP_TRY(hipMalloc(&sc->dmem, total));
    sc->dbytes = total;
    // on the scene's own stream, waited for (the host arrays are pageable and go out of
    // scope): the padding zeroed, then each section straight from its array
    HIP_TRY(hipMemsetAsync(sc->dmem, 0, total, sc->stream));
    std::vector<UploadPiece> pieces;
    host_scene_pieces(*H, pieces);
    for (const UploadPiece& p : pieces)
        HIP_TRY(hipMemcpyAsync((uint8_t*)sc->dmem + p.off, p.src, p.bytes, hipMemcpyHostToDevice, sc->stream));
    HIP_TRY(hipStreamSynchronize(sc->stream));
    SceneFacts facts{};
    host_scene_bind(*H, sc->dmem, d, tn, sc->S, facts);
    sc->flops_per_scan = facts.flops_per_scan;
    sc->n_point_lights = facts.n_point_lights;
    sc->normal_max = facts.normal_max;
    sc->num_cus = g_num_cus(sc->device);
    sc->tune = tn;
    sc->d_mats.assign(d->materials, d->materials + d->n_materials);
    sc->d_shapes.assign(d->shapes, d->shapes + d->n_shapes);
    sc->d_lights.assign(d->lights, d->lights + d->n_lights);
    sc->d_ambient = d->ambient;
    *out = sc.release();
    return RT_OK;
}

namespace {

// rt_scene_update's rebuild, in two steps so that a failure leaves every handle as it was:
// stage_scene_data waits for dst's renders and copies src's device scene into a new
// allocation on dst's device; commit_scene_data then swaps it in (rebased DevScene, the
// description, the light count's workspace consequences).
rt_status stage_scene_data(rt_scene* dst, const rt_scene* src, void** out) {
    *out = nullptr;
    HIP_TRY(hipSetDevice(dst->device));
    HIP_TRY(hipStreamSynchronize(dst->stream));
    for (auto& se : dst->ev_streams) HIP_TRY(hipEventSynchronize(se.second));  // renders on other streams
    void* mem = nullptr;
    HIP_TRY(hipMalloc(&mem, src->dbytes));
    rt_status st = RT_OK;
    if (dst->device == src->device)
        st = hip_status(hipMemcpyAsync(mem, src->dmem, src->dbytes, hipMemcpyDeviceToDevice, dst->stream));
    else
        st = hip_status(hipMemcpyPeerAsync(mem, dst->device, src->dmem, src->device, src->dbytes, dst->stream));
    if (st == RT_OK) st = hip_status(hipStreamSynchronize(dst->stream));
    if (st != RT_OK) {
        (void)hipFree(mem);
        return st;
    }
    *out = mem;
    return RT_OK;
}

void commit_scene_data(rt_scene* dst, const rt_scene* src, void* mem) {
    (void)hipSetDevice(dst->device);
    // a different light count changes the shadow queue's size and the node-index limit
    const bool new_lights = dst->n_point_lights != src->n_point_lights || dst->S.n_lights != src->S.n_lights;
    if (dst->dmem) (void)hipFree(dst->dmem);
    dst->dmem = mem;
    dst->dbytes = src->dbytes;
    dst->S = src->S;
    const uint8_t* from = (const uint8_t*)src->dmem;
    uint8_t* to = (uint8_t*)dst->dmem;
    auto rebase = [&](auto& ptr) {
        if (ptr) ptr = reinterpret_cast<std::remove_reference_t<decltype(ptr)>>(to + ((const uint8_t*)ptr - from));
    };
    DevScene& S = dst->S;
    rebase(S.dsph); rebase(S.gsph); rebase(S.tri); rebase(S.cube); rebase(S.plane); rebase(S.cubetri);
    rebase(S.shapes); rebase(S.mats); rebase(S.lights); rebase(S.bvh_nodes); rebase(S.bvh_leaves);
    rebase(S.graze_blk); rebase(S.graze_tri); rebase(S.graze_pn); rebase(S.graze_mask); rebase(S.scan_ops);
    dst->flops_per_scan = src->flops_per_scan;
    dst->normal_max = src->normal_max;
    dst->n_point_lights = src->n_point_lights;
    dst->d_mats = src->d_mats;
    dst->d_shapes = src->d_shapes;
    dst->d_lights = src->d_lights;
    dst->d_ambient = src->d_ambient;
    // deeper ray trees may need a larger pool than any pass checked so far: check again
    dst->checked_items = 0;
    dst->checked_depth = 0;
    // the kernels' LDS staging depends on the scene (node records, grazing normals, sphere
    // pairs): the persistent grids are sized from the occupancy measured again
    dst->occ_trace = 0;
    dst->generation++;
    if (new_lights) free_workspace(dst->ws);
}

}  // namespace
}  // namespace rthost

extern "C" {

rt_status rt_scene_destroy(rt_scene* s) {
    if (!s) return RT_ERR_INVALID_ARG;
    if (s->multi) rt_multi_free(s->multi);
    s->multi = nullptr;
    if (s->split) rt_multi_free(s->split);
    s->split = nullptr;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    for (auto& se : s->ev_streams) (void)hipEventSynchronize(se.second);  // renders on other streams
    free_workspace(s->ws);
    if (s->dmem) (void)hipFree(s->dmem);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    for (auto& se : s->ev_streams) (void)hipEventDestroy(se.second);
    for (hipEvent_t e : s->kt_events) (void)hipEventDestroy(e);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return RT_OK;
}

rt_status rt_host_alloc(uint64_t bytes, void** out) {
    if (!out || bytes == 0) return RT_ERR_INVALID_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return RT_ERR_NO_DEVICE;
    HIP_TRY(hipHostMalloc(out, bytes, hipHostMallocPortable));
    return RT_OK;
}

rt_status rt_host_free(void* ptr) {
    if (!ptr) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipHostFree(ptr));
    return RT_OK;
}

uint64_t rt_scene_flops_per_scan(const rt_scene* s) { return s ? s->flops_per_scan : 0; }

uint64_t rt_scene_workspace_bytes(const rt_scene* s) {
    if (!s) return 0;
    const Workspace& w = s->ws;
    uint64_t b = (uint64_t)w.out_floats * 4 + w.out8_bytes + 4 * 8 + 64;
    b += (uint64_t)w.capacity * (sizeof(Task) + 4 + 3 * 16 + 4 * w.lit_words + 2 * 16);  // tasks, node arrays
    if (w.forest) b += (uint64_t)w.capacity * (2 * 16 + 4 + 4);
    b += (uint64_t)w.sort_capacity * 8;                                      // task keys, permutation
    b += (uint64_t)w.shadow_capacity * (w.shadow_light ? 8 : 4) + (uint64_t)w.sort_shadow_capacity * 8;
    b += (uint64_t)w.sort_tmp_words * 4;
    b += (uint64_t)w.spp_buf_floats * 4;
    if (w.levels) b += RT_LEVEL_TABLE_WORDS * 4 + 64;
    return b;
}
uint64_t rt_scene_device_bytes(const rt_scene* s) { return s ? (uint64_t)s->dbytes : 0; }

rt_status rt_scene_scan_ops(rt_scene* s, uint64_t* out, uint32_t n, int32_t reset) {
    if (!s || (out && n > RT_SCAN_OPS_N)) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipDeviceSynchronize());
    if (out && n) {
        std::vector<unsigned long long> h(RT_OPS_SLOTS * RT_OPS_STRIDE);
        HIP_TRY(hipMemcpy(h.data(), s->S.scan_ops, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        for (uint32_t k = 0; k < n; k++) {
            out[k] = 0;
            for (int b = 0; b < RT_OPS_SLOTS; b++) out[k] += h[b * RT_OPS_STRIDE + k];
        }
    }
    if (reset) {
        HIP_TRY(hipMemset(s->S.scan_ops, 0, RT_OPS_SLOTS * RT_OPS_STRIDE * sizeof(unsigned long long)));
        HIP_TRY(hipDeviceSynchronize());
    }
    return RT_OK;
}

int32_t rt_scene_uses_bvh(const rt_scene* s) { return (s && s->S.use_bvh) ? 1 : 0; }

rt_status rt_scene_set_grid_share(rt_scene* s, int32_t percent) {
    if (!s || percent < 1 || percent > 100) return RT_ERR_INVALID_ARG;
    if (s->multi) (void)rt_multi_each(s->multi, [&](rt_scene* c) { return rt_scene_set_grid_share(c, percent); });
    if (s->split) (void)rt_multi_each(s->split, [&](rt_scene* c) { return rt_scene_set_grid_share(c, percent); });
    s->grid_pct = percent;
    return RT_OK;
}

rt_status rt_scene_set_tuning(rt_scene* s, const char* tuning) {
    if (!s) return RT_ERR_INVALID_ARG;
    Tune t = s->tune;
    if (!tune_apply(t, tuning, false)) return RT_ERR_INVALID_ARG;
    auto set = [&](rt_scene* c) {  // clones share the scene-build keys
        c->tune = t;
        c->occ_trace = 0;  // the kernels' LDS may differ: occupancy measured again
        return RT_OK;
    };
    (void)set(s);
    if (s->multi) (void)rt_multi_each(s->multi, set);
    if (s->split) (void)rt_multi_each(s->split, set);
    return RT_OK;
}

rt_status rt_scene_set_scan_counting(rt_scene* s, int32_t enable) {
    if (!s) return RT_ERR_INVALID_ARG;
    if (s->multi) (void)rt_multi_each(s->multi, [&](rt_scene* c) { return rt_scene_set_scan_counting(c, enable); });
    if (s->split) (void)rt_multi_each(s->split, [&](rt_scene* c) { return rt_scene_set_scan_counting(c, enable); });
    s->count_ops = enable != 0;
    return RT_OK;
}

rt_status rt_scene_set_kernel_timing(rt_scene* s, int32_t enable) {
    if (!s) return RT_ERR_INVALID_ARG;
    s->ktime = enable != 0;
    return RT_OK;
}

rt_status rt_scene_kernel_times(rt_scene* s, float* ms, uint32_t n, int32_t reset) {
    if (!s || (n && !ms)) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(s->device));
    for (uint32_t k = 0; k < n; k++) ms[k] = 0.f;
    for (const auto& sp : s->kt_spans) {
        HIP_TRY(hipEventSynchronize(s->kt_events[sp.second + 1]));
        float t = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, s->kt_events[sp.second], s->kt_events[sp.second + 1]));
        if ((uint32_t)sp.first < n) ms[sp.first] += t;
    }
    if (n > RT_KT_LAUNCHES) ms[RT_KT_LAUNCHES] = (float)s->kt_spans.size();
    if (reset) {
        s->kt_spans.clear();
        s->kt_used = 0;
    }
    return RT_OK;
}

rt_status rt_scene_clone(const rt_scene* src, int32_t device, rt_scene** out) {
    if (!src || !out) return RT_ERR_INVALID_ARG;
    std::unique_ptr<rt_scene> sc(new (std::nothrow) rt_scene());
    if (!sc) return RT_ERR_OUT_OF_MEMORY;
    rt_status st = select_device(device, &sc->device);
    if (st != RT_OK) return st;
    HIP_TRY(hipStreamCreateWithFlags(&sc->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&sc->ev0));
    HIP_TRY(hipEventCreate(&sc->ev1));
    HIP_TRY(hipMalloc(&sc->dmem, src->dbytes));
    sc->dbytes = src->dbytes;
    // on the clone's own stream and waited for: a render on any caller stream sees the copy
    if (sc->device == src->device)
        HIP_TRY(hipMemcpyAsync(sc->dmem, src->dmem, src->dbytes, hipMemcpyDeviceToDevice, sc->stream));
    else
        HIP_TRY(hipMemcpyPeerAsync(sc->dmem, sc->device, src->dmem, src->device, src->dbytes, sc->stream));
    HIP_TRY(hipMemsetAsync((uint8_t*)sc->dmem + ((const uint8_t*)src->S.scan_ops - (const uint8_t*)src->dmem), 0,
                           RT_OPS_SLOTS * RT_OPS_STRIDE * sizeof(unsigned long long), sc->stream));
    HIP_TRY(hipStreamSynchronize(sc->stream));
    // the same DevScene, every pointer rebased into the new allocation
    sc->S = src->S;
    const uint8_t* from = (const uint8_t*)src->dmem;
    uint8_t* to = (uint8_t*)sc->dmem;
    auto rebase = [&](auto& ptr) {
        if (ptr) ptr = reinterpret_cast<std::remove_reference_t<decltype(ptr)>>(to + ((const uint8_t*)ptr - from));
    };
    DevScene& S = sc->S;
    rebase(S.dsph); rebase(S.gsph); rebase(S.tri); rebase(S.cube); rebase(S.plane); rebase(S.cubetri);
    rebase(S.shapes); rebase(S.mats); rebase(S.lights); rebase(S.bvh_nodes); rebase(S.bvh_leaves);
    rebase(S.graze_blk); rebase(S.graze_tri); rebase(S.graze_pn); rebase(S.graze_mask); rebase(S.scan_ops);
    sc->flops_per_scan = src->flops_per_scan;
    sc->normal_max = src->normal_max;
    sc->n_point_lights = src->n_point_lights;
    sc->num_cus = g_num_cus(sc->device);
    sc->count_ops = src->count_ops;
    sc->tune = src->tune;
    sc->d_mats = src->d_mats;
    sc->d_shapes = src->d_shapes;
    sc->d_lights = src->d_lights;
    sc->d_ambient = src->d_ambient;
    *out = sc.release();
    return RT_OK;
}

rt_status rt_scene_set_material(rt_scene* s, uint32_t index, const rt_material* m) {
    if (!s || !m || index >= (uint32_t)s->S.n_mats) return RT_ERR_INVALID_ARG;
    MatRec cur;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    for (auto& se : s->ev_streams) HIP_TRY(hipEventSynchronize(se.second));  // renders on other streams
    HIP_TRY(hipMemcpyAsync(&cur, s->S.mats + index, sizeof(cur), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (m->kind != cur.kind) return RT_ERR_INVALID_ARG;  // the same kind, as the GUI's edits
    MatRec M;
    rt_status r = material_record(*m, M, s->normal_max);
    if (r != RT_OK) return r;
    // on the handle's stream, waited for: the next render on any caller stream sees the edit
    HIP_TRY(hipMemcpyAsync(const_cast<MatRec*>(s->S.mats) + index, &M, sizeof(M), hipMemcpyHostToDevice, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    // the handle's own copy is written first: rt_scene_update compares against it, so an edit
    // that reached this device must be recorded even if a band share or device below fails
    s->d_mats[index] = *m;
    if (s->split) {
        rt_status e = rt_multi_each(s->split, [&](rt_scene* c) { return rt_scene_set_material(c, index, m); });
        if (e != RT_OK) return e;
    }
    if (s->multi) {
        rt_status e = rt_multi_each(s->multi, [&](rt_scene* c) { return rt_scene_set_material(c, index, m); });
        if (e != RT_OK) return e;
    }
    return RT_OK;
}

rt_status rt_scene_update(rt_scene* s, const rt_scene_desc* d, int32_t* what) {
    if (what) *what = 0;
    if (!s || !d) return RT_ERR_INVALID_ARG;
    if ((d->n_materials && !d->materials) || (d->n_shapes && !d->shapes) || (d->n_lights && !d->lights))
        return RT_ERR_INVALID_ARG;
    auto same = [](const void* a, const void* b, size_t n) { return n == 0 || std::memcmp(a, b, n) == 0; };
    const bool geometry = d->n_shapes == s->d_shapes.size() && d->n_lights == s->d_lights.size() &&
                          d->n_materials == s->d_mats.size() &&
                          same(d->shapes, s->d_shapes.data(), d->n_shapes * sizeof(rt_shape)) &&
                          same(d->lights, s->d_lights.data(), d->n_lights * sizeof(rt_light)) &&
                          same(&d->ambient, &s->d_ambient, sizeof(rt_color));
    std::vector<uint32_t> edits;
    bool kinds = true;
    if (geometry) {
        for (uint32_t i = 0; i < d->n_materials; i++)
            if (!same(&d->materials[i], &s->d_mats[i], sizeof(rt_material))) {
                edits.push_back(i);
                kinds = kinds && d->materials[i].kind == s->d_mats[i].kind;
            }
        if (edits.empty()) return RT_OK;
    }
    // a stream-ordered render's unreported status is returned first (the update is then not
    // made), on every path that changes the scene
    rt_status st = rt_scene_sync_status(s);
    if (st != RT_OK) return st;
    if (s->multi) {
        st = rt_multi_each(s->multi, [](rt_scene* c) { return rt_scene_sync_status(c); });
        if (st != RT_OK) return st;
    }
    if (geometry && kinds) {
        // material edits of the same kind (the GUI's sliders, gui.rs:221-236) in place; every
        // edited material is validated before the first is applied (no partial update)
        for (uint32_t i : edits) {
            MatRec M;
            st = material_record(d->materials[i], M, s->normal_max);
            if (st != RT_OK) return st;
        }
        for (uint32_t i : edits) {
            st = rt_scene_set_material(s, i, &d->materials[i]);
            if (st != RT_OK) return st;
        }
        if (what) *what = 1;
        return RT_OK;
    }
    // anything else: the scene is rebuilt (same device and tuning) and adopted in place, so the
    // caller's handle, its stream, workspace and band shares stay valid
    rt_scene* fresh = nullptr;
    st = create_handle(d, s->device, s->tune, &fresh);
    if (st != RT_OK) return st;
    // every copy of the scene the handle renders with: its own, its band shares', its devices'
    std::vector<rt_scene*> targets{s};
    auto collect = [&](rt_scene* c) {
        targets.push_back(c);
        return RT_OK;
    };
    if (s->split) (void)rt_multi_each(s->split, collect);
    if (s->multi) (void)rt_multi_each(s->multi, collect);
    std::vector<void*> staged(targets.size(), nullptr);
    for (size_t i = 0; i < targets.size() && st == RT_OK; i++) st = stage_scene_data(targets[i], fresh, &staged[i]);
    if (st == RT_OK)
        for (size_t i = 0; i < targets.size(); i++) commit_scene_data(targets[i], fresh, staged[i]);
    else
        for (size_t i = 0; i < targets.size(); i++)
            if (staged[i]) {
                (void)hipSetDevice(targets[i]->device);
                (void)hipFree(staged[i]);
            }
    rt_scene_destroy(fresh);
    (void)hipSetDevice(s->device);
    if (st != RT_OK) return st;
    if (what) *what = 2;
    return RT_OK;
}

}  // extern "C"
