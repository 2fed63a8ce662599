// rt_multi.cpp -- the multi-GPU render inside the C ABI.
//
// The reference renders one frame on one core (src/render.rs:31-38); its pixels are
// independent, so a frame tiles across devices with a single exchange step.  A scene made
// by rt_scene_create_multi(desc, devices, n) is built once on the host, uploaded to
// devices[0] and cloned device-to-device to the others (rt_scene_clone: one workspace and
// stream per device).  rt_render / rt_render_spp on it, from ONE host thread:
//
//   rank r (device devices[r]):  rows dealt in block-cyclic bands of 8 (band b -> rank
//                                b % n), rendered into the rank's band buffer
//                                (rt_render_bands_ex_async, f32 + optional fused RGB8)
//   exchange:                    ncclGather of every band buffer to rank 0 (RCCL over xGMI;
//                                one communicator per device from ncclCommInitAll, all
//                                gathers in one ncclGroupStart / ncclGroupEnd)
//   rank 0:                      un-permute kernel -> row-major frame -> caller's buffers
//
// RCCL is loaded at rt_scene_create_multi time (dlopen of librccl.so.1): a process that
// already holds PyTorch's RCCL (same soname) shares it, and single-device use never loads
// it.  A device listed more than once shares one GPU between band shares; RCCL cannot put
// two ranks on one device, so such a scene exchanges bands with device copies instead (a
// test configuration: it runs the multi-device band logic on a one-GPU machine).
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_internal.hpp"

namespace {

#define MHIP(x)                                                                                      \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            std::fprintf(stderr, "rt_multi.cpp:%d: %s: %s\n", __LINE__, #x, hipGetErrorString(e_)); \
            return e_ == hipErrorOutOfMemory ? RT_ERR_OUT_OF_MEMORY : RT_ERR_HIP;                    \
        }                                                                                            \
    } while (0)

struct Rccl {
    void* h = nullptr;
    ncclResult_t (*init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

bool load_rccl(Rccl& r) {
    r.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!r.h) r.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!r.h) return false;
    r.init_all = (decltype(r.init_all))dlsym(r.h, "ncclCommInitAll");
    r.gather = (decltype(r.gather))dlsym(r.h, "ncclGather");
    r.group_start = (decltype(r.group_start))dlsym(r.h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(r.h, "ncclGroupEnd");
    r.destroy = (decltype(r.destroy))dlsym(r.h, "ncclCommDestroy");
    r.error_string = (decltype(r.error_string))dlsym(r.h, "ncclGetErrorString");
    return r.init_all && r.gather && r.group_start && r.group_end && r.destroy && r.error_string;
}

}  // namespace

struct rt_multi_state {
    std::vector<int> devices;
    std::vector<rt_scene*> ranks;            // ranks[0] = the primary handle (not owned here)
    std::vector<hipStream_t> streams;        // one per rank, on its device
    std::vector<hipEvent_t> done;            // per rank: its band is rendered (copy exchange)
    std::vector<hipEvent_t> copied;          // per rank: its band is in the caller's buffers (direct copy-out)
    hipEvent_t ev0 = nullptr, ev1 = nullptr; // device 0: the render's span
    std::vector<float*> band;                // per rank: rows_per_rank x x_res x 3 floats
    std::vector<uint8_t*> band8;             // per rank: ... bytes (when RGB8 is asked for)
    std::vector<unsigned long long*> counters;  // per rank: node, shadow, pixel rays
    size_t band_floats = 0;
    bool have8 = false;
    float* gathered = nullptr;               // device 0: world band buffers, rank-major
    uint8_t* gathered8 = nullptr;
    float* frame = nullptr;                  // device 0: the row-major frame
    uint8_t* frame8 = nullptr;
    size_t frame_floats = 0;
    bool rccl = false;
    Rccl lib;
    std::vector<ncclComm_t> comms;
    uint32_t band_rows = 8;                  // rows per band (block-cyclic over the ranks)
    bool direct = false;                     // the last render copied each rank's one band straight out
    bool frame_async = false;                // rt_multi_render_frame_async ran (done[0] marks its share 0)
};

rt_status rt_multi_each(rt_multi_state* m, const std::function<rt_status(rt_scene*)>& f) {
    for (size_t r = 1; r < m->ranks.size(); r++) {
        rt_status st = f(m->ranks[r]);
        if (st != RT_OK) return st;
    }
    return RT_OK;
}

static void free_buffers(rt_multi_state* m) {
    for (size_t r = 0; r < m->band.size(); r++) {
        (void)hipSetDevice(m->devices[r]);
        if (m->band[r]) (void)hipFree(m->band[r]);
        if (m->band8[r]) (void)hipFree(m->band8[r]);
        m->band[r] = nullptr;
        m->band8[r] = nullptr;
    }
    (void)hipSetDevice(m->devices[0]);
    for (void* b : {(void*)m->gathered, (void*)m->gathered8, (void*)m->frame, (void*)m->frame8})
        if (b) (void)hipFree(b);
    m->gathered = m->frame = nullptr;
    m->gathered8 = m->frame8 = nullptr;
    m->band_floats = m->frame_floats = 0;
    m->have8 = false;
}

void rt_multi_free(rt_multi_state* m) {
    if (!m) return;
    for (size_t r = 0; r < m->streams.size(); r++) {
        (void)hipSetDevice(m->devices[r]);
        if (m->streams[r]) (void)hipStreamSynchronize(m->streams[r]);
    }
    free_buffers(m);
    for (size_t r = 0; r < m->ranks.size(); r++) {
        (void)hipSetDevice(m->devices[r]);
        if (r < m->counters.size() && m->counters[r]) (void)hipFree(m->counters[r]);
        if (r < m->done.size() && m->done[r]) (void)hipEventDestroy(m->done[r]);
        if (r < m->copied.size() && m->copied[r]) (void)hipEventDestroy(m->copied[r]);
        if (r < m->streams.size() && m->streams[r]) (void)hipStreamDestroy(m->streams[r]);
        if (r > 0 && m->ranks[r]) (void)rt_scene_destroy(m->ranks[r]);
    }
    for (ncclComm_t c : m->comms)
        if (c) (void)m->lib.destroy(c);
    (void)hipSetDevice(m->devices[0]);
    if (m->ev0) (void)hipEventDestroy(m->ev0);
    if (m->ev1) (void)hipEventDestroy(m->ev1);
    delete m;  // the RCCL library stays loaded (another communicator may use it)
}

// frame_floats == 0: band buffers only (the direct copy-out needs no gather / frame buffers)
static rt_status ensure_buffers(rt_multi_state* m, size_t band_floats, size_t frame_floats, bool want8) {
    if (band_floats <= m->band_floats && frame_floats <= m->frame_floats && (!want8 || m->have8)) return RT_OK;
    free_buffers(m);
    const size_t world = m->ranks.size();
    for (size_t r = 0; r < world; r++) {
        MHIP(hipSetDevice(m->devices[r]));
        MHIP(hipMalloc(&m->band[r], band_floats * sizeof(float)));
        if (want8) MHIP(hipMalloc(&m->band8[r], band_floats));
    }
    MHIP(hipSetDevice(m->devices[0]));
    if (frame_floats) {
        MHIP(hipMalloc(&m->gathered, world * band_floats * sizeof(float)));
        MHIP(hipMalloc(&m->frame, frame_floats * sizeof(float)));
        if (want8) {
            MHIP(hipMalloc(&m->gathered8, world * band_floats));
            MHIP(hipMalloc(&m->frame8, frame_floats));
        }
    }
    m->band_floats = band_floats;
    m->frame_floats = frame_floats;
    m->have8 = want8;
    return RT_OK;
}

static rt_status multi_finish(rt_multi_state* m, const rt_render_opts* opts);

rt_status rt_multi_share_ms(rt_multi_state* m, float* ms, uint32_t n) {
    if (!m || !ms || n > m->ranks.size() || m->rccl || !m->direct) return RT_ERR_UNSUPPORTED;
    if (hipSetDevice(m->devices[0]) != hipSuccess) return RT_ERR_HIP;
    for (uint32_t r = 0; r < n; r++)
        if (hipEventElapsedTime(&ms[r], m->ev0, m->done[r]) != hipSuccess) return RT_ERR_HIP;
    return RT_OK;
}

rt_status rt_multi_copy_ms(rt_multi_state* m, float* ms, uint32_t n) {
    if (!m || !ms || n > m->ranks.size() || m->rccl || !m->direct) return RT_ERR_UNSUPPORTED;
    if (hipSetDevice(m->devices[0]) != hipSuccess) return RT_ERR_HIP;
    for (uint32_t r = 0; r < n; r++)
        if (hipEventElapsedTime(&ms[r], m->done[r], m->copied[r]) != hipSuccess) return RT_ERR_HIP;
    return RT_OK;
}

rt_status rt_multi_render(rt_scene* s, const rt_camera* cam, uint32_t depth, uint32_t spp, uint32_t seed,
                          const rt_render_opts* opts, float* rgb, uint8_t* rgb8) {
    return rt_multi_render_state(rt_scene_multi(s), cam, depth, spp, seed, opts, rgb, rgb8);
}

rt_status rt_multi_render_state(rt_multi_state* m, const rt_camera* cam, uint32_t depth, uint32_t spp, uint32_t seed,
                                const rt_render_opts* opts, float* rgb, uint8_t* rgb8) {
    if (!cam || cam->x_res == 0 || cam->y_res == 0) return RT_ERR_INVALID_ARG;
    const uint32_t world = (uint32_t)m->ranks.size(), band_rows = m->band_rows;
    const uint32_t rpr = rt_band_rows_per_rank(cam->y_res, band_rows, world);
    const size_t bf = (size_t)rpr * cam->x_res * 3u, ff = (size_t)cam->y_res * cam->x_res * 3u;
    // one band per rank on one device's copy exchange: each band goes straight to the caller
    // (below); its buffers are sized for a whole frame once, so a moving meeting row never
    // reallocates them
    const bool direct = !m->rccl && band_rows >= rpr;
    rt_status st = direct ? ensure_buffers(m, ff, 0, rgb8 != nullptr) : ensure_buffers(m, bf, ff, rgb8 != nullptr);
    if (st != RT_OK) return st;
    hipStream_t s0 = m->streams[0];
    std::vector<char> redo(world, 1);  // ranks whose bands (re-)render in this attempt
    MHIP(hipSetDevice(m->devices[0]));
    MHIP(hipEventRecord(m->ev0, s0));
    m->direct = direct;
    if (direct) {
        // Every rank holds ONE band: rows [r band_rows, (r + 1) band_rows) of the frame, row
        // major -- its band buffer is already that slice of the frame.  No gather and no
        // un-permute: each rank's slice goes from its own stream straight to the caller's
        // buffers, so the first share's copy runs while the other shares still render
        // (rt_render's seam split on one device).
        for (int attempt = 0;; attempt++) {
            for (uint32_t r = 0; r < world; r++) {
                if (!redo[r]) continue;
                MHIP(hipSetDevice(m->devices[r]));
                MHIP(hipMemsetAsync(m->counters[r], 0, 3 * sizeof(unsigned long long), m->streams[r]));
                st = rt_render_bands_ex_async(m->ranks[r], cam, 1, depth, spp, seed, band_rows, r, world, m->band[r],
                                              rgb8 ? m->band8[r] : nullptr, (uint64_t*)m->counters[r], m->streams[r]);
                if (st != RT_OK) return st;
                MHIP(hipEventRecord(m->done[r], m->streams[r]));
            }
            // the render's span on device 0's clock: from ev0 to the last share's end
            MHIP(hipSetDevice(m->devices[0]));
            for (uint32_t r = 0; r < world; r++) MHIP(hipStreamWaitEvent(s0, m->done[r], 0));
            MHIP(hipEventRecord(m->ev1, s0));
            // every render is enqueued before the first copy: a copy into pageable memory
            // may hold this thread until it is done
            for (uint32_t r = 0; r < world; r++) {
                if (!redo[r]) continue;
                const uint32_t y0 = r * band_rows;
                const uint32_t rows = y0 < cam->y_res ? std::min(band_rows, cam->y_res - y0) : 0u;
                const size_t off = (size_t)y0 * cam->x_res * 3u, len = (size_t)rows * cam->x_res * 3u;
                if (!len) continue;
                MHIP(hipSetDevice(m->devices[r]));
                MHIP(hipMemcpyAsync(rgb + off, m->band[r], len * sizeof(float), hipMemcpyDeviceToHost, m->streams[r]));
                if (rgb8)
                    MHIP(hipMemcpyAsync(rgb8 + off, m->band8[r], len, hipMemcpyDeviceToHost, m->streams[r]));
                MHIP(hipEventRecord(m->copied[r], m->streams[r]));
            }
            for (uint32_t r = 0; r < world; r++) {
                MHIP(hipSetDevice(m->devices[r]));
                MHIP(hipStreamSynchronize(m->streams[r]));
            }
            // a rank whose queues overflowed renders (and copies) its slice again with a
            // grown pool; the other slices are final
            bool overflow = false;
            for (uint32_t r = 0; r < world; r++) {
                st = rt_scene_sync_own(m->ranks[r]);
                redo[r] = st == RT_ERR_CAPACITY;
                if (redo[r])
                    overflow = true;
                else if (st != RT_OK)
                    return st;
            }
            if (!overflow) break;
            if (attempt >= 8) return RT_ERR_CAPACITY;
        }
        return multi_finish(m, opts);
    }
    for (int attempt = 0;; attempt++) {
        for (uint32_t r = 0; r < world; r++) {
            if (!redo[r]) continue;
            MHIP(hipSetDevice(m->devices[r]));
            MHIP(hipMemsetAsync(m->counters[r], 0, 3 * sizeof(unsigned long long), m->streams[r]));
            st = rt_render_bands_ex_async(m->ranks[r], cam, 1, depth, spp, seed, band_rows, r, world, m->band[r],
                                          rgb8 ? m->band8[r] : nullptr, (uint64_t*)m->counters[r], m->streams[r]);
            if (st != RT_OK) return st;
        }
        // the one exchange step: every band buffer to rank 0
        if (m->rccl) {
            if (m->lib.group_start() != ncclSuccess) return RT_ERR_HIP;
            for (uint32_t r = 0; r < world; r++) {
                ncclResult_t e = m->lib.gather(m->band[r], r == 0 ? m->gathered : nullptr, bf, ncclFloat32, 0,
                                               m->comms[r], m->streams[r]);
                if (e == ncclSuccess && rgb8)
                    e = m->lib.gather(m->band8[r], r == 0 ? m->gathered8 : nullptr, bf, ncclUint8, 0, m->comms[r],
                                      m->streams[r]);
                if (e != ncclSuccess) {
                    std::fprintf(stderr, "rt_multi.cpp: ncclGather: %s\n", m->lib.error_string(e));
                    (void)m->lib.group_end();
                    return RT_ERR_HIP;
                }
            }
            ncclResult_t e = m->lib.group_end();
            if (e != ncclSuccess) {
                std::fprintf(stderr, "rt_multi.cpp: ncclGroupEnd: %s\n", m->lib.error_string(e));
                return RT_ERR_HIP;
            }
        } else {  // every rank on one device: device copies
            for (uint32_t r = 0; r < world; r++) {
                MHIP(hipSetDevice(m->devices[r]));
                MHIP(hipEventRecord(m->done[r], m->streams[r]));
            }
            MHIP(hipSetDevice(m->devices[0]));
            for (uint32_t r = 0; r < world; r++) {
                MHIP(hipStreamWaitEvent(s0, m->done[r], 0));
                MHIP(hipMemcpyAsync(m->gathered + r * bf, m->band[r], bf * sizeof(float), hipMemcpyDeviceToDevice,
                                    s0));
                if (rgb8)
                    MHIP(hipMemcpyAsync(m->gathered8 + r * bf, m->band8[r], bf, hipMemcpyDeviceToDevice, s0));
            }
        }
        MHIP(hipSetDevice(m->devices[0]));
        st = rt_unpermute_bands_async(m->gathered, cam->x_res, cam->y_res, band_rows, world, m->frame, s0);
        if (st != RT_OK) return st;
        if (rgb8) {
            st = rt_unpermute_bands_u8_async(m->gathered8, cam->x_res, cam->y_res, band_rows, world, m->frame8, s0);
            if (st != RT_OK) return st;
        }
        MHIP(hipEventRecord(m->ev1, s0));
        MHIP(hipStreamSynchronize(s0));
        // only a rank whose ray queues overflowed renders its bands again, with a grown pool
        // (rt_scene_sync_status); every other rank's band buffer is still valid, and the
        // exchange (a collective: every rank takes part) runs once more
        bool overflow = false;
        for (uint32_t r = 0; r < world; r++) {
            st = rt_scene_sync_own(m->ranks[r]);
            redo[r] = st == RT_ERR_CAPACITY;
            if (redo[r])
                overflow = true;
            else if (st != RT_OK)
                return st;
        }
        if (!overflow) break;
        if (attempt >= 8) return RT_ERR_CAPACITY;
    }
    MHIP(hipSetDevice(m->devices[0]));
    MHIP(hipMemcpyAsync(rgb, m->frame, ff * sizeof(float), hipMemcpyDeviceToHost, s0));
    if (rgb8) MHIP(hipMemcpyAsync(rgb8, m->frame8, ff, hipMemcpyDeviceToHost, s0));
    MHIP(hipStreamSynchronize(s0));
    return multi_finish(m, opts);
}

// rt_render_frame_async: the seam split, stream-ordered.  Two band shares of one device
// (ranks[0], ranks[1]: rows [0, rows) and [rows, y_res)) fork from `stream`, render side by
// side on their own streams and join back into it.  Share 0's band buffer IS the top of the
// caller's frame (one band of `rows` rows, no padding: rows < y_res), so it renders straight
// into d_rgb; share 1's last band is padded past y_res, so it renders into its own buffer and
// one device copy moves its valid rows into place.  Counters of both shares add into
// d_counters.  Nothing here waits on the host; the last call's share spans (ev0 -> done[r])
// are read by the next call through rt_multi_async_share_ms once they have completed.
rt_status rt_multi_render_frame_async(rt_multi_state* m, const rt_camera* cam, uint32_t depth, uint32_t rows,
                                      float* d_rgb, uint8_t* d_rgb8, uint64_t* d_counters, hipStream_t stream) {
    if (!m || m->rccl || m->ranks.size() != 2 || !cam || !d_rgb || rows == 0 || rows >= cam->y_res ||
        2ull * rows < cam->y_res)
        return RT_ERR_INVALID_ARG;
    const uint32_t world = 2;
    const size_t row_floats = (size_t)cam->x_res * 3u;
    const size_t ff = (size_t)cam->y_res * row_floats;
    rt_status st = ensure_buffers(m, ff, 0, d_rgb8 != nullptr);
    if (st != RT_OK) return st;
    m->band_rows = rows;
    m->direct = true;
    MHIP(hipSetDevice(m->devices[0]));
    // Both shares fork onto the state's streams (share r always on streams[r], so calls from
    // any caller streams stay ordered on each share's workspace).  Tune::frame_fork=caller (A/B):
    // share 0 on the caller's stream itself, only share 1 forked -- 3.41 / 3.40 ms vs 3.52 /
    // 3.85, config 3 at 1080p on a created caller stream.  On the legacy null stream the fork
    // and join measured 5.3 - 5.4 ms once other streams and rt_render's shares existed in the
    // process: pass a created stream.
    const bool on_caller = rt_scene_tune(m->ranks[0]).frame_fork == 1;
    // share 0 renders on rank 0's workspace: after the previous call's share 0, whatever
    // stream that call came from (share 1 is ordered by the state's own stream)
    if (on_caller && m->frame_async) MHIP(hipStreamWaitEvent(stream, m->done[0], 0));
    m->frame_async = true;
    MHIP(hipEventRecord(m->ev0, stream));
    for (uint32_t r = 0; r < world; r++) {
        hipStream_t rs = (r == 0 && on_caller) ? stream : m->streams[r];
        if (rs != stream) MHIP(hipStreamWaitEvent(rs, m->ev0, 0));
        float* out = r == 0 ? d_rgb : m->band[r];
        uint8_t* out8 = d_rgb8 ? (r == 0 ? d_rgb8 : m->band8[r]) : nullptr;
        st = rt_render_bands_ex_async(m->ranks[r], cam, 1, depth, 1, 0, rows, r, world, out, out8, d_counters, rs);
        if (st != RT_OK) return st;
        MHIP(hipEventRecord(m->done[r], rs));
        if (r > 0) {
            const size_t off = (size_t)rows * row_floats, len = (size_t)(cam->y_res - rows) * row_floats;
            MHIP(hipMemcpyAsync(d_rgb + off, m->band[r], len * sizeof(float), hipMemcpyDeviceToDevice, rs));
            if (d_rgb8) MHIP(hipMemcpyAsync(d_rgb8 + off, m->band8[r], len, hipMemcpyDeviceToDevice, rs));
        }
        if (rs != stream) {
            MHIP(hipEventRecord(m->copied[r], rs));
            MHIP(hipStreamWaitEvent(stream, m->copied[r], 0));
        }
    }
    return RT_OK;
}

// The previous rt_multi_render_frame_async's share spans (ms from the fork to each share's
// end), if they have completed; RT_ERR_UNSUPPORTED otherwise.  Never waits.
rt_status rt_multi_async_share_ms(rt_multi_state* m, float* ms, uint32_t n) {
    if (!m || !ms || n > m->ranks.size() || m->rccl || !m->direct) return RT_ERR_UNSUPPORTED;
    if (hipSetDevice(m->devices[0]) != hipSuccess) return RT_ERR_HIP;
    if (hipEventQuery(m->ev0) != hipSuccess) return RT_ERR_UNSUPPORTED;
    for (uint32_t r = 0; r < n; r++) {
        if (hipEventQuery(m->done[r]) != hipSuccess) return RT_ERR_UNSUPPORTED;
        if (hipEventElapsedTime(&ms[r], m->ev0, m->done[r]) != hipSuccess) return RT_ERR_UNSUPPORTED;
    }
    return RT_OK;
}

// Every rank of `m` (ranks[0] included): f, first error wins.
rt_status rt_multi_each_rank(rt_multi_state* m, const std::function<rt_status(rt_scene*)>& f) {
    for (rt_scene* s : m->ranks) {
        rt_status st = f(s);
        if (st != RT_OK) return st;
    }
    return RT_OK;
}

// the render's counters (summed over the ranks) and span, for rt_render_opts
static rt_status multi_finish(rt_multi_state* m, const rt_render_opts* opts) {
    const uint32_t world = (uint32_t)m->ranks.size();
    if (opts && opts->counters) {
        rt_counters c{0, 0, 0, 0};
        for (uint32_t r = 0; r < world; r++) {
            unsigned long long h[3] = {0, 0, 0};
            MHIP(hipSetDevice(m->devices[r]));
            MHIP(hipMemcpy(h, m->counters[r], sizeof(h), hipMemcpyDeviceToHost));
            c.node_rays += h[0];
            c.shadow_rays += h[1];
            c.pixels += h[2];
        }
        *opts->counters = c;
    }
    if (opts && opts->kernel_ms) {
        float ms = 0.f;
        MHIP(hipSetDevice(m->devices[0]));
        MHIP(hipEventElapsedTime(&ms, m->ev0, m->ev1));
        *opts->kernel_ms = ms;
    }
    MHIP(hipSetDevice(m->devices[0]));
    return RT_OK;
}

rt_status rt_multi_build(rt_scene* s0, const int32_t* devices, uint32_t n_devices, bool allow_rccl,
                         rt_multi_state** out) {
    rt_status st = RT_OK;
    rt_multi_state* m = new (std::nothrow) rt_multi_state();
    if (!m) return RT_ERR_OUT_OF_MEMORY;
    m->devices.assign(devices, devices + n_devices);
    m->ranks.assign(n_devices, nullptr);
    m->ranks[0] = s0;
    m->streams.assign(n_devices, nullptr);
    m->done.assign(n_devices, nullptr);
    m->copied.assign(n_devices, nullptr);
    m->band.assign(n_devices, nullptr);
    m->band8.assign(n_devices, nullptr);
    m->counters.assign(n_devices, nullptr);
    auto fail = [&](rt_status e) {
        rt_multi_free(m);
        return e;
    };
    for (uint32_t r = 0; r < n_devices; r++) {
        if (r > 0 && (st = rt_scene_clone(s0, devices[r], &m->ranks[r])) != RT_OK) return fail(st);
        if (hipSetDevice(devices[r]) != hipSuccess ||
            hipStreamCreateWithFlags(&m->streams[r], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreate(&m->done[r]) != hipSuccess || hipEventCreate(&m->copied[r]) != hipSuccess ||
            hipMalloc(&m->counters[r], 3 * sizeof(unsigned long long)) != hipSuccess)
            return fail(RT_ERR_HIP);
    }
    if (hipSetDevice(devices[0]) != hipSuccess || hipEventCreate(&m->ev0) != hipSuccess ||
        hipEventCreate(&m->ev1) != hipSuccess)
        return fail(RT_ERR_HIP);
    std::vector<int> sorted(m->devices);
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (distinct && allow_rccl) {
        if (!load_rccl(m->lib)) {
            std::fprintf(stderr, "rt_multi.cpp: librccl.so.1 not loadable: %s\n", dlerror());
            return fail(RT_ERR_UNSUPPORTED);
        }
        m->comms.assign(n_devices, nullptr);
        ncclResult_t e = m->lib.init_all(m->comms.data(), (int)n_devices, m->devices.data());
        if (e != ncclSuccess) {
            std::fprintf(stderr, "rt_multi.cpp: ncclCommInitAll: %s\n", m->lib.error_string(e));
            m->comms.clear();
            return fail(RT_ERR_HIP);
        }
        m->rccl = true;
    }
    (void)hipSetDevice(devices[0]);
    *out = m;
    return RT_OK;
}

void rt_multi_set_band_rows(rt_multi_state* m, uint32_t band_rows) {
    if (m && band_rows > 0) m->band_rows = band_rows;
}

extern "C" {

rt_status rt_scene_create_multi(const rt_scene_desc* desc, const int32_t* devices, uint32_t n_devices,
                                rt_scene** out) {
    if (!desc || !devices || !out || n_devices == 0) return RT_ERR_INVALID_ARG;
    int n_visible = 0;
    if (hipGetDeviceCount(&n_visible) != hipSuccess || n_visible <= 0) return RT_ERR_NO_DEVICE;
    for (uint32_t r = 0; r < n_devices; r++)
        if (devices[r] < 0 || devices[r] >= n_visible) return RT_ERR_INVALID_ARG;
    rt_scene* s0 = nullptr;
    rt_status st = rt_scene_create(desc, devices[0], &s0);
    // Tune::force_rccl (RT_TUNE="force_rccl=1"): one device still renders through the band
    // render + ncclGather (a one-rank communicator) + un-permute, so a one-GPU machine
    // executes the RCCL exchange
    const bool force_rccl = st == RT_OK && rt_scene_tune(s0).force_rccl != 0;
    if (st != RT_OK || (n_devices == 1 && !force_rccl)) {
        *out = s0;
        return st;
    }
    rt_multi_state* m = nullptr;
    st = rt_multi_build(s0, devices, n_devices, true, &m);
    if (st != RT_OK) {
        rt_scene_destroy(s0);
        return st;
    }
    rt_scene_multi(s0) = m;  // rt_scene_destroy(s0) frees m from here on
    (void)hipSetDevice(devices[0]);
    *out = s0;
    return RT_OK;
}

int32_t rt_scene_device_count(const rt_scene* s) {
    if (!s) return 0;
    rt_multi_state* m = rt_scene_multi(const_cast<rt_scene*>(s));
    return m ? (int32_t)m->ranks.size() : 1;
}

int32_t rt_scene_uses_rccl(const rt_scene* s) {
    if (!s) return 0;
    rt_multi_state* m = rt_scene_multi(const_cast<rt_scene*>(s));
    return (m && m->rccl) ? 1 : 0;
}

}  // extern "C"
