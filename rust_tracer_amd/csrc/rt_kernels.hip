// rt_kernels.hip -- the gfx950 megakernel for rust_tracer's render path.
//
// One persistent kernel owns the whole per-pixel work of src/render.rs:31-103:
// primary-ray generation (Camera::get_ray, render.rs:178-185), the linear nearest-hit
// scan (Scene::intersect, scene/mod.rs:98-116) over spheres / triangles / cubes /
// planes, the point-light shadow scans (PointLight::get_energy, mod.rs:189-206), Phong
// + Schlick shading (material.rs:77-93,165-213; render.rs:129-140) and the Whitted
// recursion (reflect_ray / refract_ray, render.rs:105-125).
//
// Execution model (MI355X-first, not a translation of the recursive CPU code):
//  * Each lane runs a small state machine whose every step is ONE scene scan: either the
//    nearest-hit scan of a tree node's ray or one shadow scan.  All lanes of a wave scan
//    the same primitive at the same time, so primitive records are wave-uniform and are
//    read with scalar (SMEM) loads; the per-lane work is pure f32 VALU.
//  * The recursion becomes a post-order continuation stack (frames in scratch, one per
//    pending tree level) so children combine into the parent exactly in the reference's
//    operation order: ((ambient + lights) + reflected) + refracted.
//  * Persistent workgroups; a lane that finishes its pixel takes the next one from a
//    global counter (wave-aggregated atomicAdd), so lanes stay busy while other lanes of
//    the wave are deep in a glass-sphere ray tree (lane-level compaction).
//
// Numerics: compiled with -ffp-contract=off, IEEE division/sqrt and f32 denormals on,
// so every +,-,*,/,sqrt is the same correctly rounded operation the reference
// executes, in the same order.  powf is glibc's evaluation (rt_powf.hpp); atan2f / acosf
// (textured spheres only) come from ocml (<= 1-2 ulp from glibc).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#include "../../include/rt_api.h"
#include "rt_device.hpp"

#include "rt_common.hpp"

namespace rtdev {

template <int MAXF>
__global__ __launch_bounds__(256) void render_kernel(RenderParams P) {
    rt_pow_stage();
    const DevScene& S = P.S;
    const V3 cam_o = v3(P.cam_ox, P.cam_oy, P.cam_oz);
    const uint32_t lane = lane_id();
    ScanCnt cnt;
    cnt_init(cnt);

    Frame st[MAXF > 0 ? MAXF : 1];

    // lane state
    int32_t item = -1;     // current work item (pixel), -1 = idle
    bool exhausted = false;
    uint32_t out_idx = 0;  // float index of this pixel in P.out
    V3 ro = v3(0, 0, 0), rd = v3(0, 0, 0);  // current node ray
    int32_t lvl = 0;       // tree level of the current node
    int32_t phase = 0;     // 0 = node scan, 1 = shadow scan for light `li`
    int32_t li = 0;
    // wave-uniform counters (SGPRs): scans by kind, pixels, loop iterations
    unsigned long long n_node = 0, n_shadow = 0, n_pix = 0, n_iter = 0;

    // node being shaded
    Hit h;
    h.mat = 0;
    float n1 = 1.f, n2 = 1.f;
    V3 ka = v3(0, 0, 0), kd = v3(0, 0, 0), ks = v3(0, 0, 0), lsum = v3(0, 0, 0), ps = v3(0, 0, 0),
       ldir = v3(0, 0, 0);
    float power = 0.f;

    for (;;) {
        // ---- refill idle lanes with new pixels (one atomic per wave)
        for (;;) {
            uint64_t need = __ballot(item < 0 && !exhausted);
            if (need == 0) break;
            uint32_t first = (uint32_t)__builtin_ctzll(need);
            uint32_t n_need = (uint32_t)__builtin_popcountll(need);
            uint32_t base = 0;
            if (lane == first) base = atomicAdd(P.work_counter, n_need);
            base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)first);
            bool got = false;
            if (item < 0 && !exhausted) {
                uint32_t rank_in = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                uint32_t my = base + rank_in;
                if (my >= P.total_items) {
                    exhausted = true;
                } else {
                    uint32_t tile = my >> 6, w = my & 63u;
                    uint32_t u = (tile % P.tiles_x) * 8u + (w & 7u);
                    uint32_t lr = (tile / P.tiles_x) * 8u + (w >> 3);
                    uint32_t band = lr / P.band_rows;
                    uint32_t v = (band * P.world + P.rank) * P.band_rows + (lr - band * P.band_rows);
                    if (u < P.width && lr < P.rows_local && v < P.height) {
                        got = true;
                        out_idx = (lr * P.width + u) * 3u;
                        if (P.depth == 0) {  // trace_ray(.., 0) == BLACK
                            P.out[out_idx] = 0.f;
                            P.out[out_idx + 1] = 0.f;
                            P.out[out_idx + 2] = 0.f;
                        } else {
                            // Camera::get_ray (render.rs:178-185)
                            float x = P.x_min + (float)u * P.x_delta;
                            float y = P.y_max - (float)v * P.y_delta;
                            ro = cam_o;
                            rd = norm(sub(v3(x, y, 0.f), cam_o));
                            lvl = 0;
                            phase = 0;
                            item = (int32_t)my;
                        }
                    }
                }
            }
            n_pix += (unsigned long long)__builtin_popcountll(__ballot(got));
        }
        uint64_t active = __ballot(item >= 0);
        if (active == 0) break;
        uint64_t node_lanes = __ballot(item >= 0 && phase == 0);
        n_iter++;
        n_node += (unsigned long long)__builtin_popcountll(node_lanes);
        n_shadow += (unsigned long long)__builtin_popcountll(active & ~node_lanes);
        if (item < 0) continue;

        // ---- one scene scan
        V3 so = (phase == 0) ? ro : ps;
        V3 sd = (phase == 0) ? rd : ldir;
        float bt;
        uint32_t bk;
        scan(S, so, sd, bt, bk, cnt);
        bool hit = bk != 0xFFFFFFFFu;

        bool node_done = false;
        bool returning = false;
        V3 ret = v3(0.f, 0.f, 0.f);

        if (phase == 0) {
            if (!hit) {
                returning = true;  // trace_ray -> BLACK
            } else {
                const MatRec& M = S.mats[S.shapes[bk >> 4].mat];
                bool textured = M.kind == RT_MAT_TEXTURE_PHONG;
                h = hit_attrs(S, bk, ro, rd, textured);
                float ri = M.refraction_index;
                n1 = h.entering ? 1.f : ri;
                n2 = h.entering ? ri : 1.f;
                ka = tex_eval(M.ambient, h.tu, h.tv);
                kd = tex_eval(M.diffuse, h.tu, h.tv);
                ks = tex_eval(M.specular, h.tu, h.tv);
                power = M.power;
                lsum = v3(0.f, 0.f, 0.f);
                ps = add(h.p, mul(h.n, 0.0002f));  // render.rs:147
                li = 0;
                node_done = true;  // unless a point light needs a shadow scan (below)
            }
        } else {
            const LightRec& L = S.lights[li];
            V3 lpos = v3(L.px, L.py, L.pz);
            bool shadowed = hit && (len2(sub(add(ps, mul(sd, bt)), ps)) < len2(sub(lpos, ps)));
            V3 E = shadowed ? v3(0.f, 0.f, 0.f) : v3(L.r, L.g, L.b);
            float f = fresnel_reflection(ldir, h.n, n1, n2);
            V3 g = reflected_energy(E, ldir, h, kd, ks, power);
            lsum = add(lsum, v3(f * g.x, f * g.y, f * g.z));
            li++;
            node_done = true;
        }

        if (node_done) {
            // advance over ambient lights (no scan) to the next point light
            bool need_scan = false;
            while (li < S.n_lights) {
                const LightRec& L = S.lights[li];
                if (L.kind == RT_LIGHT_POINT) {
                    ldir = norm(sub(v3(L.px, L.py, L.pz), ps));
                    phase = 1;
                    need_scan = true;
                    break;
                }
                V3 z = v3(0.f, 0.f, 0.f);
                float f = fresnel_reflection(z, h.n, n1, n2);
                V3 g = reflected_energy(v3(L.r, L.g, L.b), z, h, kd, ks, power);
                lsum = add(lsum, v3(f * g.x, f * g.y, f * g.z));
                li++;
            }
            if (need_scan) continue;

            // ---- the node is shaded: ambient + lights; set up its children
            const MatRec& M = S.mats[h.mat];
            Frame f;
            V3 amb = v3(ka.x * S.amb_r, ka.y * S.amb_g, ka.z * S.amb_b);
            V3 loc = add(amb, lsum);
            f.ax = loc.x; f.ay = loc.y; f.az = loc.z;
            f.kdx = kd.x; f.kdy = kd.y; f.kdz = kd.z;
            f.ksx = ks.x; f.ksy = ks.y; f.ksz = ks.z;
            f.erx = 0.f; f.ery = 0.f; f.erz = 0.f;
            f.fr = 0.f; f.dr = 0.f; f.pw = 0.f; f.ft = 0.f;
            f.rox = f.roy = f.roz = f.rdx = f.rdy = f.rdz = 0.f;
            f.flags = 0;
            bool child_ok = (uint32_t)(lvl + 1) < P.depth;
            V3 rro = v3(0, 0, 0), rrd = v3(0, 0, 0);
            bool trace_refl = false, trace_refr = false;
            if (M.reflectivity > RT_EPS) {  // render.rs:70-84 with reflect_ray :105-110
                f.flags |= F_REFL;
                V3 rv = sub(mul(h.n, 2.f * dot(rd, h.n)), rd);  // vector3.rs:113-115
                rrd = neg(norm(rv));
                rro = add(h.p, mul(rrd, 0.0002f));
                f.fr = fresnel_reflection(rrd, h.n, n1, n2);
                f.dr = dot(rrd, h.n);
                V3 hv = norm(add(norm(h.eye), norm(rrd)));
                float mh = dot(h.n, hv);
                if (!(mh < 0.f)) {
                    f.flags |= F_SPEC;
                    f.pw = rtpow::powf_glibc(mh, power);
                }
                trace_refl = child_ok;
            }
            if (M.refraction_index > RT_EPS) {  // render.rs:86-98 with refract_ray :112-125
                f.flags |= F_REFR;
                float ratio = n1 / n2;
                float m_dot_r = -dot(rd, h.n);
                float cos2 = 1.f - ratio * ratio * (1.f - m_dot_r * m_dot_r);
                if (cos2 > 0.f) {
                    float ct = sqrtf(cos2);
                    V3 td = add(mul(rd, ratio), mul(h.n, ratio * m_dot_r - ct));
                    V3 to = add(h.p, mul(td, 0.0002f));
                    f.ft = 1.f - fresnel_reflection(td, neg(h.n), n1, n2);
                    f.rox = to.x; f.roy = to.y; f.roz = to.z;
                    f.rdx = td.x; f.rdy = td.y; f.rdz = td.z;
                    trace_refr = child_ok;
                } else {
                    f.flags |= F_TIR;
                }
            }
            if (!trace_refl && !trace_refr) {
                ret = combine(f, v3(0.f, 0.f, 0.f), v3(0.f, 0.f, 0.f));
                returning = true;
            } else {
                if (trace_refl) {
                    f.flags |= F_WAIT_REFL | (trace_refr ? F_PEND_REFR : 0u);
                    ro = rro;
                    rd = rrd;
                } else {
                    f.flags |= F_WAIT_REFR;
                    ro = v3(f.rox, f.roy, f.roz);
                    rd = v3(f.rdx, f.rdy, f.rdz);
                }
                st[lvl] = f;
                lvl++;
                phase = 0;
            }
        }

        if (returning) {
            // pop finished children into their parents (post-order)
            for (;;) {
                if (lvl == 0) {
                    P.out[out_idx] = ret.x;
                    P.out[out_idx + 1] = ret.y;
                    P.out[out_idx + 2] = ret.z;
                    item = -1;
                    break;
                }
                lvl--;
                Frame f = st[lvl];
                if (f.flags & F_WAIT_REFL) {
                    if (f.flags & F_PEND_REFR) {
                        st[lvl].erx = ret.x;
                        st[lvl].ery = ret.y;
                        st[lvl].erz = ret.z;
                        st[lvl].flags = (f.flags & ~(F_WAIT_REFL | F_PEND_REFR)) | F_WAIT_REFR;
                        ro = v3(f.rox, f.roy, f.roz);
                        rd = v3(f.rdx, f.rdy, f.rdz);
                        lvl++;
                        phase = 0;
                        break;
                    }
                    ret = combine(f, ret, v3(0.f, 0.f, 0.f));
                } else {
                    ret = combine(f, v3(f.erx, f.ery, f.erz), ret);
                }
            }
        }
    }

    // ---- counters: one atomic per wave (values are wave totals already)
    if (lane == 0 && P.ray_counters) {
        atomicAdd(P.ray_counters + 0, n_node);
        atomicAdd(P.ray_counters + 1, n_shadow);
        atomicAdd(P.ray_counters + 2, n_pix);
    }
    if (lane == 0 && P.iter_counter) atomicAdd(P.iter_counter, n_iter);
    cnt_flush(cnt, ops_slot(S));
}

// Scatter gathered per-rank band buffers into the row-major frame (one block row per frame
// row); T = float (RGB f32) or uint8_t (RGB8, Color::as_u8 values).
// Frame batches (blockIdx.z = frame f): rank r's bands of frame f start at row
// r * rank_rows + f * rows_per_rank of `in` (rank_rows = rows_per_rank for one frame), and
// frame f lands at out + f * height rows.
template <class T>
__global__ void unpermute_kernel(const T* __restrict__ in, uint32_t row_floats, uint32_t height,
                                 uint32_t band_rows, uint32_t world, uint32_t rows_per_rank, uint32_t rank_rows,
                                 T* __restrict__ out) {
    uint32_t v = blockIdx.y;
    if (v >= height) return;
    const uint32_t f = blockIdx.z;
    uint32_t band = v / band_rows;
    uint32_t rank = band % world;
    uint32_t lr = (band / world) * band_rows + (v - band * band_rows);
    const T* src = in + ((size_t)rank * rank_rows + (size_t)f * rows_per_rank + lr) * row_floats;
    T* dst = out + ((size_t)f * height + v) * row_floats;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < row_floats; i += gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// Color::as_u8 (color.rs:43-46): (255 * c) as u8, saturating, NaN -> 0
__global__ void quantize_kernel(const float* __restrict__ in, size_t n, uint8_t* __restrict__ out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) out[i] = as_u8(in[i]);
}

}  // namespace rtdev

// ------------------------------------------------------------------ launch wrappers
namespace rtdev {

// The scan's compile-time cube triangles must equal the host-built Cube::new table.
bool rt_cube_table_check(const float* table) {
    struct T {
        int k, sx, sy, sz, a, b, c, d, e, f;
    };
#define RT_CUBE_ROW(k, sx, sy, sz, a, b, c, d_, e, f) T{k, sx, sy, sz, a, b, c, d_, e, f},
    const T rows[12] = {RT_CUBE_TRIS(RT_CUBE_ROW)};
#undef RT_CUBE_ROW
    for (int k = 0; k < 12; k++) {
        const float* q = table + 16 * k;  // {v0 -} {e1 -} {e2 -} {n -}
        const T& r = rows[k];
        if (r.k != k) return false;
        const float want[9] = {0.5f * r.sx, 0.5f * r.sy, 0.5f * r.sz, (float)r.a, (float)r.b,
                               (float)r.c, (float)r.d, (float)r.e, (float)r.f};
        const float got[9] = {q[0], q[1], q[2], q[4], q[5], q[6], q[8], q[9], q[10]};
        for (int j = 0; j < 9; j++)
            if (want[j] != got[j]) return false;
    }
    return true;
}

hipError_t launch_render(const RenderParams& p, int blocks, hipStream_t stream) {
    int maxf = (int)p.depth - 1;
    if (maxf <= 7) {
        hipLaunchKernelGGL(render_kernel<7>, dim3(blocks), dim3(256), 0, stream, p);
    } else if (maxf <= 15) {
        hipLaunchKernelGGL(render_kernel<15>, dim3(blocks), dim3(256), 0, stream, p);
    } else {
        hipLaunchKernelGGL(render_kernel<63>, dim3(blocks), dim3(256), 0, stream, p);
    }
    return hipGetLastError();
}

hipError_t render_occupancy(uint32_t depth, int* blocks_per_cu) {
    int maxf = (int)depth - 1;
    if (maxf <= 7) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, render_kernel<7>, 256, 0);
    if (maxf <= 15) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, render_kernel<15>, 256, 0);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, render_kernel<63>, 256, 0);
}

hipError_t launch_unpermute(const float* in, uint32_t x_res, uint32_t y_res, uint32_t band_rows,
                            uint32_t world, uint32_t rows_per_rank, float* out, hipStream_t stream,
                            uint32_t frames, uint32_t rank_rows) {
    uint32_t row_floats = x_res * 3u;
    dim3 grid((row_floats + 255) / 256, y_res, frames);
    hipLaunchKernelGGL(unpermute_kernel<float>, grid, dim3(256), 0, stream, in, row_floats, y_res, band_rows, world,
                       rows_per_rank, rank_rows ? rank_rows : rows_per_rank, out);
    return hipGetLastError();
}

hipError_t launch_unpermute_u8(const uint8_t* in, uint32_t x_res, uint32_t y_res, uint32_t band_rows,
                               uint32_t world, uint32_t rows_per_rank, uint8_t* out, hipStream_t stream,
                               uint32_t frames, uint32_t rank_rows) {
    uint32_t row_bytes = x_res * 3u;
    dim3 grid((row_bytes + 255) / 256, y_res, frames);
    hipLaunchKernelGGL(unpermute_kernel<uint8_t>, grid, dim3(256), 0, stream, in, row_bytes, y_res, band_rows, world,
                       rows_per_rank, rank_rows ? rank_rows : rows_per_rank, out);
    return hipGetLastError();
}

hipError_t launch_quantize(const float* in, size_t n, uint8_t* out, hipStream_t stream) {
    size_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(quantize_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, in, n, out);
    return hipGetLastError();
}

}  // namespace rtdev

namespace rtdev {

// ---- sample batches (rt_api.cpp launch_bands_wave): the batch's samples first .. first + n - 1
// were rendered into n buffers of frame_floats floats; fold them into `out` in sample order
// -- sample 0 starts the sum, each later sample is added to it (the f32 sample-order sum of
// rt_render_spp, include/rt_api.h) -- and the batch holding the last sample divides by spp
// and writes Color::as_u8 (color.rs:43-46) of the mean.
__global__ void spp_accumulate_kernel(const float* samples, uint32_t n, size_t frame_floats, uint32_t first,
                                      uint32_t spp, float* out, uint8_t* out8) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const bool last = first + n == spp;
    const float fs = (float)spp;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < frame_floats; i += stride) {
        float acc = first == 0 ? samples[i] : out[i] + samples[i];
        for (uint32_t j = 1; j < n; j++) acc = acc + samples[(size_t)j * frame_floats + i];
        if (last) {
            acc = acc / fs;
            if (out8) out8[i] = as_u8(acc);
        }
        out[i] = acc;
    }
}

hipError_t launch_spp_accumulate(const float* samples, uint32_t n, size_t frame_floats, uint32_t first, uint32_t spp,
                                 float* out, uint8_t* out8, hipStream_t stream) {
    const uint32_t blocks = (uint32_t)std::min<size_t>((frame_floats + 255) / 256, 8192u);
    hipLaunchKernelGGL(spp_accumulate_kernel, dim3(blocks), dim3(256), 0, stream, samples, n, frame_floats, first, spp,
                       out, out8);
    return hipGetLastError();
}

}  // namespace rtdev

// ---- powf verification hooks (tests/test_powf.py): the device's powf (rt_powf.hpp) over
// arrays, on the device and compiled for the host, against the oracle's libm powf
__global__ void powf_batch_kernel(const float* x, const float* y, float* out, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = rtpow::powf_glibc(x[i], y[i]);
}

extern "C" rt_status rt_powf_batch_async(const float* d_x, const float* d_y, float* d_out, uint64_t n, void* stream) {
    if (n == 0) return RT_OK;
    if (!d_x || !d_y || !d_out) return RT_ERR_INVALID_ARG;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 255) / 256, 4096u);
    hipLaunchKernelGGL(powf_batch_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, d_x, d_y, d_out, n);
    return hipGetLastError() == hipSuccess ? RT_OK : RT_ERR_HIP;
}

extern "C" rt_status rt_powf_batch_host(const float* x, const float* y, float* out, uint64_t n) {
    if (n && (!x || !y || !out)) return RT_ERR_INVALID_ARG;
    for (uint64_t i = 0; i < n; i++) out[i] = rtpow::powf_glibc(x[i], y[i]);
    return RT_OK;
}
