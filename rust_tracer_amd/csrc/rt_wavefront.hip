// rt_wavefront.hip -- level-synchronous render pipeline (the default device path).
//
// The reference recursion (render.rs:40-103) is evaluated one TREE LEVEL at a time over
// the whole frame:
//
//   trace(level 0)  every pixel's primary ray (Camera::get_ray, render.rs:178-185)
//   trace(level k)  every level-k ray in the compacted queue written by level k-1
//                   - nearest-hit scan (Scene::intersect, scene/mod.rs:98-116)
//                   - hit attributes, then one shadow scan per point light
//                     (PointLight::get_energy, mod.rs:189-206) and Phong/Schlick shading
//                   - node record (ambient + lights, child weights) -> node pool
//                   - reflected / refracted child rays (render.rs:105-125) appended to the
//                     level k+1 queue (one wave-aggregated atomic per wave)
//   combine(level depth-1 .. 0)
//                   post-order: every node folds the colours its children reported into
//                   ((ambient + lights) + reflected) + refracted (render.rs:100) and
//                   reports its colour to its parent's slot; level 0 writes the pixel.
//
// Why levels and not one per-pixel megakernel (rt_kernels.hip): per-pixel ray trees are
// ragged (median 1 node, p99 31, max > 80 at depth 8 in config 3), so a lane that owns a
// pixel serialises up to ~350 scans while the average lane has ~110 to do: the frame
// becomes critical-path bound.  Per level, every queue entry costs the same (one node scan
// + one scan per light), so lanes stay ~fully occupied, and the post-order combine keeps
// the reference's exact operation order (pixel values reach |4000| in config 3, so a
// reassociated "throughput" formulation would break the 1e-4 tolerance).
#include "rt_common.hpp"

namespace rtdev {

enum : uint32_t { NODE_HIT = 1u << 8, NODE_MISS = 1u << 9, NODE_NONE = 1u << 10 };

struct PixelRef {
    bool valid;
    uint32_t u, v, lr;
};

// level-0 item -> pixel of this rank's band buffer (8x8 tiles, block-cyclic row bands)
__device__ __forceinline__ PixelRef pixel_of(const WaveParams& P, uint32_t item) {
    PixelRef r;
    uint32_t tile = item >> 6, w = item & 63u;
    r.u = (tile % P.tiles_x) * 8u + (w & 7u);
    r.lr = (tile / P.tiles_x) * 8u + (w >> 3);
    uint32_t band = r.lr / P.band_rows;
    r.v = (band * P.world + P.rank) * P.band_rows + (r.lr - band * P.band_rows);
    r.valid = r.u < P.width && r.lr < P.rows_local && r.v < P.height;
    return r;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    uint32_t lane = lane_id();
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

__global__ __launch_bounds__(256) void trace_level_kernel(WaveParams P, uint32_t level) {
    const DevScene& S = P.S;
    const uint32_t off = P.levels[2 * level];
    const uint32_t count = min(P.levels[2 * level + 1], off < P.capacity ? P.capacity - off : 0u);
    const uint32_t next_off = off + count;
    if (blockIdx.x == 0 && threadIdx.x == 0) P.levels[2 * (level + 1)] = next_off;
    const uint32_t lane = lane_id();
    uint32_t n_shadow = 0, n_node = 0, n_pix = 0;  // per lane, reduced at the end

    const uint32_t stride = gridDim.x * blockDim.x;
    // whole waves iterate together (the loop bound is rounded up to a wave multiple) so
    // the wave-aggregated append below always sees every lane
    const uint32_t wave_base = (blockIdx.x * blockDim.x + threadIdx.x) & ~63u;
    for (uint32_t base = wave_base; base < count; base += stride) {
        const uint32_t t = base + lane;
        bool active = t < count;
        V3 ro = v3(0, 0, 0), rd = v3(0, 0, 0);
        uint32_t parent = 0;
        uint32_t n = off + t;
        if (active) {
            if (level == 0) {
                PixelRef px = pixel_of(P, t);
                if (!px.valid) {
                    P.nodes[n].flags = NODE_NONE;
                    active = false;
                } else {
                    n_pix++;
                    if (P.depth == 0) {  // trace_ray(.., 0) == BLACK, no scan
                        P.nodes[n].flags = NODE_MISS;
                        active = false;
                    } else {
                        float x = P.x_min + (float)px.u * P.x_delta;
                        float y = P.y_max - (float)px.v * P.y_delta;
                        V3 cam = v3(P.cam_ox, P.cam_oy, P.cam_oz);
                        ro = cam;
                        rd = norm(sub(v3(x, y, 0.f), cam));
                    }
                }
            } else {
                const Task& T = P.tasks[n];
                ro = v3(T.ox, T.oy, T.oz);
                rd = v3(T.dx, T.dy, T.dz);
                parent = T.parent;
            }
        }
        bool want_refl = false, want_refr = false;
        V3 rro = v3(0, 0, 0), rrd = v3(0, 0, 0), tro = v3(0, 0, 0), trd = v3(0, 0, 0);
        if (active) {
            n_node++;
            float bt;
            uint32_t bk;
            scan(S, ro, rd, bt, bk);
            if (bk == 0xFFFFFFFFu) {
                P.nodes[n].flags = NODE_MISS;  // trace_ray -> BLACK; parent slot stays 0
            } else {
                const MatRec& M = S.mats[S.shapes[bk >> 4].mat];
                Hit h = hit_attrs(S, bk, ro, rd, M.kind == RT_MAT_TEXTURE_PHONG);
                float ri = M.refraction_index;
                float n1 = h.entering ? 1.f : ri;
                float n2 = h.entering ? ri : 1.f;
                V3 ka = tex_eval(M.ambient, h.tu, h.tv);
                V3 kd = tex_eval(M.diffuse, h.tu, h.tv);
                V3 ks = tex_eval(M.specular, h.tu, h.tv);
                // render.rs:59-68 with get_light_energy :142-153
                V3 ps = add(h.p, mul(h.n, 0.0002f));
                V3 lsum = v3(0.f, 0.f, 0.f);
                for (int li = 0; li < S.n_lights; ++li) {
                    const LightRec& L = S.lights[li];
                    V3 ldir = v3(0.f, 0.f, 0.f);
                    V3 E = v3(L.r, L.g, L.b);
                    if (L.kind == RT_LIGHT_POINT) {
                        V3 lpos = v3(L.px, L.py, L.pz);
                        ldir = norm(sub(lpos, ps));
                        float st;
                        uint32_t sk;
                        scan(S, ps, ldir, st, sk);
                        n_shadow++;
                        if (sk != 0xFFFFFFFFu && len2(sub(add(ps, mul(ldir, st)), ps)) < len2(sub(lpos, ps)))
                            E = v3(0.f, 0.f, 0.f);
                    }
                    float f = fresnel_reflection(ldir, h.n, n1, n2);
                    V3 g = reflected_energy(E, ldir, h, kd, ks, M.power);
                    lsum = add(lsum, v3(f * g.x, f * g.y, f * g.z));
                }
                V3 amb = v3(ka.x * S.amb_r, ka.y * S.amb_g, ka.z * S.amb_b);
                V3 loc = add(amb, lsum);
                NodeRec rec;
                rec.ax = loc.x; rec.ay = loc.y; rec.az = loc.z;
                rec.fr = 0.f; rec.dr = 0.f; rec.pw = 0.f; rec.ft = 0.f;
                rec.kdx = kd.x; rec.kdy = kd.y; rec.kdz = kd.z;
                rec.ksx = ks.x; rec.ksy = ks.y; rec.ksz = ks.z;
                rec.erx = 0.f; rec.ery = 0.f; rec.erz = 0.f;
                rec.etx = 0.f; rec.ety = 0.f; rec.etz = 0.f;
                rec.flags = NODE_HIT;
                rec.parent = parent;
                rec.pad[0] = rec.pad[1] = rec.pad[2] = 0u;
                bool child_ok = level + 1 < P.depth;
                if (M.reflectivity > RT_EPS) {  // render.rs:70-84, reflect_ray :105-110
                    rec.flags |= F_REFL;
                    V3 rv = sub(mul(h.n, 2.f * dot(rd, h.n)), rd);
                    rrd = neg(norm(rv));
                    rro = add(h.p, mul(rrd, 0.0002f));
                    rec.fr = fresnel_reflection(rrd, h.n, n1, n2);
                    rec.dr = dot(rrd, h.n);
                    V3 hv = norm(add(norm(h.eye), norm(rrd)));
                    float mh = dot(h.n, hv);
                    if (!(mh < 0.f)) {
                        rec.flags |= F_SPEC;
                        rec.pw = powf(mh, M.power);
                    }
                    want_refl = child_ok;
                }
                if (ri > RT_EPS) {  // render.rs:86-98, refract_ray :112-125
                    rec.flags |= F_REFR;
                    float ratio = n1 / n2;
                    float m_dot_r = -dot(rd, h.n);
                    float cos2 = 1.f - ratio * ratio * (1.f - m_dot_r * m_dot_r);
                    if (cos2 > 0.f) {
                        float ct = sqrtf(cos2);
                        trd = add(mul(rd, ratio), mul(h.n, ratio * m_dot_r - ct));
                        tro = add(h.p, mul(trd, 0.0002f));
                        rec.ft = 1.f - fresnel_reflection(trd, neg(h.n), n1, n2);
                        want_refr = child_ok;
                    } else {
                        rec.flags |= F_TIR;
                    }
                }
                P.nodes[n] = rec;
            }
        }
        // ---- append the children to the level+1 queue: one atomic per wave
        uint64_t bl = __ballot(want_refl), br = __ballot(want_refr);
        uint32_t total = (uint32_t)(__builtin_popcountll(bl) + __builtin_popcountll(br));
        if (total) {
            uint32_t wbase = 0;
            uint32_t first = (uint32_t)__builtin_ctzll(bl | br);
            if (lane == first) wbase = atomicAdd(&P.levels[2 * (level + 1) + 1], total);
            wbase = (uint32_t)__builtin_amdgcn_readlane((int)wbase, (int)first);
            uint64_t lt = lanemask_lt();
            uint32_t my = wbase + (uint32_t)(__builtin_popcountll(bl & lt) + __builtin_popcountll(br & lt));
            if (want_refl) {
                uint32_t slot = next_off + my;
                if (slot < P.capacity) {
                    Task T = {rro.x, rro.y, rro.z, rrd.x, rrd.y, rrd.z, (n << 1) | 0u, 0u};
                    P.tasks[slot] = T;
                } else {
                    atomicOr(P.overflow, 1u);
                }
                my++;
            }
            if (want_refr) {
                uint32_t slot = next_off + my;
                if (slot < P.capacity) {
                    Task T = {tro.x, tro.y, tro.z, trd.x, trd.y, trd.z, (n << 1) | 1u, 0u};
                    P.tasks[slot] = T;
                } else {
                    atomicOr(P.overflow, 1u);
                }
            }
        }
    }
    // ---- counters: wave reduction, one atomic per wave
    for (int o = 32; o > 0; o >>= 1) {
        n_node += __shfl_xor(n_node, o);
        n_shadow += __shfl_xor(n_shadow, o);
        n_pix += __shfl_xor(n_pix, o);
    }
    if (lane == 0 && P.ray_counters) {
        if (n_node) atomicAdd(P.ray_counters + 0, (unsigned long long)n_node);
        if (n_shadow) atomicAdd(P.ray_counters + 1, (unsigned long long)n_shadow);
        if (n_pix) atomicAdd(P.ray_counters + 2, (unsigned long long)n_pix);
    }
}

// render.rs:100 for every node of `level`; children (level + 1) have already reported.
__global__ __launch_bounds__(256) void combine_level_kernel(WaveParams P, uint32_t level) {
    const uint32_t off = P.levels[2 * level];
    const uint32_t count = min(P.levels[2 * level + 1], off < P.capacity ? P.capacity - off : 0u);
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < count; t += stride) {
        const uint32_t n = off + t;
        const NodeRec& R = P.nodes[n];
        uint32_t flags = R.flags;
        if (flags & NODE_NONE) {  // padding of the band buffer: defined as 0
            PixelRef px = pixel_of(P, t);
            if (level == 0 && px.u < P.width && px.lr < P.rows_local) {
                float* o = P.out + ((size_t)px.lr * P.width + px.u) * 3u;
                o[0] = 0.f;
                o[1] = 0.f;
                o[2] = 0.f;
            }
            continue;
        }
        V3 c = v3(0.f, 0.f, 0.f);
        if (flags & NODE_HIT) {
            Frame f;
            f.ax = R.ax; f.ay = R.ay; f.az = R.az;
            f.fr = R.fr; f.dr = R.dr; f.pw = R.pw; f.ft = R.ft;
            f.kdx = R.kdx; f.kdy = R.kdy; f.kdz = R.kdz;
            f.ksx = R.ksx; f.ksy = R.ksy; f.ksz = R.ksz;
            f.flags = flags;
            c = combine(f, v3(R.erx, R.ery, R.erz), v3(R.etx, R.ety, R.etz));
        } else if (level > 0) {
            continue;  // a missed child reports BLACK: the parent's slot already holds 0
        }
        if (level == 0) {
            PixelRef px = pixel_of(P, t);
            float* o = P.out + ((size_t)px.lr * P.width + px.u) * 3u;
            o[0] = c.x;
            o[1] = c.y;
            o[2] = c.z;
        } else {
            NodeRec& Q = P.nodes[R.parent >> 1];
            if (R.parent & 1u) {
                Q.etx = c.x; Q.ety = c.y; Q.etz = c.z;
            } else {
                Q.erx = c.x; Q.ery = c.y; Q.erz = c.z;
            }
        }
    }
}

// levels[] = {0, total_items, 0, 0, ...}, overflow = 0
__global__ void wave_init_kernel(uint32_t* levels, uint32_t n_words, uint32_t total_items, uint32_t* overflow) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_words) levels[i] = (i == 1) ? total_items : 0u;
    if (i == 0) *overflow = 0u;
}

hipError_t launch_wave_init(uint32_t* levels, uint32_t n_words, uint32_t total_items, uint32_t* overflow,
                            hipStream_t stream) {
    hipLaunchKernelGGL(wave_init_kernel, dim3((n_words + 255) / 256), dim3(256), 0, stream, levels, n_words,
                       total_items, overflow);
    return hipGetLastError();
}

hipError_t wave_occupancy(int* trace_blocks, int* combine_blocks) {
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(trace_blocks, trace_level_kernel, 256, 0);
    if (e != hipSuccess) return e;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(combine_blocks, combine_level_kernel, 256, 0);
}

hipError_t launch_wave_trace(const WaveParams& p, uint32_t level, int blocks, hipStream_t stream) {
    hipLaunchKernelGGL(trace_level_kernel, dim3(blocks), dim3(256), 0, stream, p, level);
    return hipGetLastError();
}

hipError_t launch_wave_combine(const WaveParams& p, uint32_t level, int blocks, hipStream_t stream) {
    hipLaunchKernelGGL(combine_level_kernel, dim3(blocks), dim3(256), 0, stream, p, level);
    return hipGetLastError();
}

}  // namespace rtdev

#if RT_STATS
// tools/scan_stats.py: read (and optionally reset) the wavefront pipeline's scan counters
extern "C" int rt_debug_scan_stats(unsigned long long* out8, int reset) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(rtdev::rt_scan_stats), 8 * sizeof(unsigned long long)) != hipSuccess)
        return 1;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(rtdev::rt_scan_stats), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif
