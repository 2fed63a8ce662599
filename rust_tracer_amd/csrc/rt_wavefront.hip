// rt_wavefront.hip -- level-synchronous render pipeline (the default device path).
//
// The reference recursion (render.rs:40-103) is evaluated breadth first over the frame:
//
//   trace(level 0)  every pixel's primary ray (Camera::get_ray, render.rs:178-185)
//   trace(level k)  every level-k ray of the compacted queue written by level k-1:
//                   nearest-hit scan (Scene::intersect, scene/mod.rs:98-116), attributes
//                   of the chosen shape, the node's shading inputs -> node pool, one
//                   shadow-queue entry per point light, reflected / refracted children
//                   (render.rs:105-125) -> level k+1 queue (one atomic per wave)
//   shadow          every shadow ray of every level in ONE launch (PointLight::get_energy,
//                   mod.rs:189-206), exact per-wave early exit (rt_scan.hpp)
//   combine(L-1..0) per node: lights (render.rs:59-68) from the shadow bits, then
//                   ((ambient + lights) + reflected) + refracted (render.rs:100) with the
//                   colours the children reported; the result goes to the parent's slot,
//                   level 0 writes the pixel.
//
// Why levels and not one per-pixel megakernel (round 1's design, 68 ms per frame; removed in
// round 4, git history): per-pixel ray trees are
// ragged (median 1 node, p99 31, max > 80 at depth 8 in config 3), so a lane that owns a
// pixel serialises up to ~350 scans while the average lane has ~110: the frame becomes
// critical-path bound.  Here every queue entry costs one scan, lanes stay full, and the
// post-order combine keeps the reference's exact operation order (pixel values reach
// |4000| in config 3, so a reassociated "throughput" formulation would break 1e-4).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <type_traits>

#include "rt_common.hpp"



namespace rtdev {

#define RT_SHADOW_COUNT(P) ((P).levels[2 * (RT_MAX_DEPTH + 1)])
#define RT_INSIDE_MASK ((1u << RT_FRAME_SHIFT) - 1u)  // Task.pixel below the frame bits

struct PixelRef {
    bool valid;
    uint32_t u, v, lr;
};

// level-0 item -> pixel of this rank's band buffer (8x8 tiles, block-cyclic row bands).  A
// wave's active items lie in one 64-item tile (waves take 64- or 32-aligned chunks), so the
// tile index is wave-uniform and its division by tiles_x runs on the scalar unit; the band
// divisor is read where it is used (opaque_u: its hoisted reciprocal would be spilled)
__device__ __forceinline__ PixelRef pixel_of(const WaveParams& P, uint32_t item) {
    PixelRef r;
    const uint32_t tile = (uint32_t)__builtin_amdgcn_readfirstlane((int)(item >> 6)), w = item & 63u;
    const uint32_t tx = opaque_u(P.tiles_x), ty = tile / tx;
    r.u = (tile - ty * tx) * 8u + (w & 7u);
    r.lr = ty * 8u + (w >> 3);
    const uint32_t br = opaque_u(P.band_rows);
    uint32_t band = r.lr / br;
    r.v = (band * P.world + P.rank) * br + (r.lr - band * br);
    r.valid = r.u < P.width && r.lr < P.rows_local && r.v < P.height;
    return r;
}

// level-0 item t of a frame batch -> (frame, item within the frame).  P.l0_interleave (the
// default): 64-item tiles dealt to the frames in turn (tile k of every frame side by side),
// so that concurrent level-0 waves of a batch trace the same place; else frame-major
__device__ __forceinline__ uint32_t item_frame(const WaveParams& P, uint32_t t, uint32_t& local) {
    if (P.frames <= 1) {
        local = t;
        return 0u;
    }
    if (P.l0_interleave) {  // (the tile is wave-uniform: pixel_of)
        const uint32_t tile = (uint32_t)__builtin_amdgcn_readfirstlane((int)(t >> 6)), nf = opaque_u(P.frames);
        const uint32_t q = tile / nf, fr = tile - q * nf;
        local = (q << 6) | (t & 63u);
        return fr;
    }
    const uint32_t fi = opaque_u(P.frame_items);
    const uint32_t fr = t / fi;
    local = t - fr * fi;
    return fr;
}

// rt_render_spp's counter hash (include/rt_api.h): jitter in [0, 1) of sample k of a
// pixel along dimension dim (0: x, 1: y); 24-bit fractions, exact in f32
__device__ __forceinline__ uint32_t spp_mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ float spp_jitter(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t dim) {
    uint32_t h = spp_mix32(spp_mix32(seed ^ 0x9e3779b9u) ^ pixel);
    h = spp_mix32(h ^ spp_mix32(2u * sample + dim + 1u));
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ uint32_t spread5(uint32_t v) {  // abcde -> a..b..c..d..e
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}
// Queue keys order the queues and nothing else (a key never reaches a result), so their
// arithmetic takes the hardware's approximate reciprocal and square root instead of the
// correctly rounded sequences the render's own arithmetic needs (measured flat against the
// exact forms, round 5)
__device__ __forceinline__ float key_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float key_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ uint32_t morton15(const DevScene& S, V3 p) {
    float sc = 16.f * key_rcp(opaque_f(S.bvh_r));
    int x = (int)fminf(fmaxf((p.x - S.bvh_cx) * sc + 16.f, 0.f), 31.f);
    int y = (int)fminf(fmaxf((p.y - S.bvh_cy) * sc + 16.f, 0.f), 31.f);
    int z = (int)fminf(fmaxf((p.z - S.bvh_cz) * sc + 16.f, 0.f), 31.f);
    return (spread5((uint32_t)x) << 2) | (spread5((uint32_t)y) << 1) | spread5((uint32_t)z);
}
__device__ __forceinline__ uint32_t octant(V3 d) {
    return (d.x < 0.f ? 1u : 0u) | (d.y < 0.f ? 2u : 0u) | (d.z < 0.f ? 4u : 0u);
}
__device__ __forceinline__ uint32_t spread6(uint32_t v) {  // abcdef -> a..b..c..d..e..f
    v = (v | (v << 8)) & 0x0000F00Fu;
    v = (v | (v << 4)) & 0x000C30C3u;
    v = (v | (v << 2)) & 0x00249249u;
    return v;
}
// 18-bit Morton code over the 64^3 grid of the same cube
__device__ __forceinline__ uint32_t morton18(const DevScene& S, V3 p) {
    float sc = 32.f * key_rcp(opaque_f(S.bvh_r));
    int x = (int)fminf(fmaxf((p.x - S.bvh_cx) * sc + 32.f, 0.f), 63.f);
    int y = (int)fminf(fmaxf((p.y - S.bvh_cy) * sc + 32.f, 0.f), 63.f);
    int z = (int)fminf(fmaxf((p.z - S.bvh_cz) * sc + 32.f, 0.f), 63.f);
    return (spread6((uint32_t)x) << 2) | (spread6((uint32_t)y) << 1) | spread6((uint32_t)z);
}

__device__ __forceinline__ uint32_t spread7(uint32_t v) {  // 7 bits -> every third bit
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}
// 21-bit Morton code over the 128^3 grid of the same cube
__device__ __forceinline__ uint32_t morton21(const DevScene& S, V3 p) {
    float sc = 64.f * key_rcp(opaque_f(S.bvh_r));
    int x = (int)fminf(fmaxf((p.x - S.bvh_cx) * sc + 64.f, 0.f), 127.f);
    int y = (int)fminf(fmaxf((p.y - S.bvh_cy) * sc + 64.f, 0.f), 127.f);
    int z = (int)fminf(fmaxf((p.z - S.bvh_cz) * sc + 64.f, 0.f), 127.f);
    return (spread7((uint32_t)x) << 2) | (spread7((uint32_t)y) << 1) | spread7((uint32_t)z);
}

// task ordering key: 16 bits (modes 0-2) or 24 bits (mode 3)
// key of a ray inside a sphere / cube (key mode 7): the flag above the outside keys' bits |
// the shape's centre (15-bit Morton) [| direction cell, frame batches]
// a batch's inside keys hold the ray's direction cell (cube face x 2x2) in their low 5 bits:
// rays leaving one shape the same way share a wave (943 / 950 / 945 vs 937 / 942 / 938
// Mpixels/s with the bits left zero)
// cube-map face of d x 4x4 cells of the face (< 96: 7 bits)
__device__ __forceinline__ uint32_t dir_cell16(V3 d) {
    float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z), u, v, m;
    uint32_t face;
    if (ax >= ay && ax >= az) { face = d.x < 0.f; u = d.y; v = d.z; m = ax; }
    else if (ay >= az) { face = 2u + (d.y < 0.f); u = d.x; v = d.z; m = ay; }
    else { face = 4u + (d.z < 0.f); u = d.x; v = d.y; m = az; }
    const float im = key_rcp(m);
    const uint32_t qu = (uint32_t)fminf(fmaxf((u * im + 1.f) * 2.f, 0.f), 3.f);
    const uint32_t qv = (uint32_t)fminf(fmaxf((v * im + 1.f) * 2.f, 0.f), 3.f);
    return (face << 4) | (qu << 2) | qv;
}
__device__ __forceinline__ uint32_t inside_key(const WaveParams& P, uint32_t center_key, V3 d) {
    if (P.task_fine == 3u) return (1u << 23) | (center_key << 8) | (dir_cell16(d) << 1);  // 24-bit, 4x4 cells
    uint32_t low = 0;
    if (P.task_fine) {
        float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z), u, v;
        uint32_t face;
        if (ax >= ay && ax >= az) { face = d.x < 0.f; u = d.y; v = d.z; }
        else if (ay >= az) { face = 2u + (d.y < 0.f); u = d.x; v = d.z; }
        else { face = 4u + (d.z < 0.f); u = d.x; v = d.y; }
        low = (face << 2) | ((u > 0.f ? 1u : 0u) << 1) | (v > 0.f ? 1u : 0u);
    }
    if (P.task_fine == 2u) return (1u << 23) | (center_key << 8) | (low << 3);  // 24-bit keys
    return P.task_fine ? (1u << 20) | (center_key << 5) | low : (1u << 15) | center_key;
}
__device__ __forceinline__ uint32_t task_key(const WaveParams& P, V3 o, V3 d) {
    if (P.key_mode == 0) return (octant(d) << 13) | (morton15(P.S, o) >> 2);  // 16 bits: 2 radix passes
    // cube-map face of d (3 bits) x 2x2 cells of the face (2 bits) | 13-bit coarse origin
    float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    uint32_t face;
    float u, v, m;
    if (ax >= ay && ax >= az) { face = d.x < 0.f; u = d.y; v = d.z; m = ax; }
    else if (ay >= az) { face = 2u + (d.y < 0.f); u = d.x; v = d.z; m = ay; }
    else { face = 4u + (d.z < 0.f); u = d.x; v = d.y; m = az; }
    if (P.key_mode >= 5 && P.key_mode <= 7) {  // Morton of a point ahead on the ray
        const float ahead = opaque_f(P.key_ahead) * P.S.bvh_r;
        const V3 q = add(o, mul(d, ahead));
        uint32_t cu = u > 0.f ? 1u : 0u, cv = v > 0.f ? 1u : 0u;
        uint32_t dir = (face << 2) | (cu << 1) | cv;
        if (P.key_mode == 7) {  // 15 bits (20 when task_fine): the bit above marks inside rays
            if (P.task_fine == 2u) return (dir << 18) | morton18(P.S, q);  // 24-bit keys (23 used outside)
            if (P.task_fine == 3u) return (dir_cell16(d) << 16) | (morton18(P.S, q) >> 2);  // 4x4 cells | 16-bit Morton
            if (P.task_fine) return (dir << 15) | morton15(P.S, q);
            return (dir << 10) | (morton15(P.S, q) >> 5);
        }
        return (dir << 11) | (morton15(P.S, q) >> 4);
    }
    if (P.key_mode >= 3) {  // face x 8x8 cells (< 384) and the 15-bit Morton origin
        float iu = u / m, iv = v / m;  // in [-1, 1]
        uint32_t qu = (uint32_t)fminf(fmaxf((iu + 1.f) * 4.f, 0.f), 7.f);
        uint32_t qv = (uint32_t)fminf(fmaxf((iv + 1.f) * 4.f, 0.f), 7.f);
        uint32_t dir = (face << 6) | (qu << 3) | qv;
        if (P.key_mode == 4) return (morton15(P.S, o) << 9) | dir;  // origin-major
        return (dir << 15) | morton15(P.S, o);
    }
    if (P.key_mode == 2) {  // face x 4x4 cells (< 96) | 9-bit coarse origin
        float iu = u / m, iv = v / m;  // in [-1, 1]
        uint32_t qu = (uint32_t)fminf(fmaxf((iu + 1.f) * 2.f, 0.f), 3.f);
        uint32_t qv = (uint32_t)fminf(fmaxf((iv + 1.f) * 2.f, 0.f), 3.f);
        uint32_t dir = (face << 4) | (qu << 2) | qv;
        return (dir << 9) | (morton15(P.S, o) >> 6);
    }
    uint32_t cu = u > 0.f ? 1u : 0u, cv = v > 0.f ? 1u : 0u;
    uint32_t dir = (face << 2) | (cu << 1) | cv;   // < 24
    return (dir << 11) | (morton15(P.S, o) >> 4);
}

// Per-block accumulation of the kernels' counters: each wave adds into LDS, then the
// block adds once per counter to global memory (RT_OPS_N scan counters in the block's
// scan_ops slot, then node / shadow / pixel ray counts).  Every wave of a frame adding
// to the same few addresses serialised in L2 (~2 ms per 1080p frame).
constexpr int RT_BC_N = RT_OPS_N + 3;
__shared__ unsigned long long rt_block_counts[RT_BC_N];

__device__ __forceinline__ void bc_init() {
    if (threadIdx.x < RT_BC_N) rt_block_counts[threadIdx.x] = 0ull;
    __syncthreads();
}
__device__ __forceinline__ void bc_add(int i, uint32_t v) {  // one lane per wave
    if (v) atomicAdd(&rt_block_counts[i], (unsigned long long)v);
}
__device__ __forceinline__ void bc_flush(unsigned long long* ops, unsigned long long* rays) {
    __syncthreads();
    if (threadIdx.x < RT_BC_N) {
        unsigned long long v = rt_block_counts[threadIdx.x];
        if (v) {
            if (threadIdx.x < RT_OPS_N) {
                if (ops) atomicAdd(ops + threadIdx.x, v);
            } else if (rays) {
                atomicAdd(rays + (threadIdx.x - RT_OPS_N), v);
            }
        }
    }
}
__device__ __forceinline__ void bc_scan(const ScanCnt& c) {
    bc_add(RT_OPS_NODE, c.node);
    bc_add(RT_OPS_DSPH, c.dsph);
    bc_add(RT_OPS_GSPH, c.gsph);
    bc_add(RT_OPS_TRI, c.tri);
    bc_add(RT_OPS_CUBE_BOX, c.cube_box);
    bc_add(RT_OPS_CUBE, c.cube);
    bc_add(RT_OPS_GRAZE, c.graze);
    bc_add(RT_OPS_PLANE, c.plane);
    bc_add(RT_OPS_GRAZE_N, c.graze_n);
    bc_add(RT_OPS_CYC_NODE, c.cyc_node);
    bc_add(RT_OPS_CYC_LEAF, c.cyc_leaf);
    bc_add(RT_OPS_CYC_GRAZE, c.cyc_graze);
    bc_add(RT_OPS_CYC_SCAN, c.cyc_scan);
    bc_add(RT_OPS_CYC_LOAD, c.cyc_load);
    bc_add(RT_OPS_CYC_POST, c.cyc_post);
    bc_add(RT_OPS_CYC_SELF, c.cyc_self);
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    uint32_t lane = lane_id();
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Work distribution of the trace launches (Tune::sched, A/B; the shadow kernel is always
// grid-stride):
//   0  grid-stride: wave w of the grid takes chunks w, w + W, w + 2W, ... (W waves)
//   1  dynamic: every wave takes its next chunk from a work counter
//   2  block-contiguous: the blocks of one XCD cover one contiguous range of the queue,
//      each block a contiguous sub-range, its 4 waves adjacent chunks
// Measured (config 3, 1080p; round 1): 0 -> 4.94 ms, 1 -> 6.68, 2 -> 11.2; the grid-stride
// block order remapped by XCD or by co-resident blocks: 5.2 - 5.6.  Grid-stride keeps the whole
// chip on one narrow front of the sorted queue, so the hierarchy nodes and records every CU
// reads at a time are few (scalar caches and L2 stay warm).  (Round 6: the kernels compiled
// without modes 1 / 2 allocate registers differently -- 16 B more scratch in the deep-level
// instantiation, -1.1% -- so the modes stay.)
// Returns the base of the wave's iteration `it`, or >= count when done.
__device__ __forceinline__ uint32_t sched_base(const WaveParams& P, uint32_t* counter, uint32_t count, uint32_t it,
                                                  uint32_t W = 64u) {
    const uint32_t wave = threadIdx.x >> 6, waves_per_block = blockDim.x >> 6;
    if (P.sched == 1) {
        uint32_t base = 0;
        if (lane_id() == 0) base = atomicAdd(counter, W);
        return (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
    }
    if (P.sched == 2) {
        const uint32_t nb = gridDim.x, per_xcd = (nb + 7u) / 8u;
        const uint32_t lb = (blockIdx.x % 8u) * per_xcd + blockIdx.x / 8u;  // XCD-major block order
        const uint32_t chunk = W * waves_per_block;
        const uint32_t iters = (count + nb * chunk - 1u) / (nb * chunk);
        if (it >= iters) return 0xFFFFFFFFu;
        return (lb * iters + it) * chunk + wave * W;
    }
    return ((blockIdx.x * waves_per_block + wave) + it * gridDim.x * waves_per_block) * W;
}

// wave-aggregated append of `n` (< 64) consecutive slots per lane to a device counter:
// one atomic per wave, slots in lane order
// ... split in two: the atomic is issued by wave_append_begin and its value read by
// wave_append_end, so that work in between overlaps its round trip (a returning append
// costs ~1.8% of the frame when waited for at once: DESIGN.md, round 5)
struct AppendTicket {
    uint32_t mine, base, first, total;
};
__device__ __forceinline__ AppendTicket wave_append_begin(uint32_t* counter, uint32_t n, uint32_t lane) {
    AppendTicket t{0u, 0u, 0u, 0u};
    uint64_t lt = lanemask_lt();
    for (int b = 0; b < 6; b++) {
        uint64_t m = __ballot((n >> b) & 1u);
        t.total += (uint32_t)__builtin_popcountll(m) << b;
        t.mine += (uint32_t)__builtin_popcountll(m & lt) << b;
    }
    if (t.total) {
        uint64_t any = __ballot(n != 0);
        t.first = (uint32_t)__builtin_ctzll(any);
        if (lane == t.first) t.base = atomicAdd(counter, t.total);
    }
    return t;
}
__device__ __forceinline__ uint32_t wave_append_end(const AppendTicket& t) {
    if (!t.total) return t.mine;
    return (uint32_t)__builtin_amdgcn_readlane((int)t.base, (int)t.first) + t.mine;
}
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, uint32_t n, uint32_t lane) {
    return wave_append_end(wave_append_begin(counter, n, lane));
}

// A node's unshadowed-light word for light li: node_lit[n] for lights 0-31, node_lit_hi for
// the rest (scenes of more than 32 lights)
__device__ __forceinline__ uint32_t* lit_word(const WaveParams& P, uint32_t n, uint32_t li) {
    return li < 32u ? &P.node_lit[n] : &P.node_lit_hi[(size_t)(P.lit_words - 1u) * n + ((li >> 5) - 1u)];
}
__device__ __forceinline__ const uint32_t* lit_more(const WaveParams& P, uint32_t n) {
    return P.node_lit_hi + (size_t)(P.lit_words > 1u ? P.lit_words - 1u : 0u) * n;
}

// The shading point's own shape, tested first for its shadow rays (trace kernel): the
// same arithmetic the scan runs for it (sph_general / the triangle test; bit-identical
// results up to the sign of a zero t, which no distance test can see).  Cubes are left
// to the shadow pass.
template <class C>
__device__ __forceinline__ void own_shape_test(const DevScene& S, uint32_t key, V3 o, V3 d, float& bt, uint32_t& bk,
                                               C& c) {
    const ShapeRec& R = S.shapes[key >> 4];
    if (R.kind == RT_SHAPE_SPHERE) {
        RT_OPS(c, gsph);
        Rec16 q;
        q.r0 = ld4(R.inv);
        q.r1 = ld4(R.inv + 4);
        q.r2 = ld4(R.inv + 8);
        q.rk = make_float4(__uint_as_float(key & ~15u), 0.f, 0.f, 0.f);
        sph_general(q, o, d, bt, bk);
    } else if (R.kind == RT_SHAPE_TRIANGLE) {
        RT_OPS(c, tri);
        float t, u, v, det;
        if (tri_hit(o, d, v3(R.a[0], R.a[1], R.a[2]), v3(R.a[3], R.a[4], R.a[5]), v3(R.a[6], R.a[7], R.a[8]), t, u,
                    v, det))
            take(t, key & ~15u, bt, bk);
    }
}

// Waves per SIMD of the walk kernels: 5 at 96 VGPRs (re-measured every round: 4 and 6 waves
// lose 1 - 3% for every instantiation; DESIGN.md "Kernels and occupancy")
constexpr int TRACE_WAVES = 5, SHADOW_WAVES = 5, COMBINE_WAVES = 5;
extern __shared__ float4 rt_dyn_lds[];

// DEEP: a level past the pixels and the inline shadow scans (level >= max(1, inline_levels)):
// the instantiation without their code (fewer live registers across the walk).  FIRST:
// level 0 only (its rays start at the camera: no task loads, no ray inside a shape).
template <bool COUNT, bool LDS, bool DEEP = false, bool FIRST = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TRACE_WAVES, 8))) void trace_level_kernel(
    WaveParams P, uint32_t level) {
    const DevScene& S = P.S;
    if (LDS) {  // stage the hierarchy's node records in LDS
        for (int i = threadIdx.x; i < 4 * S.n_bvh_nodes; i += blockDim.x) rt_dyn_lds[i] = S.bvh_nodes[i];
        // ... followed by the grazing pairs' normals for per-lane grazing sets
        if (S.graze_lane && S.graze_res)
            for (int i = threadIdx.x; i < 8 * S.n_graze_blk; i += blockDim.x)
                rt_dyn_lds[4 * S.n_bvh_nodes + i] = S.graze_pn[i];
        // ... then the hierarchy's sphere pairs (rt_scan.hpp run_dsph_lds)
        {
            float4* dst = rt_dyn_lds + 4 * S.n_bvh_nodes + ((S.graze_lane && S.graze_res) ? 8 * S.n_graze_blk : 0);
            for (int i = threadIdx.x; i < 4 * S.n_dsph_bvh; i += blockDim.x) dst[i] = S.dsph[i];
        }
        __syncthreads();
    }
    lfloat4* lnodes = (lfloat4*)rt_dyn_lds;
    const uint32_t off = P.levels[2 * level];
    const uint32_t count = min(P.levels[2 * level + 1], off < P.capacity ? P.capacity - off : 0u);
    const uint32_t next_off = off + count;
    if (blockIdx.x == 0 && threadIdx.x == 0) P.levels[2 * (level + 1)] = next_off;
    const uint32_t lane = lane_id();
    uint32_t n_node = 0, n_pix = 0, n_pre = 0;
    typename std::conditional<COUNT, ScanCnt, NoCnt>::type cnt;
    if constexpr (COUNT) cnt_init(cnt);
    bc_init();
    // point lights: one shadow ray each per hit (mod.rs:189-206); ambient lights: none

    // Task width: a level with fewer tasks than wave slots runs one task per wave and its
    // time is the slowest wave's walk, not a throughput; narrower tasks (fewer rays per
    // wave, the rest of the lanes idle) shorten that walk while slots are left over.
    uint32_t W = 64u;
    {
        const float slots = (float)(gridDim.x * (blockDim.x >> 6));
        while (W > P.task_w_min && (float)count < P.task_w_fill * slots * (float)W) W >>= 1;
    }
    // whole waves iterate together (the wave-aggregated appends see every lane)
    // key mode 7 (not for ray forests, whose tasks carry the pixel itself): a task of a ray
    // inside a sphere / cube carries that shape + 1 in the pixel word's low bits
    const bool inside_keys = P.key_mode == 7 && !P.node_pixel;
    // sorted levels, grid-stride: this lane's next permutation entry is requested one
    // iteration ahead, so a task costs one dependent load (the task), not two
    const bool pf_on = level > 0 && P.perm && P.sched == 0;
    const uint32_t pf_stride = gridDim.x * (blockDim.x >> 6) * W;
    uint32_t pf_slot = 0;
    bool pf_have = false;
#if RT_TASK_CLOCK
    // tools/trace_tail.py: each task's wall time (from this iteration's start to the next's),
    // the mean distance of its origins from the scene ball's centre (scene radii), its lanes
    uint32_t* tclk = level < 16u ? rt_trace_clock + level * (4u + 4u * RT_TRACE_CLOCK_TASKS) : nullptr;
    if (tclk && blockIdx.x == 0 && threadIdx.x == 0) {
        tclk[0] = count;
        tclk[1] = gridDim.x * (blockDim.x >> 6);
        tclk[2] = W;
    }
    uint64_t tc_prev = wall_clock64();
    uint32_t tc_task = 0xFFFFFFFFu, tc_lanes = 0;
    float tc_dmean = 0.f;
#endif
    for (uint32_t it = 0;; ++it) {
        const uint32_t base = sched_base(P, &P.levels[RT_WORK_WORD(level)], count, it, W);
#if RT_TASK_CLOCK
        {
            const uint64_t now = wall_clock64();
            if (tclk && tc_task < RT_TRACE_CLOCK_TASKS && lane == 0) {
                uint32_t* rec = tclk + 4u + 4u * tc_task;
                rec[0] = (uint32_t)(now - tc_prev);
                rec[1] = __float_as_uint(tc_dmean);
                rec[2] = tc_lanes;
                rec[3] = it;
            }
            tc_prev = now;
            tc_task = base < count ? base / W : 0xFFFFFFFFu;
        }
#endif
        if (base >= count) {
            if (P.sched == 2 && base != 0xFFFFFFFFu) continue;  // a block's tail past the queue end
            break;
        }
        const uint32_t t = base + lane;
        bool active = lane < W && t < count;
        uint32_t pf_next = 0;
        if (pf_on) {
            const uint32_t tn = t + pf_stride;
            pf_next = (lane < W && tn < count) ? P.perm[off + tn] : 0u;
        }
        typedef decltype(cnt) CntT;
        RT_T0(CntT, t_load);
        V3 ro = v3(0, 0, 0), rd = v3(0, 0, 0);
        uint32_t parent = 0, pix = 0, in_shape = 0;
        const uint32_t n = off + t;
        if (active) {
            if (FIRST || (!DEEP && level == 0)) {
                uint32_t local;
                const uint32_t fr = item_frame(P, t, local);
                PixelRef px = pixel_of(P, local);
                if (!px.valid) {
                    P.node_flags[n] = NODE_NONE;
                    active = false;
                } else {
                    n_pix++;
                    pix = px.v * P.width + px.u;
                    if (P.depth == 0) {  // trace_ray(.., 0) == BLACK, no scan
                        P.node_flags[n] = NODE_MISS;
                        active = false;
                    } else {
                        float fu = (float)px.u, fv = (float)px.v;
                        if (P.spp > 1) {  // sample `P.sample` (+ frame: a sample batch) of the pixel: (u + jx, v + jy)
                            const uint32_t smp = P.sample + (P.spp_batch ? fr : 0u);
                            fu = fu + spp_jitter(P.seed, pix, smp, 0u);
                            fv = fv + spp_jitter(P.seed, pix, smp, 1u);
                        }
                        // the frame's camera (cams[0] = the camera when frames == 1); a
                        // wave's 64 items are one tile of one frame: fr is wave-uniform
                        const FrameCam& C = P.cams[__builtin_amdgcn_readfirstlane(fr)];
                        float x = C.x_min + fu * C.x_delta;
                        float y = C.y_max - fv * C.y_delta;
                        V3 cam = v3(C.ox, C.oy, C.oz);
                        ro = cam;
                        rd = norm(sub(v3(x, y, 0.f), cam));
                        pix |= fr << RT_FRAME_SHIFT;  // children carry the frame
                    }
                }
            } else {
                const Task& T = P.tasks[P.perm ? (pf_have ? pf_slot : P.perm[n]) : n];
                ro = v3(T.ox, T.oy, T.oz);
                rd = v3(T.dx, T.dy, T.dz);
                parent = T.parent;
                pix = T.pixel;
                if (inside_keys) {  // a ray inside a sphere / cube: that shape + 1 below the frame bits
                    in_shape = pix & RT_INSIDE_MASK;
                    pix &= ~RT_INSIDE_MASK;
                }
            }
        }
#if RT_TASK_CLOCK
        {
            const float dx = ro.x - S.bvh_cx, dy = ro.y - S.bvh_cy, dz = ro.z - S.bvh_cz;
            float dd = active ? sqrtf(dx * dx + dy * dy + dz * dz) / S.bvh_r : 0.f;
            for (int o = 32; o > 0; o >>= 1) dd += __shfl_xor(dd, o);
            tc_lanes = (uint32_t)__builtin_popcountll(__ballot(active)) | ((in_shape ? 1u : 0u) << 16);
            tc_dmean = dd / (float)max(tc_lanes & 0xFFFFu, 1u);
        }
#endif
        bool want_refl = false, want_refr = false, hit = false;
        bool refl_in = false, refr_in = false;  // the child starts inside the hit sphere / cube
        uint32_t hit_flags = 0;  // node_flags of a hit, F_HAS_R / F_HAS_T added once queued
        uint32_t decided = 0;  // point lights whose shadow ray the own-shape test settled
        uint32_t mort = 0;  // Morton code of the shadow-ray origin (queue ordering key)
        V3 rro = v3(0, 0, 0), rrd = v3(0, 0, 0), tro = v3(0, 0, 0), trd = v3(0, 0, 0);
        V3 sh_ps = v3(0, 0, 0), sh_n = v3(0, 0, 0);  // the hit's shadow-ray origin and normal
        bool sh_entering = false;
        uint32_t sh_key = 0;
        // deep levels: both appends issued and read before the wave iteration's first store.
        // Stores count in vmcnt on gfx9 and the compiler waits with vmcnt(0) once loads and
        // stores are both outstanding, so an append read after a store waits for that store's
        // acknowledgement (level 0 too: -4%, its inline scans spill the stores' data)
        constexpr bool DEFER = DEEP;
        int32_t sh_kind = 0;             // the hit shape's kind,
        uint32_t own_ck = 0;             // ... its centre key (inside keys),
        float sh_tu = 0.f, sh_tv = 0.f;  // DEFER: the hit's texture coordinates (node record)
        bool missed = false;             // ... and a miss whose stores are still to do
        uint32_t it_load = 0, it_scan0 = 0, it_self0 = 0;  // phase accounting (instrumented variant)
        uint32_t it_scan_self = 0;  // scan cycles spent inside the self phase (inline shadow scans)
        if constexpr (CntT::kCount) {
            it_load = rt_clock() - t_load;
            cnt.cyc_load += it_load;
            it_scan0 = cnt.cyc_scan;
            it_self0 = cnt.cyc_self;
        }
        if (active) {
            n_node++;
            float bt = __builtin_huge_valf();
            uint32_t bk = 0xFFFFFFFFu;
            bool buf_ok = false;
            uint32_t buf_leaf = 0;
            if (!FIRST && in_shape) {  // the enclosing sphere first: its exit point bounds the walk from the start
                const ShapeRec& R = S.shapes[in_shape - 1u];
                if (R.kind == RT_SHAPE_SPHERE) {
                    RT_OPS(cnt, gsph);
                    Rec16 q;
                    q.r0 = ld4(R.inv);
                    q.r1 = ld4(R.inv + 4);
                    q.r2 = ld4(R.inv + 8);
                    q.rk = make_float4(__uint_as_float((in_shape - 1u) << 4), 0.f, 0.f, 0.f);
                    sph_general(q, ro, rd, bt, bk);
                    if (R.pad1 && bt < __builtin_huge_valf()) {  // segment in the ball: its shape buffer
                        const V3 c = v3(R.a[0], R.a[1], R.a[2]);
                        const float rc2 = R.a[3] * R.a[3];
                        buf_ok = len2(sub(ro, c)) <= rc2 && len2(sub(add(ro, mul(rd, bt)), c)) <= rc2;
                        buf_leaf = (uint32_t)R.pad1 - 1u;
                    }
                }
            }
            if (FIRST)
                scan_from<LDS>(S, ro, rd, bt, bk, cnt, lnodes);
            else
                scan_buffered<LDS>(S, ro, rd, bt, bk, cnt, lnodes, buf_ok, buf_leaf);
            if (bk == 0xFFFFFFFFu) {
                // trace_ray -> BLACK: the parent's child slot gets BLACK (forest: direction 0)
                if constexpr (DEFER) {
                    missed = true;
                } else {
                    P.node_flags[n] = NODE_MISS;
                    if (level > 0) {
                        P.node_ec[parent] = make_float4(0.f, 0.f, 0.f, 0.f);
                        if (P.node_dc) P.node_dc[parent] = make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                }
            } else {
                hit = true;
                // the hit shape's record whole, then its material whole: two round trips
                const ShapeW SR = load_shape(S.shapes, bk >> 4);
                const MatRec M = load_mat(S.mats, (uint32_t)SR.mat());
                Hit h = hit_attrs_w(S, SR, bk, ro, rd, M.kind == RT_MAT_TEXTURE_PHONG);
                float ri = M.refraction_index;
                float n1 = h.entering ? 1.f : ri;
                float n2 = h.entering ? ri : 1.f;
                V3 ps = add(h.p, mul(h.n, 0.0002f));  // render.rs:147
                if (P.shadow_keys)
                    mort = P.shadow_fine == 21u ? morton21(S, ps) : (P.shadow_fine ? morton18(S, ps) : morton15(S, ps));
#if RT_DIAG
                {  // hit points outside the Morton cube (clamped to its faces)
                    const float dx = fabsf(ps.x - S.bvh_cx), dy = fabsf(ps.y - S.bvh_cy), dz = fabsf(ps.z - S.bvh_cz);
                    const bool out = fmaxf(dx, fmaxf(dy, dz)) > S.bvh_r;
                    atomicAdd(&rt_scan_stats[11 + (out ? 1 : 0)], 1ull);
                    if (level == 0) atomicAdd(&rt_scan_stats[13 + (out ? 1 : 0)], 1ull);
                }
#endif
                // PointLight::get_energy (mod.rs:189-206) decided here when the planes and
                // the shape just hit settle it: a plane's t < 0 is the nearest hit; else any
                // hit nearer than the light means the nearest one is too (shadow_scan)
                sh_ps = ps;
                sh_n = h.n;
                sh_entering = h.entering;
                sh_key = bk;
                // the shape's kind and centre key from its record now: no load after the
                // iteration's first store (it would wait for that store's acknowledgement)
                sh_kind = SR.kind();
                own_ck = __float_as_uint(SR.w[0].z);
                if constexpr (DEFER) {
                    sh_tu = h.tu;
                    sh_tv = h.tv;
                }
                if (P.node_dc) {  // ray forest: the shape id as the reference records it, the pixel
                    uint32_t shape = bk >> 4;
                    P.node_key[n] = (S.shapes[shape].kind == RT_SHAPE_CUBE) ? (bk & 15u) : shape;
                    P.node_pixel[n] = pix;
                }
                const bool child_ok = level + 1 < P.depth;
                if (inside_keys) {  // closed shapes: refraction enters from outside, reflection stays inside
                    const int32_t kind = sh_kind;
                    const bool closed = kind == RT_SHAPE_SPHERE || kind == RT_SHAPE_CUBE;
                    refr_in = closed && h.entering;
                    refl_in = closed && !h.entering;
                }
                if (M.reflectivity > RT_EPS && child_ok) {  // render.rs:70-84, reflect_ray :105-110
                    rrd = reflect_dir(rd, h.n);
                    rro = add(h.p, mul(rrd, 0.0002f));
                    want_refl = true;
                }
                if (ri > RT_EPS && child_ok && refract_dir(rd, h.n, n1, n2, trd)) {  // render.rs:86-98, :112-125
                    tro = add(h.p, mul(trd, 0.0002f));
                    want_refr = true;
                }
                // the node record: what the combine pass cannot re-derive (rt_device.hpp)
                hit_flags = NODE_HIT | (h.entering ? F_ENTER : 0u) | ((uint32_t)h.mat << F_MAT_SHIFT);
                if constexpr (!DEFER) {
                    P.node_ps[n] = make_float4(ps.x, ps.y, ps.z, h.tu);
                    P.node_n[n] = make_float4(h.n.x, h.n.y, h.n.z, h.tv);
                    P.node_d[n] = make_float4(rd.x, rd.y, rd.z, __uint_as_float(parent));
                }
            }
        }
        // ---- children -> level k+1 queue
        const uint32_t nc = (want_refl ? 1u : 0u) + (want_refr ? 1u : 0u);
        // my: the lane's first child slot past next_off (wave_append_end)
        auto write_children = [&](uint32_t my) {
        const uint32_t fkey = (P.frames > 1 && P.frame_keys) ? ((pix >> RT_FRAME_SHIFT) << P.task_frame_shift) : 0u;
        // inside keys: the children carry the frame bits and the enclosing shape + 1
        const uint32_t cpix = inside_keys ? (pix & ~RT_INSIDE_MASK) : pix, own = sh_key >> 4;
        if (want_refl) {
            uint32_t slot = next_off + my;
            if (slot < P.capacity) {
                Task T = {rro.x, rro.y, rro.z, rrd.x, rrd.y, rrd.z, (n << 1) | 0u, refl_in ? cpix | (own + 1u) : cpix};
                P.tasks[slot] = T;
                if (P.task_keys)
                    P.task_keys[slot] = (refl_in ? inside_key(P, own_ck, rrd) : task_key(P, rro, rrd)) | fkey;
                hit_flags |= F_HAS_R;
            } else {
                atomicOr(P.overflow, 1u);
            }
            my++;
        }
        if (want_refr) {
            uint32_t slot = next_off + my;
            if (slot < P.capacity) {
                Task T = {tro.x, tro.y, tro.z, trd.x, trd.y, trd.z, (n << 1) | 1u, refr_in ? cpix | (own + 1u) : cpix};
                P.tasks[slot] = T;
                if (P.task_keys)
                    P.task_keys[slot] = (refr_in ? inside_key(P, own_ck, trd) : task_key(P, tro, trd)) | fkey;
                hit_flags |= F_HAS_T;
            } else {
                atomicOr(P.overflow, 1u);
            }
        }
        if (hit) P.node_flags[n] = hit_flags;
        };
        // ---- shadow rays the own shape decides, and (levels < inline_levels) the rest:
        // after the node record and the children are out, so that little stays live
        // across the shadow scans (DEFER: before the appends and every store)
        uint32_t lit_pre = 0u;
        // lights 32 and up (scenes of more than 32 lights) are never decided here: their
        // shadow rays all go to the shadow queue, their bits start at 0 (node_lit words 1..)
        const int lights32 = min(S.n_lights, 32);
        // (a 64-bit shift: lights 32 and up read a 0 bit, undecided)
        auto undecided = [&](int li) { return !(((uint64_t)decided >> min(li, 63)) & 1u); };
        auto store_lit = [&]() { P.node_lit[n] = lit_pre; };  // (node_lit_hi: zeroed per pass by the host)
        auto self_tests = [&]() {
        if (hit) {
            if constexpr (CntT::kCount) it_scan_self = cnt.cyc_scan;
            RT_T0(CntT, t_self);
            if (P.self_shadow) {
                // the own shape can only shadow a light behind the offset point's
                // surface (or any light, from inside a sphere); elsewhere the test is
                // skipped (never deciding is always exact: the shadow pass decides)
                const uint32_t own_kind = (uint32_t)sh_kind;
                const bool own_any = own_kind == RT_SHAPE_SPHERE && !sh_entering;
                const bool own_ok = own_kind == RT_SHAPE_SPHERE || own_kind == RT_SHAPE_TRIANGLE;
                for (int li = 0; li < lights32; ++li) {
                    const LightRec L = light_at(S, li);
                    if (L.kind != RT_LIGHT_POINT) continue;
                    const V3 lpos = v3(L.px, L.py, L.pz);
                    if (!own_ok || !(own_any || dot(sub(lpos, sh_ps), sh_n) <= 0.f)) continue;
                    const V3 ldir = norm(sub(lpos, sh_ps));  // mod.rs:191
                    const float l2 = len2(sub(lpos, sh_ps));
                    float st = __builtin_huge_valf();
                    uint32_t sk = 0xFFFFFFFFu;
                    planes(S, sh_ps, ldir, st, sk, cnt);
                    if (!(st < 0.f)) own_shape_test(S, sh_key, sh_ps, ldir, st, sk, cnt);
                    if (shadow_decided(sh_ps, ldir, st, l2)) {
                        decided |= 1u << li;
                        if (!shadow_hit(sh_ps, ldir, st, l2)) lit_pre |= 1u << li;
                    }
                }
                n_pre += (uint32_t)__builtin_popcount(decided);
            }
            if (!DEEP && level < P.inline_levels) {  // the level's remaining shadow rays, right here
                for (int li = 0; li < lights32; ++li) {
                    const LightRec L = light_at(S, li);
                    if (L.kind != RT_LIGHT_POINT || ((decided >> li) & 1u)) continue;
                    // the origin re-read per light: what the scan derives from it alone (o +- h,
                    // |o|) is recomputed instead of hoisted out of this loop and spilled
                    const V3 ps = opaque_v3(sh_ps);
                    const V3 lpos = v3(L.px, L.py, L.pz);
                    const V3 ldir = norm(sub(lpos, ps));  // mod.rs:191
                    if (!shadow_scan<LDS>(S, ps, ldir, lpos, cnt, lnodes, L.lb_base)) lit_pre |= 1u << li;
                    decided |= 1u << li;
                    n_pre++;
                }
            }
            RT_T1(CntT, cnt, cyc_self, t_self);
            if constexpr (CntT::kCount) it_scan_self = cnt.cyc_scan - it_scan_self;
            if constexpr (!DEFER) store_lit();
        }
        };
        // ---- one shadow entry per point light, grouped by light within the wave
        // ([light a: this wave's hits in lane order][light b: ...]) so that a shadow wave
        // holds rays from neighbouring points towards ONE light.  shadow_begin issues the
        // append, shadow_entries(base) writes the entries from the slot base it returned.
        uint64_t hits = 0;
        uint32_t s_first = 0, s_raw = 0;
        auto shadow_begin = [&]() {
            hits = __ballot(hit);
            if (hits) {
                // entries still to trace: per point light, the hit lanes it was not decided for
                uint32_t total = 0;
                for (int li = 0; li < S.n_lights; ++li)
                    if (light_at(S, li).kind == RT_LIGHT_POINT)
                        total += (uint32_t)__builtin_popcountll(__ballot(hit && undecided(li)));
                s_first = (uint32_t)__builtin_ctzll(hits);
                if (lane == s_first && total) s_raw = atomicAdd(&RT_SHADOW_COUNT(P), total);
            }
        };
        auto shadow_base = [&]() -> uint32_t {
            if (!hits) return s_raw;
            return (uint32_t)__builtin_amdgcn_readlane((int)s_raw, (int)s_first);
        };
        auto shadow_entries = [&](uint32_t sbase) {
        if (hits) {
            uint32_t group = 0;  // entries of the earlier lights
            // the key's light-buffer tier test (rt_scan.hpp lb_tier): D once per lane
            const float key_d = P.shadow_cell ? key_sqrt(len2(v3(sh_ps.x - S.bvh_cx, sh_ps.y - S.bvh_cy,
                                                                     sh_ps.z - S.bvh_cz))) + S.bvh_r
                                              : 0.f;
            for (int li = 0; li < S.n_lights; ++li) {
                if (light_at(S, li).kind != RT_LIGHT_POINT) continue;
                const bool want = hit && undecided(li);
                const uint64_t m = __ballot(want);
                const uint32_t slot = sbase + group + (uint32_t)__builtin_popcountll(m & lanemask_lt());
                group += (uint32_t)__builtin_popcountll(m);
                if (want) {
                    if (slot < P.shadow_capacity) {
                        if (P.shadow_light) {  // wide entries (> 256 lights)
                            P.shadow[slot] = n;
                            P.shadow_light[slot] = (uint32_t)li;
                        } else {
                            P.shadow[slot] = (n << P.light_bits) | (uint32_t)li;
                        }
                        if (P.shadow_keys) {
                            uint32_t low = mort;
                            if (P.shadow_cell) {
                                // the light-buffer cell this shadow ray will test (its direction
                                // seen from the light), or flag | Morton for rays that walk
                                // (the cell of the unnormalised direction: lb_cell divides by the
                                // largest component, so the length cancels up to rounding)
                                const LightRec L = light_at(S, li);
                                const V3 raw = sub(v3(L.px, L.py, L.pz), sh_ps);
                                const float l2 = len2(raw);
                                const V3 dir = neg(raw);
                                const bool lb = lb_tier_at(S, L.lb_base, key_d, l2) >= 0;
                                if (!lb) {
                                    low = P.shadow_walk_flag |
                                          (P.shadow_fine >= 19u ? mort << (P.shadow_fine - 19u) : mort >> (19u - P.shadow_fine));
                                } else if (P.shadow_cell == 2u) {  // cell | 3-bit distance from the light
                                    const float dl = key_sqrt(l2) * (8.f / RT_LB_LMAX);
                                    low = (lb_cell(S.lb_res, dir) << 3) | (uint32_t)fminf(dl, 7.f);
                                } else if (P.shadow_cell == 4u) {  // cell | 7-bit distance (24-bit keys)
                                    const float dl = key_sqrt(l2) * (128.f / RT_LB_LMAX);
                                    low = (lb_cell(S.lb_res, dir) << 7) | (uint32_t)fminf(dl, 127.f);
                                } else if (P.shadow_cell == 3u) {  // cell | 4-bit distance (frame batches)
                                    const float dl = key_sqrt(l2) * (16.f / RT_LB_LMAX);
                                    low = (lb_cell(S.lb_res, dir) << 4) | (uint32_t)fminf(dl, 15.f);
                                } else {
                                    low = lb_cell(S.lb_res, dir);
                                }
                                if (lb) low |= P.shadow_lb_flag;
                            }
                            P.shadow_keys[slot] = (P.shadow_fine ? (((uint32_t)li << P.shadow_li_shift) | low)
                                                                   : ((uint32_t)li << P.light_shift) | (mort >> (15u - P.light_shift)))
                                                  | ((P.frames > 1 && P.frame_keys) ? ((pix >> RT_FRAME_SHIFT) << P.shadow_frame_shift) : 0u);
                        }
                    } else
                        atomicOr(P.overflow, 2u);
                }
            }
        }
        };
        if constexpr (DEFER) {
            // every load and both appends' values first, then the stores
            self_tests();
            const AppendTicket child_ticket = wave_append_begin(&P.levels[2 * (level + 1) + 1], nc, lane);
            shadow_begin();
            const uint32_t my = wave_append_end(child_ticket);
            const uint32_t sbase = shadow_base();
            write_children(my);
            if (hit) {
                P.node_ps[n] = make_float4(sh_ps.x, sh_ps.y, sh_ps.z, sh_tu);
                P.node_n[n] = make_float4(sh_n.x, sh_n.y, sh_n.z, sh_tv);
                P.node_d[n] = make_float4(rd.x, rd.y, rd.z, __uint_as_float(parent));
                store_lit();
            } else if (missed) {
                P.node_flags[n] = NODE_MISS;
                if (level > 0) {
                    P.node_ec[parent] = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (P.node_dc) P.node_dc[parent] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
            shadow_entries(sbase);
        } else {
            const AppendTicket child_ticket = wave_append_begin(&P.levels[2 * (level + 1) + 1], nc, lane);
            write_children(wave_append_end(child_ticket));
            self_tests();
            shadow_begin();
            shadow_entries(shadow_base());
        }
        if constexpr (CntT::kCount)  // the rest of the iteration: attributes, records, children, entries
            cnt.cyc_post += (rt_clock() - t_load) - it_load - (cnt.cyc_scan - it_scan0 - it_scan_self) -
                            (cnt.cyc_self - it_self0);
        pf_slot = pf_next;
        pf_have = pf_on;
    }
    for (int o = 32; o > 0; o >>= 1) {
        n_node += __shfl_xor(n_node, o);
        n_pix += __shfl_xor(n_pix, o);
        n_pre += __shfl_xor(n_pre, o);
    }
    if (lane == 0) {
        if constexpr (COUNT) bc_scan(cnt);
        bc_add(RT_OPS_N + 0, n_node);
        bc_add(RT_OPS_N + 1, n_pre);  // shadow rays decided here count as shadow scans
        bc_add(RT_OPS_N + 2, n_pix);
    }
    bc_flush(ops_slot(S), P.ray_counters);
}

// Every shadow ray of the frame: PointLight::get_energy's scan + distance test, result as
// a bit in the node record.

// the shadow kernel stages up to this many lights in LDS
constexpr int LDS_LIGHTS = 64;
// shadow entry t of the (sorted) queue -> its node and light.  Packed: (node << light_bits) |
// light.  Wide (> 256 lights): shadow_in holds the entry's slot (or null: slot t), the node
// and light sit in shadow[slot] and shadow_light[slot].
__device__ __forceinline__ uint32_t shadow_raw(const WaveParams& P, uint32_t t) {
    return P.shadow_in ? P.shadow_in[t] : t;
}
__device__ __forceinline__ void shadow_unpack(const WaveParams& P, uint32_t e, uint32_t& n, uint32_t& li) {
    if (P.shadow_light) {
        n = P.shadow[e];
        li = P.shadow_light[e];
    } else {
        n = e >> P.light_bits;
        li = e & ((1u << P.light_bits) - 1u);
    }
}
__device__ __forceinline__ uint32_t shadow_node(const WaveParams& P, uint32_t e) {
    return P.shadow_light ? P.shadow[e] : e >> P.light_bits;
}

template <bool LDS, bool COUNT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SHADOW_WAVES, 8))) void shadow_kernel(WaveParams P) {
    const DevScene& S = P.S;
    if (LDS) {  // stage the hierarchy's node records in LDS
        for (int i = threadIdx.x; i < 4 * S.n_bvh_nodes; i += blockDim.x) rt_dyn_lds[i] = S.bvh_nodes[i];
        // ... followed by the grazing pairs' normals for per-lane grazing sets
        if (S.graze_lane && S.graze_res)
            for (int i = threadIdx.x; i < 8 * S.n_graze_blk; i += blockDim.x)
                rt_dyn_lds[4 * S.n_bvh_nodes + i] = S.graze_pn[i];
        // ... then the hierarchy's sphere pairs (rt_scan.hpp run_dsph_lds)
        {
            float4* dst = rt_dyn_lds + 4 * S.n_bvh_nodes + ((S.graze_lane && S.graze_res) ? 8 * S.n_graze_blk : 0);
            for (int i = threadIdx.x; i < 4 * S.n_dsph_bvh; i += blockDim.x) dst[i] = S.dsph[i];
        }
        __syncthreads();
    }
    // the lights' positions and light-buffer bases in LDS (an entry's light is per lane): read
    // with an LDS load, not a vector load that would wait for the previous lit-bit atomic
    __shared__ float4 lds_lights[LDS_LIGHTS];
    const bool lights_lds = S.n_lights <= LDS_LIGHTS;
    if (lights_lds) {
        for (int i = threadIdx.x; i < S.n_lights; i += blockDim.x) {
            const LightRec L = light_at(S, i);
            lds_lights[i] = make_float4(L.px, L.py, L.pz, __uint_as_float(L.lb_base));
        }
        __syncthreads();
    }
    lfloat4* lnodes = (lfloat4*)rt_dyn_lds;
    const uint32_t count = min(RT_SHADOW_COUNT(P), P.shadow_capacity);
    const uint32_t lane = lane_id();
    uint32_t n_shadow = 0;
    typename std::conditional<COUNT, ScanCnt, NoCnt>::type cnt;
    if constexpr (COUNT) cnt_init(cnt);
    bc_init();
    {
        // grid-stride, software-pipelined: the next iteration's entry is requested before this
        // iteration's scan and its origin before this iteration's lit-bit atomic, so the next
        // iteration waits neither for an HBM round trip nor for the atomic (vmcnt counts loads,
        // stores and atomics in issue order)
        const uint32_t stride = gridDim.x * (blockDim.x >> 6) * 64u;
        uint32_t base = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64u;
        uint32_t t = base + lane;
        uint32_t e = t < count ? shadow_raw(P, t) : 0u;
        float4 q = t < count ? P.node_ps[shadow_node(P, e)] : make_float4(0.f, 0.f, 0.f, 0.f);
#if RT_TASK_CLOCK
        // tools/shadow_tail.py: wall clock (100 MHz) of every 64-entry task of the queue, and the
        // distance of its origins from the scene ball's centre in scene radii (mean, max)
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            rt_shadow_clock[0] = count;
            rt_shadow_clock[1] = stride / 64u;
        }
        uint64_t tc0 = wall_clock64();
#endif
        while (base < count) {
            const uint32_t tn = t + stride;
            const uint32_t en = tn < count ? shadow_raw(P, tn) : 0u;
            bool lit = false;
            uint32_t n = 0, li = 0;
            if (t < count) shadow_unpack(P, e, n, li);
#if RT_TASK_CLOCK
            const float q0x = q.x, q0y = q.y, q0z = q.z;
#endif
            if (t < count) {
                V3 ps = v3(q.x, q.y, q.z);
                float4 lq;
                if (lights_lds) {
                    lq = lds_lights[li];
                } else {
                    const LightRec L = light_at(S, (int)li);
                    lq = make_float4(L.px, L.py, L.pz, __uint_as_float(L.lb_base));
                }
                V3 lpos = v3(lq.x, lq.y, lq.z);
                V3 ldir = norm(sub(lpos, ps));  // mod.rs:191
                n_shadow++;
                lit = !shadow_scan<LDS, decltype(cnt), true>(S, ps, ldir, lpos, cnt, lnodes, __float_as_uint(lq.w));
            }
            q = tn < count ? P.node_ps[shadow_node(P, en)] : make_float4(0.f, 0.f, 0.f, 0.f);
            if (lit) atomicOr(lit_word(P, n, li), 1u << (li & 31u));
#if RT_TASK_CLOCK
            {
                const uint64_t tc1 = wall_clock64();
                const uint32_t task = base / 64u;
                float dd = 0.f;
                if (t < count) {
                    const float dx = q0x - S.bvh_cx, dy = q0y - S.bvh_cy, dz = q0z - S.bvh_cz;
                    dd = sqrtf(dx * dx + dy * dy + dz * dz) / S.bvh_r;
                }
                float dsum = dd, dmax = dd;
                for (int o = 32; o > 0; o >>= 1) {
                    dsum += __shfl_xor(dsum, o);
                    dmax = fmaxf(dmax, __shfl_xor(dmax, o));
                }
                const uint32_t nl = (uint32_t)__builtin_popcountll(__ballot(t < count));
                if (lane == 0 && 2u + 4u * task + 3u < RT_SHADOW_CLOCK_WORDS) {
                    uint32_t* rec = rt_shadow_clock + 2u + 4u * task;
                    rec[0] = (uint32_t)(tc1 - tc0);
                    rec[1] = __float_as_uint(dsum / (float)max(nl, 1u));
                    rec[2] = __float_as_uint(dmax);
                    rec[3] = nl | (li << 8);
                }
                tc0 = tc1;
            }
#endif
            base += stride;
            t = tn;
            e = en;
        }
    }
    for (int o = 32; o > 0; o >>= 1) n_shadow += __shfl_xor(n_shadow, o);
    if (lane == 0) {
        if constexpr (COUNT) bc_scan(cnt);
        bc_add(RT_OPS_N + 1, n_shadow);
    }
    bc_flush(ops_slot(S), P.ray_counters);
}

// The stored part of a hit node (rt_device.hpp) and what the shading passes derive from it:
// eye_dir = -norm(ray direction) (the Intersection's eye_dir, sphere.rs:81 etc.), n1 / n2
// from `entering` (render.rs:51-55), the material's textures at (u, v).
struct NodeIn {
    Hit h;
    V3 ps, rd;
    float n1, n2;
    uint32_t parent;
};
__device__ __forceinline__ NodeIn node_in(float4 a, float4 b, float4 c, uint32_t flags, const MatRec& M) {
    NodeIn q;
    q.ps = xyz(a);
    q.h.n = xyz(b);
    q.rd = xyz(c);
    q.h.tu = a.w;
    q.h.tv = b.w;
    q.parent = __float_as_uint(c.w);
    q.h.eye = neg(norm(q.rd));
    const bool entering = (flags & F_ENTER) != 0u;
    const float ri = M.refraction_index;
    q.n1 = entering ? 1.f : ri;
    q.n2 = entering ? ri : 1.f;
    return q;
}

// sum over the lights of fresnel(ldir) * get_reflected_energy(E, ldir) (render.rs:59-68,
// get_light_energy :142-153), the shadow decisions taken from `litmask`; Sum starts at
// BLACK (color.rs:164-167).  ne = norm(eye_dir).
// A shadowed point light (E = BLACK) adds f * ((l.n * 0) * kd + (pw * 0) * ks), which is
// +-0 in every channel whenever f, l.n, kd, ks and (m.h)^power are finite -- and adding a
// +-0 to the running sum changes nothing: the sum starts at +0 and can never become -0
// under round-to-nearest (x + (-0) = x, +0 + (-0) = +0).  So such a light is skipped when
// the material guarantees finite terms (MatRec::dark_zero: power in [0, 1e6], n1 + n2 != 0,
// finite colours), the scene's normals are finite and bounded (DevScene::dark_skip), and the
// half vector norm(ne + norm(ldir)) cannot degenerate (ldir not within ~8 degrees of -ne;
// exactly opposite vectors give 0 / 0 = NaN, which the reference propagates).  A shadowed
// light's direction is finite: a NaN direction hits nothing, so it is never shadowed.
// (lit_more: the node's node_lit_hi words, lights 32 and up)
__device__ __forceinline__ V3 light_sum(const DevScene& S, const MatRec& M, const NodeIn& q, V3 ne, uint32_t litmask,
                                        V3 kd, V3 ks, float power, const uint32_t* lit_more) {
    V3 lsum = v3(0.f, 0.f, 0.f);
    const bool dark_ok = S.dark_skip && M.dark_zero;
    for (int li = 0; li < S.n_lights; ++li) {
        const LightRec L = light_at(S, li);
        V3 ldir = v3(0.f, 0.f, 0.f);
        V3 E = v3(L.r, L.g, L.b);
        if (L.kind == RT_LIGHT_POINT) {
            const V3 raw = sub(v3(L.px, L.py, L.pz), q.ps);
            if (!(((li < 32 ? litmask : lit_more[(li >> 5) - 1]) >> (li & 31)) & 1u)) {
                if (dark_ok) {
                    const float r2 = len2(raw), c = dot(raw, ne);
                    if (r2 > 1e-30f && r2 < 1e30f && !(c < 0.f && c * c > 0.98f * r2)) continue;
                }
                E = v3(0.f, 0.f, 0.f);
            }
            ldir = norm(raw);
        }
        float f = fresnel_reflection(ldir, q.h.n, q.n1, q.n2);
        V3 g = reflected_energy_ne(E, ldir, q.h.n, ne, kd, ks, power);
        lsum = add(lsum, v3(f * g.x, f * g.y, f * g.z));
    }
    return lsum;
}

// render.rs:57-68 + :100 for every node of `level`; children (level + 1) already reported.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(COMBINE_WAVES, 8))) void combine_level_kernel(
    WaveParams P, uint32_t level) {
    rt_pow_stage();
    const DevScene& S = P.S;
    const uint32_t off = P.levels[2 * level];
    const uint32_t count = min(P.levels[2 * level + 1], off < P.capacity ? P.capacity - off : 0u);
    const uint32_t stride = gridDim.x * blockDim.x;
    // the last launch of a pass: latch this pass's queue overflows into the sticky word
    // rt_scene_sync_status reads (every producer of the pass ran before this launch)
    if (level == 0 && blockIdx.x == 0 && threadIdx.x == 0 && P.overflow_sticky && *P.overflow)
        atomicOr(P.overflow_sticky, *P.overflow);
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < count; t += stride) {
        const uint32_t n = off + t;
        const uint32_t flags = P.node_flags[n];
        // every input of the node requested at once (one memory round trip, not three: flags,
        // then the record, then the children's colours); the slots of a miss, of padding or of
        // an absent child hold stale values that are never used.  The children's
        // colours are read only where a child was queued, together with the material record
        // that needs the flags anyway (no extra round trip; 64% of config 3's nodes have none)
        const float4 qa = P.node_ps[n], qb = P.node_n[n], qc = P.node_d[n];
        const uint32_t litmask = P.node_lit[n];
        // frame batches: level-0 node t belongs to frame t / frame_items
        uint32_t local = t;
        const uint32_t fr = level == 0 ? item_frame(P, t, local) : 0u;
        if (flags & NODE_NONE) {  // padding of the band buffer: defined as 0
            PixelRef px = pixel_of(P, local);
            if (level == 0 && px.u < P.width && px.lr < P.rows_local && !(P.direct && px.v >= P.height)) {
                const size_t i = (size_t)(P.direct ? px.v : px.lr) * P.width + px.u;
                if (P.out) {
                    float* o = P.out + (size_t)fr * P.frame_floats + i * 3u;
                    o[0] = 0.f;
                    o[1] = 0.f;
                    o[2] = 0.f;
                }
                if (P.out8) {
                    uint8_t* o8 = P.out8 + (size_t)fr * P.frame_floats + i * 3u;
                    o8[0] = o8[1] = o8[2] = 0;
                }
            }
            continue;
        }
        V3 c = v3(0.f, 0.f, 0.f);
        uint32_t parent = 0;
        if (flags & NODE_HIT) {
            const MatRec M = load_mat(S.mats, flags >> F_MAT_SHIFT);
            const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 er = (flags & F_HAS_R) ? P.node_ec[2u * n] : z4;
            const float4 et = (flags & F_HAS_T) ? P.node_ec[2u * n + 1u] : z4;
            const NodeIn q = node_in(qa, qb, qc, flags, M);
            parent = q.parent;
            const V3 ka = tex_eval(M.ambient, q.h.tu, q.h.tv);
            const V3 kd = tex_eval(M.diffuse, q.h.tu, q.h.tv);
            const V3 ks = tex_eval(M.specular, q.h.tu, q.h.tv);
            const V3 ne = norm(q.h.eye);
            const V3 lsum = light_sum(S, M, q, ne, litmask, kd, ks, M.power, lit_more(P, n));
            // ambient = mat.ambient(tex) * scene.ambient (render.rs:57), then + lights
            const V3 loc = add(v3(ka.x * S.amb_r, ka.y * S.amb_g, ka.z * S.amb_b), lsum);
            Frame f;
            node_weights(M, q.rd, q.h.n, ne, q.n1, q.n2, f);
            f.ax = loc.x; f.ay = loc.y; f.az = loc.z;
            f.kdx = kd.x; f.kdy = kd.y; f.kdz = kd.z;
            f.ksx = ks.x; f.ksy = ks.y; f.ksz = ks.z;
            // a child that was never queued (depth limit: trace_ray(.., 0)) reports BLACK
            const V3 zero = v3(0.f, 0.f, 0.f);
            c = combine(f, (flags & F_HAS_R) ? xyz(er) : zero, (flags & F_HAS_T) ? xyz(et) : zero);
        } else if (level > 0) {
            continue;  // a missed child: the trace pass wrote BLACK to its parent's slot
        }
        if (level == 0) {
            PixelRef px = pixel_of(P, local);
            const size_t i = (size_t)(P.direct ? px.v : px.lr) * P.width + px.u;
            bool last = true;
            if (P.out) {  // (null: an RGB8-only pass, spp == 1)
                float* o = P.out + (size_t)fr * P.frame_floats + i * 3u;
                if (P.spp_batch) {  // this sample's raw colour; spp_accumulate_kernel sums in sample order
                    last = false;
                } else if (P.spp > 1) {  // the f32 sum of the samples in sample order, then / spp
                    if (P.sample > 0) c = v3(o[0] + c.x, o[1] + c.y, o[2] + c.z);
                    last = P.sample + 1 == P.spp;
                    if (last) {
                        const float fs = (float)P.spp;
                        c = v3(c.x / fs, c.y / fs, c.z / fs);
                    }
                }
                o[0] = c.x;
                o[1] = c.y;
                o[2] = c.z;
            }
            if (P.out8 && last) {  // Color::as_u8 (color.rs:43-46) fused into the epilogue
                uint8_t* o8 = P.out8 + (size_t)fr * P.frame_floats + i * 3u;
                o8[0] = as_u8(c.x);
                o8[1] = as_u8(c.y);
                o8[2] = as_u8(c.z);
            }
        } else {
            P.node_ec[parent] = make_float4(c.x, c.y, c.z, 0.f);
        }
    }
}

// ---------------------------------------------------------------- ray forest
// render_ray_tree (render_tree.rs:214-255) for every node of `level`, bottom-up like the
// combine pass but with the forest's own shading, from the CURRENT materials (a material
// edited since the build shows up, as through the reference's RefCell):
//   n1, n2        from the material's refraction index and the hit's `entering`
//   lights        sum over lights of fresnel(ldir) * reflected_energy(E, ldir)  (as render.rs)
//   reflected     fresnel(dir_r) * reflected_energy(E_r, eye_dir)   -- eye_dir as light dir
//   refracted     (1 - fresnel(dir_t, -n)) * E_t                     -- no diffuse factor
//   colour        ((ambient + lights) + reflected) + refracted, reported with dir = -eye_dir
// (E, dir) of a missing child = (BLACK, 0); a missed child wrote (BLACK, 0) at build time.
// dirty != null: only nodes of marked pixels are shaded (render_forest_filter).
__global__ __launch_bounds__(256) void forest_shade_level_kernel(WaveParams P, uint32_t level, float* frame) {
    rt_pow_stage();
    const DevScene& S = P.S;
    const uint32_t off = P.levels[2 * level];
    const uint32_t count = min(P.levels[2 * level + 1], off < P.capacity ? P.capacity - off : 0u);
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < count; t += stride) {
        const uint32_t n = off + t;
        const uint32_t flags = P.node_flags[n];
        if (flags & NODE_NONE) continue;
        if (!(flags & NODE_HIT)) {  // RayTreeNode::None: (BLACK, 0)
            if (level == 0) {
                PixelRef px = pixel_of(P, t);
                uint32_t pix = px.v * P.width + px.u;
                if (!P.dirty || P.dirty[pix]) {
                    float* o = frame + (size_t)pix * 3u;
                    o[0] = 0.f;
                    o[1] = 0.f;
                    o[2] = 0.f;
                }
            }
            continue;
        }
        const uint32_t pix = P.node_pixel[n];
        if (P.dirty && !P.dirty[pix]) continue;
        const MatRec& M = S.mats[flags >> F_MAT_SHIFT];
        const NodeIn q = node_in(P.node_ps[n], P.node_n[n], P.node_d[n], flags, M);
        const V3 kd = tex_eval(M.diffuse, q.h.tu, q.h.tv), ks = tex_eval(M.specular, q.h.tu, q.h.tv);
        const V3 ne = norm(q.h.eye);
        const V3 lsum = light_sum(S, M, q, ne, P.node_lit[n], kd, ks, M.power, lit_more(P, n));
        const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
        const bool has_r = (flags & F_HAS_R) != 0u, has_t = (flags & F_HAS_T) != 0u;
        const V3 er = xyz(has_r ? P.node_ec[2u * n] : zero), dr = xyz(has_r ? P.node_dc[2u * n] : zero);
        const V3 et = xyz(has_t ? P.node_ec[2u * n + 1u] : zero), dt = xyz(has_t ? P.node_dc[2u * n + 1u] : zero);
        float fr = fresnel_reflection(dr, q.h.n, q.n1, q.n2);
        V3 gr = reflected_energy_ne(er, q.h.eye, q.h.n, ne, kd, ks, M.power);
        V3 refl = v3(fr * gr.x, fr * gr.y, fr * gr.z);
        float ft = 1.f - fresnel_reflection(dt, neg(q.h.n), q.n1, q.n2);
        V3 refr = v3(ft * et.x, ft * et.y, ft * et.z);
        V3 ka = tex_eval(M.ambient, q.h.tu, q.h.tv);
        V3 amb = v3(ka.x * S.amb_r, ka.y * S.amb_g, ka.z * S.amb_b);
        V3 c = add(add(add(amb, lsum), refl), refr);
        if (level == 0) {
            float* o = frame + (size_t)pix * 3u;
            o[0] = c.x;
            o[1] = c.y;
            o[2] = c.z;
        } else {  // the parent's slot: colour and the direction -eye_dir (render_tree.rs:252)
            const V3 d = neg(q.h.eye);
            P.node_ec[q.parent] = make_float4(c.x, c.y, c.z, 0.f);
            P.node_dc[q.parent] = make_float4(d.x, d.y, d.z, 0.f);
        }
    }
}

// mark[pixel] = 1 for every pixel whose tree holds a node with key_mask[id] set
// (render_forest_filter's shapes ∩ mutated, render_tree.rs:138-140); also counts the
// hit nodes per pixel when sizes != null (RayTree::size, :39-48)
__global__ void forest_mark_kernel(const uint32_t* node_key, const uint32_t* node_pixel, const uint32_t* node_flags,
                                   uint32_t n_nodes, const uint8_t* key_mask, uint32_t n_keys, uint8_t* mark,
                                   uint32_t* sizes) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n_nodes; i += gridDim.x * blockDim.x) {
        if (!(node_flags[i] & NODE_HIT)) continue;
        uint32_t pix = node_pixel[i];
        if (sizes) atomicAdd(&sizes[pix], 1u);
        if (key_mask) {
            uint32_t k = node_key[i];
            if (k < n_keys && key_mask[k]) mark[pix] = 1;
        }
    }
}

// levels[] = {0, total_items, 0, ...} (incl. the shadow count), overflow 0 (if given)
__global__ void wave_init_kernel(uint32_t* levels, uint32_t n_words, uint32_t total_items, uint32_t* overflow) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_words) levels[i] = (i == 1) ? total_items : 0u;
    if (i == 0 && overflow) *overflow = 0u;  // null: keep an earlier sample's overflow
}

hipError_t launch_wave_init(uint32_t* levels, uint32_t n_words, uint32_t total_items, uint32_t* overflow,
                            hipStream_t stream) {
    hipLaunchKernelGGL(wave_init_kernel, dim3((n_words + 255) / 256), dim3(256), 0, stream, levels, n_words,
                       total_items, overflow);
    return hipGetLastError();
}

// The walk kernels' LDS variant stages the hierarchy's node records, the grazing pairs'
// normals and the hierarchy's sphere pairs when they fit in 32 KB (five 256-thread blocks
// per CU, the trace kernel's VGPR limit; config 3 stages 22.5 KB, which leaves the shadow
// kernel its six); Tune::lds_nodes=0: never, =trace / =shadow: only that kernel (A/B).  The
// hierarchy's triangle pairs staged as well (27.9 KB; records from LDS in VGPRs instead of
// SGPRs, shadow kernel down to five blocks) lost 7.5%: 865 / 867 / 862 vs 936 / 932 / 933.
// kernel_bit 1: the trace kernels, 2: shadow (the same records today)
static size_t lds_bytes(const WaveParams& p, uint32_t kernel_bit) {
    (void)kernel_bit;
    return (size_t)p.S.n_bvh_nodes * 64 + ((p.S.graze_lane && p.S.graze_res) ? (size_t)p.S.n_graze_blk * 128 : 0) +
           (size_t)p.S.n_dsph_bvh * 64;
}
static bool lds_nodes_for(const WaveParams& p, uint32_t kernel_bit) {
    size_t lds = lds_bytes(p, kernel_bit);
    if (!(p.lds_mask & kernel_bit)) return false;
    return p.S.use_bvh && lds > 0 && lds <= 32 * 1024;
}

// Blocks per CU of the instantiations that launch: the LDS variants at the scene's LDS
// bytes (the persistent grids are sized from these, so that every block is resident)
hipError_t wave_occupancy(const WaveParams& p, int* trace_blocks, int* shadow_blocks, int* combine_blocks,
                          int* trace_each) {
    const size_t lds = lds_bytes(p, 1u), lds_sh = lds_bytes(p, 2u);
    const bool aware = true;  // (grids sized as if no LDS were used: blocks waited for a slot)
    // every trace instantiation launch_wave_trace may pick (generic, level 0, deep levels):
    // the grid is sized by the least occupancy among them, so every block is resident
    const bool tl = aware && lds_nodes_for(p, 1u);
    int tv[3] = {0, 0, 0};
    hipError_t e =
        tl ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&tv[0], trace_level_kernel<false, true>, 256, lds)
           : hipOccupancyMaxActiveBlocksPerMultiprocessor(&tv[0], trace_level_kernel<false, false>, 256, 0);
    if (e != hipSuccess) return e;
    e = tl ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&tv[1], trace_level_kernel<false, true, false, true>, 256, lds)
           : hipOccupancyMaxActiveBlocksPerMultiprocessor(&tv[1], trace_level_kernel<false, false, false, true>, 256, 0);
    if (e != hipSuccess) return e;
    e = tl ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&tv[2], trace_level_kernel<false, true, true>, 256, lds)
           : hipOccupancyMaxActiveBlocksPerMultiprocessor(&tv[2], trace_level_kernel<false, false, true>, 256, 0);
    if (e != hipSuccess) return e;
    *trace_blocks = std::min(tv[0], std::min(tv[1], tv[2]));
    if (trace_each)
        for (int i = 0; i < 3; i++) trace_each[i] = tv[i];
    e = aware && lds_nodes_for(p, 2u)
            ? hipOccupancyMaxActiveBlocksPerMultiprocessor(shadow_blocks, shadow_kernel<true, false>, 256, lds_sh)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(shadow_blocks, shadow_kernel<false, false>, 256, 0);
    if (e != hipSuccess) return e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(combine_blocks, combine_level_kernel, 256, 0);
#if RT_DIAG
    if (getenv("RT_OCC_DEBUG"))
        fprintf(stderr, "rt occupancy: lds %zu B (nodes %d, graze blocks %d, sphere pairs %d, tri pairs %d); blocks per CU trace %d shadow %d combine %d\n",
                lds, p.S.n_bvh_nodes, p.S.n_graze_blk, p.S.n_dsph_bvh, p.S.n_tri_bvh, *trace_blocks, *shadow_blocks, *combine_blocks);
#endif
    return e;
}

// occ_each (optional): blocks per CU of the generic / level-0 / deep instantiations, occ_min
// their least (what `blocks` was sized by): with RT_OCC_EACH=1 a launch of an instantiation
// with more resident blocks per CU gets its grid scaled up to match
hipError_t launch_wave_trace(const WaveParams& p, uint32_t level, int blocks, hipStream_t stream,
                             const int* occ_each, int occ_min) {
    const size_t lds = lds_bytes(p, 1u);
    const bool use = lds_nodes_for(p, 1u);
    // the deep instantiation past level 0 and the inline shadow levels (deep_kernel=0: never, A/B)
    const bool deep_ok = p.deep_kernel != 0;
    const bool deep = deep_ok && level > 0 && level >= p.inline_levels && !(p.count_mask & 1u);
    // occ_each=1 (builds whose instantiations differ in occupancy)
    const bool occ_each_on = p.occ_each != 0;
    if (occ_each_on && occ_each && occ_min > 0 && !(p.count_mask & 1u)) {
        const int v = (level == 0 && deep_ok) ? 1 : (deep ? 2 : 0);
        if (occ_each[v] > occ_min) blocks = (int)((long long)blocks * occ_each[v] / occ_min);
    }
    if (p.count_mask & 1u) {
        if (use)
            hipLaunchKernelGGL((trace_level_kernel<true, true>), dim3(blocks), dim3(256), lds, stream, p, level);
        else
            hipLaunchKernelGGL((trace_level_kernel<true, false>), dim3(blocks), dim3(256), 0, stream, p, level);
    } else if (level == 0 && deep_ok) {
        if (use)
            hipLaunchKernelGGL((trace_level_kernel<false, true, false, true>), dim3(blocks), dim3(256), lds, stream, p, level);
        else
            hipLaunchKernelGGL((trace_level_kernel<false, false, false, true>), dim3(blocks), dim3(256), 0, stream, p, level);
    } else if (deep) {
        if (use)
            hipLaunchKernelGGL((trace_level_kernel<false, true, true>), dim3(blocks), dim3(256), lds, stream, p, level);
        else
            hipLaunchKernelGGL((trace_level_kernel<false, false, true>), dim3(blocks), dim3(256), 0, stream, p, level);
    } else {
        if (use)
            hipLaunchKernelGGL((trace_level_kernel<false, true>), dim3(blocks), dim3(256), lds, stream, p, level);
        else
            hipLaunchKernelGGL((trace_level_kernel<false, false>), dim3(blocks), dim3(256), 0, stream, p, level);
    }
    return hipGetLastError();
}

hipError_t launch_wave_shadow(const WaveParams& p, int blocks, hipStream_t stream) {
    const size_t lds = lds_bytes(p, 2u);
    const bool use = lds_nodes_for(p, 2u);
    const bool count = (p.count_mask & 2u) != 0;
    if (use && count)
        hipLaunchKernelGGL((shadow_kernel<true, true>), dim3(blocks), dim3(256), lds, stream, p);
    else if (use)
        hipLaunchKernelGGL((shadow_kernel<true, false>), dim3(blocks), dim3(256), lds, stream, p);
    else if (count)
        hipLaunchKernelGGL((shadow_kernel<false, true>), dim3(blocks), dim3(256), 0, stream, p);
    else
        hipLaunchKernelGGL((shadow_kernel<false, false>), dim3(blocks), dim3(256), 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_forest_shade(const WaveParams& p, uint32_t level, int blocks, float* frame, hipStream_t stream) {
    hipLaunchKernelGGL(forest_shade_level_kernel, dim3(blocks), dim3(256), 0, stream, p, level, frame);
    return hipGetLastError();
}

hipError_t launch_forest_mark(const uint32_t* node_key, const uint32_t* node_pixel, const uint32_t* node_flags,
                              uint32_t n_nodes, const uint8_t* key_mask, uint32_t n_keys, uint8_t* mark,
                              uint32_t* sizes, hipStream_t stream) {
    if (n_nodes == 0) return hipSuccess;
    uint32_t blocks = std::min<uint32_t>((n_nodes + 255) / 256, 4096u);
    hipLaunchKernelGGL(forest_mark_kernel, dim3(blocks), dim3(256), 0, stream, node_key, node_pixel, node_flags, n_nodes,
                       key_mask, n_keys, mark, sizes);
    return hipGetLastError();
}

hipError_t launch_wave_combine(const WaveParams& p, uint32_t level, int blocks, hipStream_t stream) {
    hipLaunchKernelGGL(combine_level_kernel, dim3(blocks), dim3(256), 0, stream, p, level);
    return hipGetLastError();
}

}  // namespace rtdev

#if RT_TASK_CLOCK
// tools/shadow_tail.py (build: tools/build_variant.sh clock -DRT_TASK_CLOCK=1): the shadow kernel's task clock of the last pass (entries, waves of the
// grid, then per 64-entry task: 10-ns ticks, mean and max origin distance / scene radius,
// lanes | light << 8)
extern "C" int rt_debug_shadow_clock(uint32_t* out, uint32_t words) {
    if (words > RT_SHADOW_CLOCK_WORDS) words = RT_SHADOW_CLOCK_WORDS;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(rtdev::rt_shadow_clock), words * sizeof(uint32_t)) != hipSuccess;
}
// tools/trace_tail.py: the trace kernels' task clocks of the last pass, per level (rt_scan.hpp)
extern "C" int rt_debug_trace_clock(uint32_t* out, uint32_t words) {
    if (words > RT_TRACE_CLOCK_WORDS) words = RT_TRACE_CLOCK_WORDS;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(rtdev::rt_trace_clock), words * sizeof(uint32_t)) != hipSuccess;
}
#endif
#if RT_DIAG
// tools/scan_stats.py: read (and optionally reset) the wavefront pipeline's scan counters
extern "C" int rt_debug_scan_stats(unsigned long long* out40, int reset) {
    if (hipMemcpyFromSymbol(out40, HIP_SYMBOL(rtdev::rt_scan_stats), 40 * sizeof(unsigned long long)) != hipSuccess)
        return 1;
    if (reset) {
        unsigned long long z[40] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(rtdev::rt_scan_stats), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif
