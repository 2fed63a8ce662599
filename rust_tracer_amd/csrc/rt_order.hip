// rt_order.hip -- ordering of the ray queues: an LSD radix sort sized on the device.
//
// The level-synchronous pipeline (rt_wavefront.hip) reorders each level's ray tasks and
// the frame's shadow rays by a spatial key (direction cell or light, then the Morton code
// of the origin) so that a wave's 64 rays walk nearly the same path through the culling
// hierarchy.  Order never changes a result: every task carries its parent slot and a
// shadow entry its node and light.
//
// Why not a library sort: device-wide sorts take the element count on the host, which
// costs a device-to-host copy and a stream sync per level (~50 us of idle GPU each), and
// atomics-based counting sorts are slow here (same-bin atomics from many waves serialise
// beyond the L2).  This sort reads its extent (offset, count) from the pipeline's level
// counters, so a whole frame is enqueued without a host round trip, and uses no global
// atomics.  One 8-bit pass per key byte (2 for 16-bit keys, 3 for 24), each reduce-then-scan:
//   count    per 4096-key tile, a digit histogram in LDS -> tile_counts[digit][tile]
//   scan     per digit, exclusive scan over its tiles (one block per digit) + digit total
//   scatter  per tile, stable block rank (rocprim::block_radix_rank, wave "match"
//            algorithm: keys warp-striped, ranks ordered by (wave, item, lane) = index
//            order) -> position = digit base + the tile's offset within the digit + rank
// Every pass but the last writes (key, value) to scratch; the last writes only the values
// to their final place; stability keeps the previous passes' order within a digit.
#include <hip/hip_runtime.h>

#include <rocprim/block/block_radix_rank.hpp>

#include "rt_common.hpp"

namespace rtdev {

constexpr uint32_t SORT_THREADS = 256, SORT_ITEMS = 16, SORT_TILE = SORT_THREADS * SORT_ITEMS;

// the queue being ordered: a task level (offset / count in levels[2l], levels[2l + 1]) or
// the shadow queue (count in levels[2 (RT_MAX_DEPTH + 1)], offset 0)
struct SortRef {
    const uint32_t* levels;
    int32_t level;  // -1: the shadow queue
    uint32_t cap;   // slots of the queue's buffers
};

__device__ __forceinline__ uint32_t sort_extent(const SortRef& r, uint32_t& off) {
    if (r.level < 0) {
        off = 0;
        return min(r.levels[2 * (RT_MAX_DEPTH + 1)], r.cap);
    }
    off = r.levels[2 * r.level];
    return min(r.levels[2 * r.level + 1], off < r.cap ? r.cap - off : 0u);
}

// exclusive scan of one value per thread over a 256-thread block; `total` = the sum
__device__ __forceinline__ uint32_t block_exscan_256(uint32_t v, uint32_t& total, uint32_t* lds4) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63u) lds4[w] = x;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t k = 0; k < w; k++) before += lds4[k];
    total = lds4[0] + lds4[1] + lds4[2] + lds4[3];
    __syncthreads();  // lds4 may be reused right after
    return before + x - v;
}

// LDS digit count: one add when the whole wave holds one digit (pass 2 on ordered
// input), else one per lane (pass 1's low digits are nearly distinct across a wave)
__device__ __forceinline__ void lds_digit_add(uint32_t* h, uint32_t d, bool valid) {
    const uint64_t act = __ballot(valid);
    if (!act) return;
    const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)__builtin_ctzll(act));
    if (__ballot(valid && d != d0) == 0) {
        if (lane_id() == (uint32_t)__builtin_ctzll(act)) atomicAdd(&h[d0], (uint32_t)__builtin_popcountll(act));
    } else if (valid) {
        atomicAdd(&h[d], 1u);
    }
}

__global__ __launch_bounds__(SORT_THREADS) void sort_count_kernel(SortRef r, const uint32_t* keys, int keys_abs,
                                                                  uint32_t shift, uint32_t* tile_counts,
                                                                  uint32_t max_tiles) {
    __shared__ uint32_t h[256];
    uint32_t off;
    const uint32_t n = sort_extent(r, off);
    const uint32_t tiles = (n + SORT_TILE - 1) / SORT_TILE;
    const uint32_t* kin = keys + (keys_abs ? off : 0u);
    const uint32_t t = threadIdx.x;
    for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        h[t] = 0u;
        __syncthreads();
        for (uint32_t i = 0; i < SORT_ITEMS; i++) {
            const uint32_t idx = tile * SORT_TILE + i * SORT_THREADS + t;
            const bool valid = idx < n;
            lds_digit_add(h, valid ? (kin[idx] >> shift) & 255u : 0u, valid);
        }
        __syncthreads();
        tile_counts[t * max_tiles + tile] = h[t];
        __syncthreads();
    }
}

// block d: exclusive scan of digit d's tile counts (in place), total -> digit_totals[d]
__global__ __launch_bounds__(SORT_THREADS) void sort_scan_kernel(SortRef r, uint32_t* tile_counts, uint32_t max_tiles,
                                                                 uint32_t* digit_totals) {
    __shared__ uint32_t lds4[4];
    uint32_t off;
    const uint32_t n = sort_extent(r, off);
    const uint32_t tiles = (n + SORT_TILE - 1) / SORT_TILE;
    uint32_t* row = tile_counts + (size_t)blockIdx.x * max_tiles;
    uint32_t running = 0;
    for (uint32_t base = 0; base < tiles; base += SORT_THREADS) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < tiles ? row[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_exscan_256(v, total, lds4);
        if (i < tiles) row[i] = running + ex;
        running += total;
    }
    if (threadIdx.x == 0) digit_totals[blockIdx.x] = running;
}

using SortRank = rocprim::block_radix_rank<SORT_THREADS, 8, rocprim::block_radix_rank_algorithm::match>;

// vals == null: the value of entry i is off + i (a task's slot); keys_out == null: keys
// are not written (last pass)
__global__ __launch_bounds__(SORT_THREADS) void sort_scatter_kernel(SortRef r, const uint32_t* keys, const uint32_t* vals,
                                                                    int in_abs, uint32_t shift,
                                                                    const uint32_t* tile_counts, uint32_t max_tiles,
                                                                    const uint32_t* digit_totals, uint32_t* keys_out,
                                                                    uint32_t* vals_out, int out_abs) {
    __shared__ SortRank::storage_type rank_storage;
    __shared__ uint32_t base[256];
    __shared__ uint32_t lds4[4];
    uint32_t off;
    const uint32_t n = sort_extent(r, off);
    const uint32_t tiles = (n + SORT_TILE - 1) / SORT_TILE;
    const uint32_t t = threadIdx.x;
    uint32_t all;
    const uint32_t digit_base = block_exscan_256(digit_totals[t], all, lds4);  // thread t: digit t
    const uint32_t in_off = in_abs ? off : 0u, out_off = out_abs ? off : 0u;
    for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        uint32_t k[SORT_ITEMS], v[SORT_ITEMS], rank[SORT_ITEMS];
        // warp-striped: item i of lane l in wave w is entry w * 1024 + i * 64 + l of the tile
        const uint32_t first = tile * SORT_TILE + (t >> 6) * (64u * SORT_ITEMS) + (t & 63u);
        for (uint32_t i = 0; i < SORT_ITEMS; i++) {
            const uint32_t idx = first + i * 64u;
            const bool valid = idx < n;
            // padding sorts last (digit 255, after every real entry) and is never written
            k[i] = valid ? keys[in_off + idx] : 0xFFFFFFFFu;
            v[i] = valid ? (vals ? vals[in_off + idx] : off + idx) : 0u;
        }
        unsigned int pre[1], cnt[1];
        SortRank().rank_keys(k, rank, rank_storage, [shift](const uint32_t& key) { return (key >> shift) & 255u; },
                             pre, cnt);
        base[t] = digit_base + tile_counts[(size_t)t * max_tiles + tile] - pre[0];
        __syncthreads();
        for (uint32_t i = 0; i < SORT_ITEMS; i++) {
            if (first + i * 64u < n) {
                const uint32_t pos = base[(k[i] >> shift) & 255u] + rank[i];
                if (keys_out) keys_out[out_off + pos] = k[i];
                vals_out[out_off + pos] = v[i];
            }
        }
        __syncthreads();  // rank_storage and base are reused by the next tile
    }
}

uint32_t sort_max_tiles(uint32_t cap) { return (cap + SORT_TILE - 1) / SORT_TILE; }

// Sorts the queue `r` (keys at absolute slots) by `bits`-bit keys (8-bit digits, LSD);
// its values (vals, or the slots themselves when vals == null) land in vals_out at the
// same offset.  tmp: 2 x r.cap slots (keys, values) per intermediate buffer -- one for
// two passes, two (ping-pong) for three or four; tile_counts: 256 x sort_max_tiles(r.cap);
// digit_totals: 256.
hipError_t launch_sort(const uint32_t* levels, int32_t level, uint32_t cap, uint32_t bits, const uint32_t* keys,
                       const uint32_t* vals, uint32_t* tmp, uint32_t* vals_out, uint32_t* tile_counts,
                       uint32_t* digit_totals, int blocks, hipStream_t stream) {
    const SortRef r{levels, level, cap};
    const uint32_t mt = sort_max_tiles(cap);
    const int nb = (int)std::min<uint32_t>((uint32_t)blocks, mt > 0 ? mt : 1u);
    uint32_t passes = std::max(1u, std::min(4u, (bits + 7u) / 8u));
    // RT_SORT_TOP=k (A/B): sort by the top k key bytes only (skip the low passes)
    uint32_t skip = 0;
    if (const char* e = getenv("RT_SORT_TOP")) {
        const uint32_t k = (uint32_t)atoi(e);
        if (k >= 1 && k < passes) skip = passes - k;
    }
    const uint32_t* kin = keys;
    const uint32_t* vin = vals;
    int in_abs = 1;
    for (uint32_t p = skip; p < passes; p++) {
        const uint32_t shift = 8u * p;
        const bool last = p + 1 == passes;
        uint32_t* kout = last ? nullptr : tmp + (size_t)((p - skip) & 1u) * 2u * cap;
        uint32_t* vout = last ? vals_out : kout + cap;
        hipLaunchKernelGGL(sort_count_kernel, dim3(nb), dim3(SORT_THREADS), 0, stream, r, kin, in_abs, shift,
                           tile_counts, mt);
        hipLaunchKernelGGL(sort_scan_kernel, dim3(256), dim3(SORT_THREADS), 0, stream, r, tile_counts, mt,
                           digit_totals);
        hipLaunchKernelGGL(sort_scatter_kernel, dim3(nb), dim3(SORT_THREADS), 0, stream, r, kin, vin, in_abs, shift,
                           (const uint32_t*)tile_counts, mt, (const uint32_t*)digit_totals, kout, vout,
                           last ? 1 : 0);
        kin = kout;
        vin = vout;
        in_abs = 0;  // scratch buffers are relative to the queue's offset
    }
    return hipGetLastError();
}

}  // namespace rtdev
