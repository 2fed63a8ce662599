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
// atomics.  Passes of 8- to 11-bit digits, as few as the key needs (2 for keys of up to
// 22 bits), each reduce-then-scan:
//   count    per tile (256 x RT_SORT_ITEMS keys), a digit histogram in LDS -> tile_counts[digit][tile]
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

// Keys per thread of a tile (a tile = 256 x RT_SORT_ITEMS keys).  Round 6, K = 20 on three
// boxes, 12 against 16: +1.8 / +0.7 / -0.3%, K = 64 +2.1%; 8 / 10 / 14 / 20: -1.9 / -1.1 /
// +0.4 / -3% (profiles/r6ab/r6ax_sort_items.log; rounds 2-3 had measured 8 / 24 / 32 against
// 16 at smaller passes).  (A build flag, not a tuning key: the tile size shapes the kernels.)
#ifndef RT_SORT_ITEMS
#define RT_SORT_ITEMS 12
#endif
constexpr uint32_t SORT_THREADS = 256, SORT_ITEMS = RT_SORT_ITEMS, SORT_TILE = SORT_THREADS * SORT_ITEMS;
constexpr uint32_t SORT_MAX_DIGIT_BITS = 11, SORT_MAX_DIGITS = 1u << SORT_MAX_DIGIT_BITS;

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

// Digits of DB bits (2^DB digits, DB = 8..11): thread t owns digits t * DPT .. t * DPT + DPT - 1.
template <uint32_t DB>
__global__ __launch_bounds__(SORT_THREADS) void sort_count_kernel(SortRef r, const uint32_t* keys, int keys_abs,
                                                                  uint32_t shift, uint32_t dmask,
                                                                  uint32_t* tile_counts, uint32_t max_tiles) {
    constexpr uint32_t ND = 1u << DB, DPT = ND / SORT_THREADS;
    __shared__ uint32_t h[ND];
    uint32_t off;
    const uint32_t n = sort_extent(r, off);
    const uint32_t tiles = (n + SORT_TILE - 1) / SORT_TILE;
    const uint32_t* kin = keys + (keys_abs ? off : 0u);
    const uint32_t t = threadIdx.x;
    for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        for (uint32_t j = 0; j < DPT; j++) h[t * DPT + j] = 0u;
        // every key of the tile requested before the first is counted (in-bounds clamped
        // addresses, no per-item branch): one memory round trip per tile, not SORT_ITEMS
        uint32_t kk[SORT_ITEMS];
#pragma unroll
        for (uint32_t i = 0; i < SORT_ITEMS; i++) kk[i] = kin[min(tile * SORT_TILE + i * SORT_THREADS + t, n - 1u)];
        __syncthreads();
#pragma unroll
        for (uint32_t i = 0; i < SORT_ITEMS; i++) {
            const uint32_t idx = tile * SORT_TILE + i * SORT_THREADS + t;
            const bool valid = idx < n;
            lds_digit_add(h, valid ? (kk[i] >> shift) & dmask : 0u, valid);
        }
        __syncthreads();
        for (uint32_t j = 0; j < DPT; j++) tile_counts[(size_t)(t * DPT + j) * max_tiles + tile] = h[t * DPT + j];
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

// vals == null: the value of entry i is off + i (a task's slot); keys_out == null: keys
// are not written (last pass)
template <uint32_t DB>
__global__ __launch_bounds__(SORT_THREADS) void sort_scatter_kernel(SortRef r, const uint32_t* keys, const uint32_t* vals,
                                                                    int in_abs, uint32_t shift, uint32_t dmask,
                                                                    const uint32_t* tile_counts, uint32_t max_tiles,
                                                                    const uint32_t* digit_totals, uint32_t* keys_out,
                                                                    uint32_t* vals_out, int out_abs) {
    constexpr uint32_t ND = 1u << DB, DPT = ND / SORT_THREADS;
    using SortRank = rocprim::block_radix_rank<SORT_THREADS, DB, rocprim::block_radix_rank_algorithm::match>;
    static_assert(SortRank::digits_per_thread == DPT, "digit ownership must match the ranker's");
    __shared__ typename SortRank::storage_type rank_storage;
    __shared__ uint32_t base[ND];
    __shared__ uint32_t lds4[4];
    uint32_t off;
    const uint32_t n = sort_extent(r, off);
    const uint32_t tiles = (n + SORT_TILE - 1) / SORT_TILE;
    if (blockIdx.x >= tiles) return;  // a block without a tile (the grid is sized for the queue's capacity)
    const uint32_t t = threadIdx.x;
    // thread t: digits t * DPT ..; their global bases (exclusive scan over every digit)
    uint32_t dtot[DPT], dsum = 0;
    for (uint32_t j = 0; j < DPT; j++) {
        dtot[j] = digit_totals[t * DPT + j];
        dsum += dtot[j];
    }
    uint32_t all;
    uint32_t digit_base[DPT];
    digit_base[0] = block_exscan_256(dsum, all, lds4);
    for (uint32_t j = 1; j < DPT; j++) digit_base[j] = digit_base[j - 1] + dtot[j - 1];
    const uint32_t in_off = in_abs ? off : 0u, out_off = out_abs ? off : 0u;
    for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        uint32_t k[SORT_ITEMS], v[SORT_ITEMS], rank[SORT_ITEMS];
        // warp-striped: item i of lane l in wave w is entry w * 1024 + i * 64 + l of the tile
        const uint32_t first = tile * SORT_TILE + (t >> 6) * (64u * SORT_ITEMS) + (t & 63u);
        // every key and value requested at once (clamped in-bounds addresses, no per-item
        // branch between the loads); padding is patched in afterwards: it ranks after every
        // real entry of its digit (it is last in the tile) and is never written
        if (vals) {
#pragma unroll
            for (uint32_t i = 0; i < SORT_ITEMS; i++) {
                const uint32_t idc = min(first + i * 64u, n - 1u);
                k[i] = keys[in_off + idc];
                v[i] = vals[in_off + idc];
            }
        } else {
#pragma unroll
            for (uint32_t i = 0; i < SORT_ITEMS; i++) {
                const uint32_t idc = min(first + i * 64u, n - 1u);
                k[i] = keys[in_off + idc];
                v[i] = off + idc;
            }
        }
#pragma unroll
        for (uint32_t i = 0; i < SORT_ITEMS; i++) {
            if (first + i * 64u >= n) {
                k[i] = 0xFFFFFFFFu;
                v[i] = 0u;
            }
        }
        unsigned int pre[DPT], cnt[DPT];
        SortRank().rank_keys(k, rank, rank_storage, [shift, dmask](const uint32_t& key) { return (key >> shift) & dmask; },
                             pre, cnt);
        for (uint32_t j = 0; j < DPT; j++)
            base[t * DPT + j] = digit_base[j] + tile_counts[(size_t)(t * DPT + j) * max_tiles + tile] - pre[j];
        __syncthreads();
        for (uint32_t i = 0; i < SORT_ITEMS; i++) {
            if (first + i * 64u < n) {
                const uint32_t pos = base[(k[i] >> shift) & dmask] + rank[i];
                if (keys_out) keys_out[out_off + pos] = k[i];
                vals_out[out_off + pos] = v[i];
            }
        }
        __syncthreads();  // rank_storage and base are reused by the next tile
    }
}

uint32_t sort_max_tiles(uint32_t cap) { return (cap + SORT_TILE - 1) / SORT_TILE; }
uint32_t sort_max_digits() { return SORT_MAX_DIGITS; }

template <uint32_t DB>
static void sort_pass(const SortRef& r, int nb, uint32_t mt, const uint32_t* kin, const uint32_t* vin, int in_abs,
                      uint32_t shift, uint32_t dmask, uint32_t* tile_counts, uint32_t* digit_totals, uint32_t* kout,
                      uint32_t* vout, int out_abs, hipStream_t stream) {
    hipLaunchKernelGGL(sort_count_kernel<DB>, dim3(nb), dim3(SORT_THREADS), 0, stream, r, kin, in_abs, shift, dmask,
                       tile_counts, mt);
    hipLaunchKernelGGL(sort_scan_kernel, dim3(1u << DB), dim3(SORT_THREADS), 0, stream, r, tile_counts, mt,
                       digit_totals);
    hipLaunchKernelGGL(sort_scatter_kernel<DB>, dim3(nb), dim3(SORT_THREADS), 0, stream, r, kin, vin, in_abs, shift,
                       dmask, (const uint32_t*)tile_counts, mt, (const uint32_t*)digit_totals, kout, vout, out_abs);
}

// Sorts the queue `r` (keys at absolute slots) by `bits`-bit keys, LSD, in as few passes
// as digits of up to `max_digit` (8..11) bits allow, the bits split evenly over the passes
// (16 bits: 2 x 8; 17: 2 x 9; 21: 2 x 11).  Its values (vals, or the slots themselves when
// vals == null) land in vals_out at the same offset.  tmp: 2 x r.cap slots (keys, values)
// per intermediate buffer -- one for two passes, two (ping-pong) for three or more;
// tile_counts: sort_max_digits() x sort_max_tiles(r.cap); digit_totals: sort_max_digits().
hipError_t launch_sort(const uint32_t* levels, int32_t level, uint32_t cap, uint32_t bits, const uint32_t* keys,
                       const uint32_t* vals, uint32_t* tmp, uint32_t* vals_out, uint32_t* tile_counts,
                       uint32_t* digit_totals, int blocks, hipStream_t stream, uint32_t max_digit) {
    const SortRef r{levels, level, cap};
    const uint32_t mt = sort_max_tiles(cap);
    const int nb = (int)std::min<uint32_t>((uint32_t)blocks, mt > 0 ? mt : 1u);
    max_digit = std::max(8u, std::min(SORT_MAX_DIGIT_BITS, max_digit));
    bits = std::max(1u, std::min(32u, bits));
    const uint32_t passes = (bits + max_digit - 1u) / max_digit;
    const uint32_t db = std::max(8u, (bits + passes - 1u) / passes);
    const uint32_t* kin = keys;
    const uint32_t* vin = vals;
    int in_abs = 1;
    for (uint32_t p = 0; p < passes; p++) {
        const uint32_t shift = db * p;
        const bool last = p + 1 == passes;
        uint32_t* kout = last ? nullptr : tmp + (size_t)(p & 1u) * 2u * cap;
        uint32_t* vout = last ? vals_out : kout + cap;
        const int oa = last ? 1 : 0;
        // the key's bits above `bits` are not sorted on: the last pass's digit may be narrower
        const uint32_t w = std::min(db, bits - shift);
        const uint32_t dm = (1u << w) - 1u;
        switch (db) {
            case 8: sort_pass<8>(r, nb, mt, kin, vin, in_abs, shift, dm, tile_counts, digit_totals, kout, vout, oa, stream); break;
            case 9: sort_pass<9>(r, nb, mt, kin, vin, in_abs, shift, dm, tile_counts, digit_totals, kout, vout, oa, stream); break;
            case 10: sort_pass<10>(r, nb, mt, kin, vin, in_abs, shift, dm, tile_counts, digit_totals, kout, vout, oa, stream); break;
            default: sort_pass<11>(r, nb, mt, kin, vin, in_abs, shift, dm, tile_counts, digit_totals, kout, vout, oa, stream); break;
        }
        kin = kout;
        vin = vout;
        in_abs = 0;  // scratch buffers are relative to the queue's offset
    }
    return hipGetLastError();
}

}  // namespace rtdev
