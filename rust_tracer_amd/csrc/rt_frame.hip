// rt_frame.hip -- frame assembly kernels of the render path (gfx950).
//
//  * unpermute: the block-cyclic band buffers of the multi-rank render (one gather per
//    pass) back into row-major frames (rust_tracer_amd/dist.py, rt_multi.cpp);
//  * quantize: Color::as_u8 (color.rs:43-46) over a float frame;
//  * spp accumulate: config 5's sample batches folded in sample order (rt_render_spp);
//  * the host check of the scan's compile-time cube triangles against Cube::new.
// The render kernels themselves are in rt_wavefront.hip (trace / shadow / combine) and
// rt_order.hip (queue sorts).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#include "../../include/rt_api.h"
#include "rt_device.hpp"

#include "rt_common.hpp"

namespace rtdev {

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


// ---- sample batches (rt_render.cpp launch_bands_wave): the batch's samples first .. first + n - 1
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
