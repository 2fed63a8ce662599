// rt_libm_selftest.hip -- TEST INFRASTRUCTURE (not part of the product library).
//
// The device path evaluates the reference's libm calls with restatements of glibc's own
// algorithms: powf (rust_tracer_amd/csrc/rt_powf.hpp, material.rs:211) and atan2f / acosf
// (rt_libmf.hpp, sphere.rs:40-45).  This library runs exactly those header functions over
// arrays -- on the device (the code the render kernels inline) and compiled for the host --
// so tests/test_libm.py can compare them bit for bit with the host's libm.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../rust_tracer_amd/csrc/rt_libmf.hpp"
#include "../../rust_tracer_amd/csrc/rt_powf.hpp"

enum { FN_POWF = 0, FN_ATAN2F = 1, FN_ACOSF = 2, FN_ATANF = 3 };

__host__ __device__ inline float eval(int fn, float x, float y) {
    switch (fn) {
        case FN_POWF: return rtpow::powf_glibc(x, y);
        case FN_ATAN2F: return rtlibm::atan2f_fd(x, y);  // atan2f(y = x[i], x = y[i])
        case FN_ACOSF: return rtlibm::acosf_fd(x);
        default: return rtlibm::atanf_fd(x);
    }
}

__global__ void libm_batch_kernel(int fn, const float* x, const float* y, float* out, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = eval(fn, x[i], y ? y[i] : 0.f);
}

// 0 = ok, 1 = bad argument, 2 = HIP error
extern "C" int rt_libm_batch_async(int fn, const float* d_x, const float* d_y, float* d_out, uint64_t n,
                                   void* stream) {
    if (n == 0) return 0;
    if (fn < 0 || fn > 3 || !d_x || !d_out || ((fn == FN_POWF || fn == FN_ATAN2F) && !d_y)) return 1;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 255) / 256, 4096u);
    hipLaunchKernelGGL(libm_batch_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, fn, d_x, d_y, d_out, n);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rt_libm_batch_host(int fn, const float* x, const float* y, float* out, uint64_t n) {
    if (fn < 0 || fn > 3 || (n && (!x || !out || ((fn == FN_POWF || fn == FN_ATAN2F) && !y)))) return 1;
    for (uint64_t i = 0; i < n; i++) out[i] = eval(fn, x[i], y ? y[i] : 0.f);
    return 0;
}
