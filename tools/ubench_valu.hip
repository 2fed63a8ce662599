// ubench_valu.hip -- throughput of f32 VALU forms on gfx950 (tooling, not product).
// Each thread runs 8 independent chains of one instruction form; 8 waves per SIMD.
// Prints ns per wave-instruction per SIMD -> cycles at the measured clock.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

#define ITERS 4096

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, float s) {
    float a[8];
    f2 b[8];
    for (int i = 0; i < 8; i++) {
        a[i] = threadIdx.x * 1e-3f + i;
        b[i] = f2{a[i], a[i] + 0.5f};
    }
    f2 s2 = f2{s, s * 0.5f};
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (KIND == 0) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(a[i]) : "v"(s));
            if (KIND == 1) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(b[i]) : "v"(s2));
            if (KIND == 2) asm volatile("v_fma_f32 %0, %1, %0, %1" : "+v"(a[i]) : "v"(s));
            if (KIND == 3) asm volatile("v_pk_fma_f32 %0, %1, %0, %1" : "+v"(b[i]) : "v"(s2));
            if (KIND == 4) asm volatile("v_add_f32 %0, %1, %0" : "+v"(a[i]) : "v"(s));
            if (KIND == 5) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(b[i]) : "v"(s2));
            if (KIND == 6) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(a[i]) : "s"(s));
            if (KIND == 7) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(b[i]) : "s"(s2));
        }
    }
    float r = 0;
    for (int i = 0; i < 8; i++) r += a[i] + b[i].x + b[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int KIND>
float run(float* d, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, d, 1.0001f);
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, d, 1.0001f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    int cus = p.multiProcessorCount;
    int blocks = cus * 8;  // 8 blocks x 4 waves = 32 waves/CU = 8 per SIMD
    float* d;
    hipMalloc(&d, (size_t)blocks * 256 * 4);
    const char* names[] = {"v_mul_f32", "v_pk_mul_f32", "v_fma_f32", "v_pk_fma_f32",
                           "v_add_f32", "v_pk_add_f32", "v_mul_f32 sgpr", "v_pk_mul_f32 sgpr"};
    float ms[8] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks),
                   run<4>(d, blocks), run<5>(d, blocks), run<6>(d, blocks), run<7>(d, blocks)};
    double wave_instr_per_simd = (double)blocks * 4 / (cus * 4) * ITERS * 8;
    for (int i = 0; i < 8; i++) {
        double ns = ms[i] * 1e6 / wave_instr_per_simd;
        printf("%-20s %.3f ms  %.3f ns/wave-instr/SIMD  (%.2f cycles @2.4GHz)\n", names[i], ms[i], ns, ns * 2.4);
    }
    return 0;
}
