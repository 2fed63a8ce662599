#!/bin/bash
# Build librt_hip_clk.so (per wave-iteration wall-clock records in the trace kernel,
# RT_TASK_CLOCK) next to the product library; run with RT_LIB pointing at it.
set -e
cd "$(dirname "$0")/../rust_tracer_amd/csrc"
make -s
mkdir -p build_clk
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -munsafe-fp-atomics -DRT_TASK_CLOCK_BUILD=1"
/opt/rocm/bin/hipcc $F -c -o build_clk/rt_wavefront.o rt_wavefront.hip
/opt/rocm/bin/hipcc $F -shared -o ../librt_hip_clk.so build/rt_kernels.o build_clk/rt_wavefront.o \
    build/rt_order.o build/rt_api.o build/rt_bvh.o build/scene.o build/image_io.o
