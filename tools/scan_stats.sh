#!/bin/bash
# Build librt_hip_stats.so (scan hit-path and leaf-occupancy counters on) next to the
# product library (same objects otherwise).
set -e
cd "$(dirname "$0")/../rust_tracer_amd/csrc"
make -s
mkdir -p build_stats
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -munsafe-fp-atomics -DRT_STATS=1"
/opt/rocm/bin/hipcc $F -c -o build_stats/rt_kernels.o rt_kernels.hip
/opt/rocm/bin/hipcc $F -c -o build_stats/rt_wavefront.o rt_wavefront.hip
/opt/rocm/bin/hipcc $F -shared -o ../librt_hip_stats.so build_stats/rt_kernels.o build_stats/rt_wavefront.o \
    build/rt_order.o build/rt_api.o build/rt_multi.o build/rt_bvh.o build/scene.o build/image_io.o
