#!/bin/bash
# Build librt_hip_stats.so (scan hit-path counters on) next to the product library.
set -e
cd "$(dirname "$0")/../rust_tracer_amd/csrc"
mkdir -p build_stats
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -munsafe-fp-atomics -DRT_STATS=1"
/opt/rocm/bin/hipcc $F -c -o build_stats/rt_kernels.o rt_kernels.hip
/opt/rocm/bin/hipcc $F -c -o build_stats/rt_wavefront.o rt_wavefront.hip
/opt/rocm/bin/hipcc $F -shared -o ../librt_hip_stats.so build_stats/rt_kernels.o build_stats/rt_wavefront.o build/rt_api.o build/scene.o
