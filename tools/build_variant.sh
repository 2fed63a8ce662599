#!/bin/bash
# Builds an A/B variant of the product library with extra device-compile flags on the
# wavefront and ordering kernels: tools/build_variant.sh NAME "-DFOO=1 ..." -> rust_tracer_amd/librt_hip_NAME.so
# (the other objects are the product's own; run `make` first).  Use with RT_LIB=... .
set -e
NAME=$1; shift
cd "$(dirname "$0")/../rust_tracer_amd/csrc"
make -s
T=/tmp/rt_variant_$NAME
mkdir -p $T
F="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall --offload-arch=gfx950 -munsafe-fp-atomics"
/opt/rocm/bin/hipcc $F "$@" -c -o $T/rt_wavefront.o rt_wavefront.hip
/opt/rocm/bin/hipcc $F "$@" -c -o $T/rt_order.o rt_order.hip
/opt/rocm/bin/hipcc $F -shared -o ../librt_hip_$NAME.so build/rt_kernels.o $T/rt_wavefront.o \
    $T/rt_order.o build/rt_api.o build/rt_multi.o build/rt_bvh.o build/scene.o build/image_io.o
echo built rust_tracer_amd/librt_hip_$NAME.so
