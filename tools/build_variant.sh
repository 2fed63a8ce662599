#!/bin/bash
# Builds an A/B variant of the product library with extra compile flags:
#   tools/build_variant.sh NAME "-DRT_SWITCH=0 ..."  -> rust_tracer_amd/librt_hip_NAME.so
# (load it with RT_LIB=rust_tracer_amd/librt_hip_NAME.so; tools/ab_env.sh takes RT_LIB=...)
# "-DRT_DIAG=1" builds the diagnostic knobs (result-changing measurement switches, debug
# prints, the scan hit-path and leaf-occupancy counters of tools/scan_stats.py) that the
# product library does not contain.
set -e
NAME=$1; FLAGS=$2
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/rust_tracer_amd/csrc
B=/tmp/rt_variant_$NAME
rm -rf $B && mkdir -p $B  # (a stale object of an older layout would link twice)
HF="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall --offload-arch=gfx950 -munsafe-fp-atomics $FLAGS"
CF="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall $FLAGS"
WFFLAGS=${WFFLAGS--mllvm -amdgpu-atomic-optimizer-strategy=None}  # as the Makefile (WFFLAGS= : the compiler's default)
/opt/rocm/bin/hipcc $HF $WFFLAGS -c -o $B/rt_wavefront.o $C/rt_wavefront.hip &
for f in rt_frame rt_order; do /opt/rocm/bin/hipcc $HF -c -o $B/$f.o $C/$f.hip & done
for f in rt_build rt_scene rt_render rt_forest rt_multi; do /opt/rocm/bin/hipcc $HF -c -o $B/$f.o $C/$f.cpp & done
/opt/rocm/bin/hipcc $CF -x c++ -c -o $B/rt_bvh.o $C/rt_bvh.cpp &
/opt/rocm/bin/hipcc $CF -x c++ -c -o $B/rt_tune.o $C/rt_tune.cpp &
/opt/rocm/bin/hipcc $CF -x c++ -c -o $B/image_io.o $C/host/image_io.cpp &
/opt/rocm/bin/hipcc $CF -x c++ -c -o $B/scene.o $C/host/scene.cpp &
for j in $(jobs -p); do wait $j || { echo "compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc $HF -shared -o $R/rust_tracer_amd/librt_hip_$NAME.so $B/*.o -ldl
echo built rust_tracer_amd/librt_hip_$NAME.so
