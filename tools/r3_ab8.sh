#!/bin/bash
# round-3 A/B batch 8: machine scheduler strategies for the wavefront kernels
set -o pipefail
mkdir -p gpurun_out
REPS=2 bash tools/ab_env.sh "RT_X=0" "RT_LIB=rust_tracer_amd/librt_hip_schedilp.so" "RT_LIB=rust_tracer_amd/librt_hip_schedtrk.so" "RT_LIB=rust_tracer_amd/librt_hip_schedclause.so" > gpurun_out/r3ab8.txt 2>&1 || exit 1
echo done
