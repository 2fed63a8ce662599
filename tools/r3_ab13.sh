#!/bin/bash
# round-3 A/B batch 13: hierarchy leaf records staged in LDS (RT_LDS_LEAVES, default build)
# against scalar loads (librt_hip_noldsleaf.so: tools/build_variant.sh noldsleaf -DRT_LDS_LEAVES=0)
# (RT_LDS_LEAVES was removed after this run: DESIGN.md, round 3)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullframe.py tests/test_gpu_parity.py tests/test_gpu_bvh.py tests/test_gpu_cull_stress.py \
  > gpurun_out/r3ab13_tests.txt 2>&1 || exit 1
O=gpurun_out/r3ab13_seam.jsonl
: > $O
for v in "RT_X=0" "RT_LIB=rust_tracer_amd/librt_hip_noldsleaf.so" "RT_X=0" "RT_LIB=rust_tracer_amd/librt_hip_noldsleaf.so"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 2
done
REPS=3 bash tools/ab_env.sh "RT_X=0" "RT_LIB=rust_tracer_amd/librt_hip_noldsleaf.so" > gpurun_out/r3ab13.txt 2>&1 || exit 3
echo done
