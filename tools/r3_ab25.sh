#!/bin/bash
# round-3 A/B batch 25: level 0's trace instantiation at 4 waves per SIMD (128 VGPRs, no
# scratch; librt_hip_first4.so: tools/build_variant.sh first4 -DRT_FIRST_WAVES=4) against the
# default 5 waves (96 VGPRs, 116 B of scratch per lane); deep levels keep 5 waves and their
# grid (launch_wave_trace scales each instantiation's grid by its own occupancy)
set -o pipefail
mkdir -p gpurun_out
V=rust_tracer_amd/librt_hip_first4.so
export RT_OCC_EACH=1
RT_LIB=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullframe.py tests/test_gpu_parity.py > gpurun_out/r3ab25_tests.txt 2>&1 || exit 1
O=gpurun_out/r3ab25_frame.jsonl
: > $O
for v in "RT_X=0" "RT_LIB=$V" "RT_X=0" "RT_LIB=$V"; do
  env $v timeout -k 10 150 python tools/frame_async_time.py --stream side >> $O 2>> gpurun_out/r3ab25.err || exit 2
done
REPS=3 bash tools/ab_env.sh "RT_X=0" "RT_LIB=$V" > gpurun_out/r3ab25.txt 2>&1 || exit 3
echo done
