#!/bin/bash
# round-3 A/B batch 4: batched sort loads, bulk material loads in the combine
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_parity.py -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3ab4.tests.log 2>&1 || exit 1
REPS=3 bash tools/ab_env.sh "RT_X=0" "RT_LIB=rust_tracer_amd/librt_hip_nomatbulk.so" "RT_LIB=rust_tracer_amd/librt_hip_oldsort.so" > gpurun_out/r3ab4.txt 2>&1 || exit 2
for L in rust_tracer_amd/librt_hip.so rust_tracer_amd/librt_hip_oldsort.so; do
  RT_LIB=$L timeout -k 10 200 python tools/seam_time.py >> gpurun_out/r3ab4_seam.jsonl 2>> gpurun_out/seam.err || exit 3
done
echo done
