#!/bin/bash
# round-3 A/B batch 5: whole shape / material records in the trace kernel's hit phase
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh.py tests/test_gpu_forest.py tests/test_gpu_fullframe.py -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3ab5.tests.log 2>&1 || exit 1
REPS=3 bash tools/ab_env.sh "RT_X=0" "RT_LIB=rust_tracer_amd/librt_hip_nohitbulk.so" > gpurun_out/r3ab5.txt 2>&1 || exit 2
for L in rust_tracer_amd/librt_hip.so rust_tracer_amd/librt_hip_nohitbulk.so; do
  RT_LIB=$L timeout -k 10 200 python tools/seam_time.py >> gpurun_out/r3ab5_seam.jsonl 2>> gpurun_out/seam.err || exit 3
done
echo done
