#!/bin/bash
# round-3 A/B batch 7: lazy child-colour loads in the combine
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_seam.py tests/test_gpu_fullframe.py -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3ab7.tests.log 2>&1 || exit 1
REPS=3 bash tools/ab_env.sh "RT_X=0" "RT_LIB=rust_tracer_amd/librt_hip_eceager.so" > gpurun_out/r3ab7.txt 2>&1 || exit 2
echo done
