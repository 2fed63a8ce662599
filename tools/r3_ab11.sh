#!/bin/bash
# round-3 A/B batch 11: a shadow pass per trace level on a side stream (RT_SHADOW_LEVELS=1):
# (RT_SHADOW_LEVELS was removed after these runs: DESIGN.md, round 3)
# parity first, then one-pass / seam timings, then the bench
set -o pipefail
mkdir -p gpurun_out
RT_SHADOW_LEVELS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullframe.py tests/test_gpu_parity.py tests/test_gpu_bvh.py tests/test_gpu_spp.py tests/test_gpu_forest.py \
  > gpurun_out/r3ab11_tests.txt 2>&1 || exit 1
O=gpurun_out/r3ab11_seam.jsonl
: > $O
for v in "RT_X=0" "RT_SHADOW_LEVELS=1" "RT_X=0" "RT_SHADOW_LEVELS=1"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 2
done
REPS=2 bash tools/ab_env.sh "RT_X=0" "RT_SHADOW_LEVELS=1" > gpurun_out/r3ab11.txt 2>&1 || exit 3
echo done
