#!/bin/bash
# round-3 A/B batch 24: RT_L0_INTERLEAVE again (parity with it on, then 4 alternating pairs)
set -o pipefail
mkdir -p gpurun_out
RT_L0_INTERLEAVE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_spp.py > gpurun_out/r3ab24_tests.txt 2>&1 || exit 1
REPS=4 bash tools/ab_env.sh "RT_L0_INTERLEAVE=1" "RT_X=0" > gpurun_out/r3ab24.txt 2>&1 || exit 2
echo done
