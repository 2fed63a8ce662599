#!/bin/bash
# round-3 A/B batch 22: Hilbert instead of Morton order in the 24-bit task keys (RT_TASK_CURVE)
# (RT_TASK_CURVE was removed after this run: DESIGN.md, round 3)
set -o pipefail
mkdir -p gpurun_out
RT_TASK_CURVE=hilbert timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > gpurun_out/r3ab22_tests.txt 2>&1 || exit 1
REPS=3 bash tools/ab_env.sh "RT_X=0" "RT_TASK_CURVE=hilbert" > gpurun_out/r3ab22.txt 2>&1 || exit 3
echo done
