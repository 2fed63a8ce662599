#!/bin/bash
# round-3 A/B batch 10: two shadow rays per lane (RT_DUAL=1) and the LDS-staged sort scatter
# (RT_SORT_STAGE=1): parity first (full frames against the oracle), then the bench.
# Both variants were removed after this run (profiles/r3ab/r3ab10.txt).
set -o pipefail
mkdir -p gpurun_out
RT_DUAL=1 RT_SORT_STAGE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_sort.py tests/test_gpu_cull_stress.py tests/test_gpu_fullframe.py tests/test_gpu_parity.py tests/test_gpu_bvh.py > gpurun_out/r3ab10_tests.txt 2>&1 || exit 1
REPS=2 bash tools/ab_env.sh "RT_X=0" "RT_DUAL=1" "RT_SORT_STAGE=1" "RT_DUAL=1 RT_SORT_STAGE=1" > gpurun_out/r3ab10.txt 2>&1 || exit 2
echo done
