#!/bin/bash
# round-3 A/B batch 21: tile-local task order (RT_LOCAL_SORT bit mask of levels) against the
# global 3-pass radix sort: parity with it on, then one-pass timings and the bench
# (RT_LOCAL_SORT was removed after this run: DESIGN.md, round 3)
set -o pipefail
mkdir -p gpurun_out
RT_LOCAL_SORT=0xfe timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullframe.py > gpurun_out/r3ab21_tests.txt 2>&1 || exit 1
O=gpurun_out/r3ab21_seam.jsonl
: > $O
for v in "RT_X=0" "RT_LOCAL_SORT=0xfe" "RT_LOCAL_SORT=0xf0"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 2
done
REPS=2 bash tools/ab_env.sh "RT_X=0" "RT_LOCAL_SORT=0xfe" "RT_LOCAL_SORT=0xf0" "RT_LOCAL_SORT=0x80" > gpurun_out/r3ab21.txt 2>&1 || exit 3
echo done
