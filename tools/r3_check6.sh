#!/bin/bash
# round-3 check 6: the seam split's meeting row aimed at share 1 finishing as share 0's rows
# reach the caller (default) vs balanced finish times (RT_SEAM_ADAPT=device) vs the even split
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_seam.py > gpurun_out/r3c6_tests.txt 2>&1 || exit 1
O=gpurun_out/r3c6_seam.jsonl
: > $O
for rep in 1 2; do
for v in "RT_X=0" "RT_SEAM_ADAPT=device" "RT_SEAM_ADAPT=0"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 2
done
done
echo done
