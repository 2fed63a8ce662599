#!/bin/bash
# round-3 check 5: rt_render's adaptive seam split (meeting row follows the shares' finish
# times) with the shares' grids at 80%: seam tests, then the seam timings against the
# even split at full grids
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_seam.py tests/test_gpu_fullframe.py > gpurun_out/r3c5_tests.txt 2>&1 || exit 1
O=gpurun_out/r3c5_seam.jsonl
: > $O
for v in "RT_X=0" "RT_SEAM_ADAPT=0 RT_SEAM_GRID_PCT=100" "RT_X=0" "RT_SEAM_ADAPT=0 RT_SEAM_GRID_PCT=100"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 2
done
echo done
