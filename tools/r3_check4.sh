#!/bin/bash
# round-3 check 4: rt_render's seam split copies each share's rows straight to the caller
# (no gather / un-permute): seam tests, whole frames, then the seam timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_seam.py tests/test_gpu_fullframe.py tests/test_gpu_parity.py > gpurun_out/r3c4_tests.txt 2>&1 || exit 1
O=gpurun_out/r3c4_seam.jsonl
: > $O
for v in "RT_X=0" "RT_X=0"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 2
done
echo done
