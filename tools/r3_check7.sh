#!/bin/bash
# round-3 check 7: sort scatter blocks without a tile leave at once: sort tests, parity, seam timings, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_sort.py tests/test_gpu_parity.py tests/test_gpu_fullframe.py > gpurun_out/r3c7_tests.txt 2>&1 || exit 1
O=gpurun_out/r3c7_seam.jsonl
: > $O
for v in "RT_X=0" "RT_X=0"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 2
done
REPS=2 bash tools/ab_env.sh "RT_X=0" > gpurun_out/r3c7_bench.txt 2>&1 || exit 3
echo done
