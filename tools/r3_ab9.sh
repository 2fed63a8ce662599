#!/bin/bash
# round-3 A/B batch 9: does a wave's walk cost scale with its rays?  32-ray tasks everywhere
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3ab9_seam.jsonl
: > $O
for v in "RT_X=0" "RT_TASK_W=32 RT_TASK_FILL=1e9" "RT_TASK_W=16 RT_TASK_FILL=1e9"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 1
done
REPS=1 bash tools/ab_env.sh "RT_X=0" "RT_TASK_W=32 RT_TASK_FILL=1e9" "RT_TASK_W=16 RT_TASK_FILL=1e9" > gpurun_out/r3ab9.txt 2>&1 || exit 2
echo done
