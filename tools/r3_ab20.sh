#!/bin/bash
# round-3 A/B batch 20: rt_render's seam split -- shares and their grid share
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3ab20_seam.jsonl
: > $O
for v in "RT_X=0" "RT_SEAM_GRID_PCT=70" "RT_SEAM_GRID_PCT=90" "RT_SEAM_SPLIT=3 RT_SEAM_GRID_PCT=50" "RT_SEAM_SPLIT=3 RT_SEAM_GRID_PCT=65" "RT_SEAM_SPLIT=3 RT_SEAM_GRID_PCT=80" "RT_X=0"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 2
done
echo done
