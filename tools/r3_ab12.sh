#!/bin/bash
# round-3 A/B batch 12: per-level shadow passes with the shadow / trace grids sharing the chip
# (RT_SHADOW_LEVELS was removed after these runs: DESIGN.md, round 3)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3ab12_seam.jsonl
: > $O
for v in "RT_X=0" "RT_SHADOW_LEVELS=1 RT_GRID_PCT_SHADOW=25" "RT_SHADOW_LEVELS=1 RT_GRID_PCT=75 RT_GRID_PCT_SHADOW=25" \
         "RT_GRID_PCT=75" "RT_SHADOW_LEVELS=1 RT_GRID_PCT=50 RT_GRID_PCT_SHADOW=50" "RT_SHADOW_LEVELS=1 RT_SEAM_SPLIT=1"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 2
done
REPS=1 bash tools/ab_env.sh "RT_X=0" "RT_SHADOW_LEVELS=1 RT_GRID_PCT_SHADOW=25" "RT_SHADOW_LEVELS=1 RT_GRID_PCT_SHADOW=50" > gpurun_out/r3ab12.txt 2>&1 || exit 3
echo done
