#!/bin/bash
# round-3 A/B batch 14: rt_render's seam split -- where the two shares meet (RT_SEAM_BAND_ROWS:
# share 0 = rows [0, n), share 1 the rest; default 544) and the persistent grids' share
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3ab14_seam.jsonl
: > $O
for v in "RT_X=0" "RT_SEAM_BAND_ROWS=480" "RT_SEAM_BAND_ROWS=512" "RT_SEAM_BAND_ROWS=576" "RT_SEAM_BAND_ROWS=608" \
         "RT_GRID_PCT=75" "RT_GRID_PCT=90" "RT_X=0"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 2
done
echo done
