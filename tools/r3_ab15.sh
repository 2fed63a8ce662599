#!/bin/bash
# round-3 A/B batch 15: the seam split's meeting row and grid share combined
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3ab15_seam.jsonl
: > $O
for rep in 1 2; do
for v in "RT_X=0" "RT_SEAM_BAND_ROWS=576 RT_GRID_PCT=90" "RT_SEAM_BAND_ROWS=576 RT_GRID_PCT=80" "RT_SEAM_BAND_ROWS=560 RT_GRID_PCT=90" "RT_SEAM_BAND_ROWS=592 RT_GRID_PCT=90"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 2
done
done
echo done
