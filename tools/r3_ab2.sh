#!/bin/bash
# round-3 A/B batch 2: seam split variants, 24-bit keys
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3seam2.jsonl
: > $O
for v in "RT_SEAM_SPLIT=1" "RT_SEAM_SPLIT=2" "RT_SEAM_SPLIT=3" "RT_SEAM_BAND_ROWS=16" "RT_SEAM_BAND_ROWS=64" "RT_SEAM_BAND_ROWS=544" "RT_FINE1=1"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 1
done
REPS=2 bash tools/ab_env.sh "RT_KEY24=0" "RT_KEY24=1" > gpurun_out/r3ab_key24.txt 2>&1 || exit 2
echo done
