#!/bin/bash
# round-3 A/B batch 3: level-0 interleave, key layouts, seam share sizes
set -o pipefail
mkdir -p gpurun_out
REPS=2 bash tools/ab_env.sh "RT_X=0" "RT_L0_INTERLEAVE=1" "RT_KEY24_DIR=16" "RT_KEY_AHEAD=0.15" "RT_KEY_AHEAD=0.4" > gpurun_out/r3ab3.txt 2>&1 || exit 1
O=gpurun_out/r3seam3.jsonl
: > $O
for v in "RT_SEAM_BAND_ROWS=480" "RT_SEAM_BAND_ROWS=600" "RT_SEAM_BAND_ROWS=544"; do
  env $v timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 2
done
echo done
