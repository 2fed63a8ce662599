#!/bin/bash
# round-3 A/B batch 16: grid share per pass at the new defaults (K = 64, 4 passes of 16)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3ab16.txt
: > $O
for rep in 1 2; do
for v in "RT_X=0" "RT_GRID_PCT=65" "RT_GRID_PCT=85" "RT_GRID_PCT=100"; do
  env $v timeout -k 10 300 python bench.py --warmup 4 --cpu-baseline 0 --seam-stats 0 --count-frame 0 > gpurun_out/ab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$v', d['value'], d.get('frame_check'), flush=True)" >> $O
done
done
echo done
