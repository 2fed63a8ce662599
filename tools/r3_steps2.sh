#!/bin/bash
# frames per pass / passes in flight at K = 64 and 128
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3_steps2.txt
: > $O
for rep in 1 2; do
for cfg in "--steps 64" "--steps 64 --batch 16" "--steps 64 --batch 11 --inflight 3" "--steps 128" "--steps 128 --batch 16" "--steps 64 --batch 10 --inflight 4"; do
  timeout -k 10 300 python bench.py $cfg --warmup 4 --cpu-baseline 0 --seam-stats 0 --count-frame 0 > gpurun_out/steps.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/steps.json'));c=d['config'];print('$cfg', d['value'], c['frames_per_pass'], c['passes_in_flight'], d.get('frame_check'), c['workspace_bytes_all_slots'], flush=True)" >> $O
done
done
echo done
