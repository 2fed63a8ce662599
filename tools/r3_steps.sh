#!/bin/bash
# bench throughput against the timed frame count K (default 20): bigger K lets every slot run
# several passes of up to 8 frames
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3_steps.txt
: > $O
for rep in 1 2; do
for k in 20 40 64 96; do
  timeout -k 10 200 python bench.py --steps $k --warmup 4 --cpu-baseline 0 --seam-stats 0 --count-frame 0 > gpurun_out/steps.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/steps.json'));c=d['config'];print('K', $k, d['value'], c['frames_per_pass'], c['passes_in_flight'], c.get('frame_check'), d.get('frame_check'), flush=True)" >> $O
done
done
echo done
