#!/bin/bash
# round-3 A/B batch 19: more hardware queues (GPU_MAX_HW_QUEUES, 4 on the box) and passes in
# flight, K = 64, frame checks on
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3ab19.txt
: > $O
for rep in 1 2; do
for cfg in "RT_X=0:--inflight 4 --batch 16" "GPU_MAX_HW_QUEUES=8:--inflight 8 --batch 8" "GPU_MAX_HW_QUEUES=8:--inflight 6 --batch 11" "GPU_MAX_HW_QUEUES=8:--inflight 4 --batch 16" "RT_X=0:--inflight 8 --batch 8"; do
  e=${cfg%%:*}; a=${cfg#*:}
  env $e timeout -k 10 300 python bench.py $a --warmup 4 --cpu-baseline 0 --seam-stats 0 --count-frame 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));c=d['config'];print('$e $a', d['value'], d.get('frame_check'), c['workspace_bytes_all_slots'], flush=True)" >> $O
done
done
echo done
