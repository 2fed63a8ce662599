#!/bin/bash
# round-3 A/B batch 18: passes of 32 frames (librt_hip_frames32.so: -DRT_MAX_FRAMES=32, frame
# index in Task.pixel bits 27-31) against the default 4 x 16, K = 64, frame checks on
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3ab18.txt
: > $O
L=rust_tracer_amd/librt_hip_frames32.so
for rep in 1 2; do
for cfg in "RT_X=0:--inflight 4 --batch 16" "RT_LIB=$L:--inflight 2 --batch 32" "RT_LIB=$L:--inflight 3 --batch 22" "RT_LIB=$L:--inflight 4 --batch 16"; do
  e=${cfg%%:*}; a=${cfg#*:}
  env $e timeout -k 10 300 python bench.py $a --warmup 4 --cpu-baseline 0 --seam-stats 0 --count-frame 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));c=d['config'];print('$e $a', d['value'], d.get('frame_check'), c['workspace_bytes_all_slots'], flush=True)" >> $O
done
done
echo done
