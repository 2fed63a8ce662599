#!/bin/bash
# A/B of tuning strings on the drop-in seam numbers (bench.py's `seam` extras: one frame at a
# time through rt_render_frame_async, rt_render with its host copy) and the headline, at the
# driver's settings.  usage: tools/ab_seam.sh TAG "RT_TUNE=..." "RT_TUNE=..." ...
set -o pipefail
TAG=${1:?tag}; shift
mkdir -p gpurun_out/$TAG
for rep in $(seq ${REPS:-1}); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 240 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/$TAG/ab.json 2> gpurun_out/$TAG/ab.err || { tail -5 gpurun_out/$TAG/ab.err; exit 3; }
    python -c "
import json;d=json.load(open('gpurun_out/$TAG/ab.json'));s=d['seam']
print('$cfg', d['value'], 'frame_async', s['one_frame_at_a_time_ms'], 'one_pass', s['one_pass_ms'], 'rt_render', s['rt_render_with_host_copy_ms'], 'pinned', s['rt_render_pinned_host_copy_ms'], flush=True)" | tee -a gpurun_out/$TAG/ab.txt
  done
done
