#!/bin/bash
# seam A/B: one_frame_at_a_time_ms per RT_TUNE setting (bench seam stats), 2 reps
set -o pipefail
mkdir -p gpurun_out/r5seam
for rep in 1 2; do
for t in "x=0" "seam_grid_pct=100" "seam_grid_pct=90" "seam_split=3" "seam_split=1"; do
  tt=$t; [ "$t" = "x=0" ] && tt=""
  RT_TUNE="$tt" timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --count-frame 0 > gpurun_out/r5seam/b.json 2>/dev/null || exit 3
  python -c "import json;d=json.load(open('gpurun_out/r5seam/b.json'));s=d['seam'];print('$t', s['one_frame_at_a_time_ms'], s['rt_render_with_host_copy_ms'], s.get('rt_render_pinned_host_copy_ms'), flush=True)"
done
done
