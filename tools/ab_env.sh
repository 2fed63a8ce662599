#!/bin/bash
# A/B of tuning keys (rt_tune.hpp) on the benchmark (GPU side):
#   tools/ab_env.sh "RT_TUNE=lb_res=0,task_w=32" "RT_TUNE=lb_res=64" "RT_LIB=rust_tracer_amd/librt_hip_X.so" ...
# ('+' joins several variables of one setting: "RT_LIB=...+RT_TUNE=occ_each=1")
# Each setting runs REPS times (default 2), alternating, at the bench defaults (frames in flight;
# K timed frames, default 20 = the driver's run).
set -o pipefail
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for cfg in "$@"; do
    env ${cfg//+/ } timeout -k 10 200 python bench.py --steps ${K:-20} --warmup 5 --cpu-baseline 0 --seam-stats 0 --count-frame 0 > gpurun_out/ab.json 2>/dev/null || exit 3
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$cfg', d['value'], flush=True)"
  done
done
