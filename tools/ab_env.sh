#!/bin/bash
# A/B of RT_* switches on the benchmark (GPU side): tools/ab_env.sh "ENV1=a ENV2=b" "ENV1=c" ...
# Each setting runs REPS times (default 2), alternating, at the bench defaults (frames in flight).
set -o pipefail
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 4 --cpu-baseline 0 --seam-stats 0 --count-frame 0 > gpurun_out/ab.json 2>/dev/null || exit 3
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$cfg', d['value'], flush=True)"
  done
done
