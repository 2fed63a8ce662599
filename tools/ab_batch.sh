#!/bin/bash
# frames per pass x passes in flight at N = 1 (GPU side): STEPS=K tools/ab_batch.sh "B F" ...
set -o pipefail
mkdir -p gpurun_out
cfgs=("$@")
for rep in 1 2; do
for bf in "${cfgs[@]}"; do
  read b f <<< "$bf"
  timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup 5 --cpu-baseline 0 --seam-stats 0 --count-frame 0 --batch $b --inflight $f > gpurun_out/abn1.json 2>/dev/null || exit 3
  python -c "import json;d=json.load(open('gpurun_out/abn1.json'));print('steps ${STEPS:-20} batch $b inflight $f', d['value'], d['config']['pass_latency_ms'], flush=True)"
done
done
