#!/bin/bash
# marginal cost of each stage at the bench defaults: launch it twice (RT_DUP: s = every queue
# sort, h = the shadow pass, c = every combine; each is idempotent)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3_dup.txt
: > $O
for rep in 1 2; do
for v in "RT_X=0" "RT_DUP=s" "RT_DUP=h" "RT_DUP=c"; do
  env $v timeout -k 10 300 python bench.py --warmup 4 --cpu-baseline 0 --seam-stats 0 --count-frame 0 --check 0 > gpurun_out/ab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$v', d['value'], d['ms_per_step'], flush=True)" >> $O
done
done
echo done
