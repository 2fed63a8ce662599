#!/bin/bash
# per-kernel phase cycles of the counting frame: trace kernels only / shadow kernel only
set -o pipefail
mkdir -p gpurun_out/r3count
for k in trace shadow; do
  RT_COUNT=$k timeout -k 10 200 python bench.py --steps 4 --warmup 1 --cpu-baseline 0 --seam-stats 0 --check 0 \
    > gpurun_out/r3count/$k.json 2> gpurun_out/r3count/$k.err || exit 1
done
RT_OCC_DEBUG=1 RT_BVH_DEBUG=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --seam-stats 0 --check 0 \
    --count-frame 0 > gpurun_out/r3count/occ.json 2> gpurun_out/r3count/occ.err || exit 2
echo done
