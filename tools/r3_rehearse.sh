#!/bin/bash
# multi-rank rehearsal of the bench defaults on one GPU (gloo exchange, ranks share the card):
# the N = 2 / 4 code paths with K = 64 and passes of up to 16 frames, frame checks on
set -o pipefail
mkdir -p gpurun_out/rehearse
for n in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port 2955$n bench.py --gpus $n --backend gloo --cpu-baseline 0 --seam-stats 0 \
      > gpurun_out/rehearse/n$n.json 2> gpurun_out/rehearse/n$n.err || exit $n
done
echo done
