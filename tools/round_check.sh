#!/bin/bash
# The round-end GPU sequence (driver order) plus a torchrun N=1 bench over RCCL and the
# profile of HEAD: tools/round_check.sh TAG
set -o pipefail
TAG=${1:-r1}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG.smoke.log 2>&1 || exit 2
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 1 --steps 5 --warmup 1 --cpu-baseline 0 > gpurun_out/$TAG.torchrun.log 2>&1 || exit 3
bash tools/gpu_profile.sh $TAG || exit 4
