#!/bin/bash
# instruction-cache counters of the render kernels (bench.py, frames in flight, default kernels only)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-icache}
mkdir -p gpurun_out/$TAG
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
    --output-format csv -d gpurun_out/$TAG/ic -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --seam-stats 0 --count-frame 0 > gpurun_out/$TAG/ic.log 2>&1 || exit 3
echo done
