#!/bin/bash
# scalar-cache counters of the render kernels (one frame of bench.py)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-sqc}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE \
    --output-format csv -d gpurun_out/$TAG/sqc -o run -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/$TAG/sqc.log 2>&1 || exit 3
echo done
