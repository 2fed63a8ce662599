#!/bin/bash
# round-3 A/B batch 6: trace grid share with the new ordering; kernel trace at the defaults
set -o pipefail
mkdir -p gpurun_out/r3t
export TMPDIR=/tmp
REPS=2 bash tools/ab_env.sh "RT_GRID_PCT=75" "RT_GRID_PCT=65" "RT_GRID_PCT=85" "RT_GRID_PCT=100" "RT_GRID_PCT_SHADOW=75" > gpurun_out/r3ab6.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3t/trace -o run -- \
    python bench.py --steps 20 --warmup 4 --cpu-baseline 0 --seam-stats 0 --check 0 --count-frame 0 > gpurun_out/r3t/trace.log 2>&1 || exit 2
echo done
