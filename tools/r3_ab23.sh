#!/bin/bash
# round-3 A/B batch 23: level-0 tiles interleaved over a pass's frames (RT_L0_INTERLEAVE) at
# the K = 64 / 16-frame defaults
set -o pipefail
mkdir -p gpurun_out
REPS=3 bash tools/ab_env.sh "RT_X=0" "RT_L0_INTERLEAVE=1" > gpurun_out/r3ab23.txt 2>&1 || exit 1
echo done
