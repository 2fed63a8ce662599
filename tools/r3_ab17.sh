#!/bin/bash
# round-3 A/B batch 17: switches re-checked at the new bench defaults (16-frame passes)
# (ran at K = 20: tools/ab_env.sh still passed --steps 20 then)
set -o pipefail
REPS=2 bash tools/ab_env.sh "RT_X=0" "RT_INLINE_SHADOW=0" "RT_LB_RES=40" "RT_LB_RES=56" "RT_KEY_AHEAD=0.3" "RT_KEY_AHEAD=0.2" "RT_SELF_SHADOW=0" > gpurun_out/r3ab17.txt 2>&1 || exit 1
echo done
