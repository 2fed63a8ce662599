set -o pipefail
timeout -k 10 200 python tools/ab_time.py 3 7 - RT_INLINE_SHADOW=0 RT_INLINE_SHADOW=2 RT_LB_RES=32 RT_LB_RES=64 RT_KEY_AHEAD=0.35 RT_KEY_AHEAD=0.15 - > gpurun_out/ab36.log 2>&1
