#!/bin/bash
# Seam A/B on one GPU: tools/seam_time.py under several RT_* settings (each its own process)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/${1:-r3seam}.jsonl
: > $O
timeout -k 10 200 python tools/seam_time.py 2 4 >> $O 2> gpurun_out/seam.err || exit 1
RT_FINE1=1 timeout -k 10 200 python tools/seam_time.py 2 >> $O 2>> gpurun_out/seam.err || exit 2
RT_REVERSE=0xfffffffe timeout -k 10 200 python tools/seam_time.py >> $O 2>> gpurun_out/seam.err || exit 4
RT_GRID_PCT=50 timeout -k 10 200 python tools/seam_time.py 2 >> $O 2>> gpurun_out/seam.err || exit 3
echo done
