#!/bin/bash
# K = 64 at N = 4 / 8: 4 slots x 16 frames against 3 x 11 (the bench's default since r3_share2)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3_share5.txt
: > $O
for rep in 1 2; do
  echo "== N=4,8 F=4 B=16" >> $O
  FLIGHT=4 BATCHES=16 WORLDS=4,8 K=64 REPS=2 timeout -k 10 300 python tools/share_burst.py >> $O 2>&1 || exit 1
  echo "== N=4,8 F=3 B=11" >> $O
  FLIGHT=3 BATCHES=11 WORLDS=4,8 K=64 REPS=2 timeout -k 10 300 python tools/share_burst.py >> $O 2>&1 || exit 2
  echo "== N=4,8 F=4 B=8" >> $O
  FLIGHT=4 BATCHES=8 WORLDS=4,8 K=64 REPS=2 timeout -k 10 300 python tools/share_burst.py >> $O 2>&1 || exit 3
done
echo done
