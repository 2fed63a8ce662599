#!/bin/bash
# one rank's share of a K = 64 burst at the bench defaults: N = 1, 2 (4 slots x 16 frames) and
# N = 4, 8 (3 slots x 11 frames)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3_share4.txt
: > $O
for rep in 1 2; do
  echo "== N=1,2 F=4 B=16" >> $O
  FLIGHT=4 BATCHES=16 WORLDS=1,2 K=64 REPS=2 timeout -k 10 300 python tools/share_burst.py >> $O 2>&1 || exit 1
  echo "== N=4,8 F=3 B=11" >> $O
  FLIGHT=3 BATCHES=11 WORLDS=4,8 K=64 REPS=2 timeout -k 10 300 python tools/share_burst.py >> $O 2>&1 || exit 2
done
echo done
