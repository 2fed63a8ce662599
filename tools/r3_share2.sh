#!/bin/bash
# one rank's share of a K = 20 burst at N = 8 / 4: passes in flight x frames per pass
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3_share2.txt
: > $O
for cfg in "FLIGHT=4 BATCHES=5" "FLIGHT=2 BATCHES=10" "FLIGHT=3 BATCHES=7" "FLIGHT=1 BATCHES=20 GRID_SHARE=100" "FLIGHT=4 BATCHES=5"; do
  echo "== $cfg" >> $O
  env $cfg WORLDS=8,4 K=20 REPS=3 timeout -k 10 200 python tools/share_burst.py >> $O 2>&1 || exit 1
done
echo done
