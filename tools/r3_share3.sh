#!/bin/bash
# one rank's share of a K = 20 burst at N = 8 / 4 with 3 passes in flight: grid share per pass
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3_share3.txt
: > $O
for cfg in "FLIGHT=3 BATCHES=7 GRID_SHARE=75" "FLIGHT=3 BATCHES=7 GRID_SHARE=50" "FLIGHT=3 BATCHES=7 GRID_SHARE=60" "FLIGHT=3 BATCHES=7 GRID_SHARE=90" "FLIGHT=3 BATCHES=7 GRID_SHARE=100" "FLIGHT=3 BATCHES=7 GRID_SHARE=75"; do
  echo "== $cfg" >> $O
  env $cfg WORLDS=8,4 K=20 REPS=3 timeout -k 10 200 python tools/share_burst.py >> $O 2>&1 || exit 1
done
echo done
