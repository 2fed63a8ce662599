#!/bin/bash
# Every BASELINE config at HEAD (bench.py --config C at its default K, frame_check), GPU side:
# tools/configs_run.sh TAG -> gpurun_out/TAG/config{2,3,4,5}.json
set -o pipefail
OUT=gpurun_out/${1:-configs}
mkdir -p $OUT
for c in 2 3 4; do
  timeout -k 10 300 python bench.py --config $c --warmup 4 --check 1 --cpu-baseline 0 --seam-stats 0 --count-frame 0 > $OUT/config$c.json 2> $OUT/config$c.err || exit $c
done
timeout -k 10 400 python bench.py --config 5 --steps 4 --warmup 1 --check 1 --cpu-baseline 0 --seam-stats 0 --count-frame 0 > $OUT/config5.json 2> $OUT/config5.err || exit 5
echo done
