#!/bin/bash
# the default bench line (driver's N = 1 run) and its wall time; config 4 beside it
set -o pipefail
mkdir -p gpurun_out
time timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
time timeout -k 10 400 python bench.py --config 4 --cpu-baseline 0 --seam-stats 0 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit 2
echo done
