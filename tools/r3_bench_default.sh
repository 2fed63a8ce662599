#!/bin/bash
# the default bench line (driver's N = 1 run) and its wall time
set -o pipefail
mkdir -p gpurun_out
time timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
echo done
