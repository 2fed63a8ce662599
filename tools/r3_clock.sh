#!/bin/bash
# per wave-iteration timing of one 1080p config-3 frame (librt_hip_clk.so): where the slow tasks sit
set -o pipefail
mkdir -p gpurun_out
RT_LIB=rust_tracer_amd/librt_hip_clk.so timeout -k 10 200 python tools/task_clock.py 3 1 > gpurun_out/r3_clock.txt 2>&1 || exit 1
echo done
