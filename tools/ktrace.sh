#!/bin/bash
# per-kernel durations of the render pipeline for one config (rocprofv3 kernel trace)
# usage: tools/ktrace.sh TAG [diag args]
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$TAG -o run -- python tools/diag_runtime.py timing > gpurun_out/$TAG.log 2>&1
