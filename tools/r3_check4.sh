#!/bin/bash
# GPU suite + default bench + every BASELINE config (frame checks)
set -o pipefail
TAG=${1:-r3e}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit 1; fi
timeout -k 10 400 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || exit 2
bash tools/configs_run.sh $TAG.configs || exit 3
echo "done (pytest rc $rc)"
