#!/bin/bash
# GPU check of HEAD: the -m gpu suite, then one bench line (tools/r2_check.sh TAG [bench args])
set -o pipefail
TAG=${1:-r2}; shift
mkdir -p gpurun_out
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())" > gpurun_out/$TAG.host.log
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || exit 2
echo done
