#!/bin/bash
# the driver's round-end sequence at HEAD: pytest -m gpu, smoke, the default bench line
set -o pipefail
TAG=${1:-r3v}
mkdir -p gpurun_out/$TAG
git rev-parse --short=12 HEAD > gpurun_out/$TAG/commit.txt 2>/dev/null
timeout -k 10 420 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit 2
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench_default.json 2> gpurun_out/$TAG/bench_default.err || exit 3
echo done
