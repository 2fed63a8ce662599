#!/bin/bash
# round-3 end-of-work GPU sequence: the driver's order (pytest -m gpu, smoke, default bench)
# then the profile of HEAD (tools/prof3.sh TAG): tools/r3_round.sh TAG
set -o pipefail
TAG=${1:-r3r}
mkdir -p gpurun_out/$TAG
timeout -k 10 420 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit 2
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench_default.json 2> gpurun_out/$TAG/bench_default.err || exit 3
bash tools/prof3.sh $TAG || exit 4
echo done
