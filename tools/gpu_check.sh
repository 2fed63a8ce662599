#!/bin/bash
# The driver's round-end sequence on the GPU box: pytest -m gpu, smoke, the driver's bench
# line (--steps 20 --warmup 5).  Usage: tools/gpu_check.sh TAG [pytest args...]
# Results under gpurun_out/TAG/.
set -o pipefail
TAG=${1:?tag}
shift
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread "$@" \
    > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -3 gpurun_out/$TAG/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit 2
cat gpurun_out/$TAG/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench.json \
    2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/$TAG/bench.json'));print(d['value'],d['ms_per_step'],d.get('frame_check'))"
