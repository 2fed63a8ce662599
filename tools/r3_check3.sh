#!/bin/bash
# GPU suite + default bench + slots x frames-per-pass sweep at the new defaults
set -o pipefail
TAG=${1:-r3d}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit 1; fi
timeout -k 10 400 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || exit 2
for v in "--inflight 4 --batch 5" "--inflight 2 --batch 10" "--inflight 5 --batch 4" "--inflight 3 --batch 7" "--inflight 1 --batch 16" "--inflight 2 --batch 16 --steps 32"; do
  for rep in 1 2; do
    timeout -k 10 200 python bench.py $v --cpu-baseline 0 --count-frame 0 --seam-stats 0 > gpurun_out/ab.json 2>/dev/null || exit 3
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));c=d['config'];print('$v', d['value'], d.get('frame_check'), c['pass_latency_ms'], round(c['workspace_bytes_all_slots']/1e9,1), flush=True)" >> gpurun_out/$TAG.sweep.txt
  done
done
echo "done (pytest rc $rc)"
