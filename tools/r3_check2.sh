#!/bin/bash
# GPU suite + default bench + the batch-key / animation A/B at the bench defaults
set -o pipefail
TAG=${1:-r3c}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit 1; fi
timeout -k 10 400 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || exit 2
for v in "RT_FRAME_KEYS=frame" "RT_FRAME_KEYS=mixfine"; do
  for a in 0 1; do
    env $v timeout -k 10 200 python bench.py --animate $a --cpu-baseline 0 --count-frame 0 > gpurun_out/ab.json 2>/dev/null || exit 3
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));s=d['seam'];print('$v animate $a', d['value'], d.get('frame_check'), {k:v for k,v in s.items() if 'mpixels' in k or k.endswith('_ms')}, flush=True)" >> gpurun_out/$TAG.keys.txt
  done
done
echo "done (pytest rc $rc)"
