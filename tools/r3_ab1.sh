#!/bin/bash
# round-3 A/B batch 1 (GPU side): powf / workspace cost, seam variants, batch key layouts,
# config 5 sample batches
set -o pipefail
mkdir -p gpurun_out
REPS=2 bash tools/ab_env.sh "RT_NODE_FACTOR=6" "RT_LIB=rust_tracer_amd/librt_hip_ocmlpow.so" "RT_LIB=rust_tracer_amd/librt_hip_ldspow.so" "RT_NODE_FACTOR=12" > gpurun_out/r3ab_pow.txt 2>&1 || exit 1
bash tools/r3_seam.sh r3seam || exit 2
REPS=2 bash tools/ab_env.sh "RT_FRAME_KEYS=frame" "RT_FRAME_KEYS=mix" "RT_FRAME_KEYS=mixfine" "RT_REVERSE=0xfffffffe" > gpurun_out/r3ab_keys.txt 2>&1 || exit 3
for v in "RT_SPP_KEYS=mix" "RT_SPP_KEYS=mixfine" "RT_SPP_KEYS=frame" "RT_SPP_BATCH=1"; do
  env $v timeout -k 10 300 python bench.py --config 5 --steps 4 --warmup 1 --cpu-baseline 0 --seam-stats 0 --count-frame 0 > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 4
  python -c "import json;d=json.load(open('gpurun_out/c5.json'));c=d['config'];print('$v', d['value'], c['msamples_per_s'], d.get('frame_check'), c['workspace_bytes_per_slot'], flush=True)" >> gpurun_out/r3ab_c5.txt
done
echo done
