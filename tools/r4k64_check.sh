set -o pipefail
mkdir -p gpurun_out/r4k64
for r in 1 2; do
  for sb in 1 2 4; do
    timeout -k 10 300 python bench.py --steps 64 --warmup 4 --cpu-baseline 0 --seam-stats 0 --count-frame 0 --check 0 --sub-bands $sb > gpurun_out/r4k64/b.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r4k64/b.json'));c=d['config'];print('K=64 sub_bands $sb', d['value'], c['frames_per_pass'], c['passes_in_flight'])"
  done
  for sb in 1 2 4; do
    timeout -k 10 300 python bench.py --steps 40 --warmup 4 --cpu-baseline 0 --seam-stats 0 --count-frame 0 --check 0 --sub-bands $sb > gpurun_out/r4k64/b.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r4k64/b.json'));c=d['config'];print('K=40 sub_bands $sb', d['value'], c['frames_per_pass'], c['passes_in_flight'])"
  done
done
