set -o pipefail
bash tools/r4l_check.sh || exit 1
bash tools/r4w_check.sh || exit 2
timeout -k 10 200 python tools/kernel_ops.py > gpurun_out/r4l/kernel_ops.txt 2>&1 || exit 3
for rep in 1 2; do
  for br in 8 32 64 272; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --seam-stats 0 --count-frame 0 --check 0 --band-rows $br > gpurun_out/r4l/br.json 2>/dev/null || exit 4
    python -c "import json;d=json.load(open('gpurun_out/r4l/br.json'));print('band_rows $br', d['value'])" >> gpurun_out/r4l/band_rows.txt
  done
done
cat gpurun_out/r4l/band_rows.txt
