set -o pipefail
mkdir -p gpurun_out/r4y
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/r4y/k20.json 2> gpurun_out/r4y/k20.err || exit 1
bash tools/configs_run.sh r4y/cfg || exit 2
for f in k20 cfg/config2 cfg/config3 cfg/config4 cfg/config5; do
  python -c "import json;d=json.load(open('gpurun_out/r4y/$f.json'));c=d['config'];print('$f', d['value'], c['frames_per_pass'], c.get('sub_bands'), d.get('frame_check'), c.get('msamples_per_s'))"
done
