# 32-frame passes: sub-band groups of 4 at K = 20, and the whole-frame K = 64 line unchanged
set -o pipefail
O=gpurun_out/r4t
mkdir -p $O
M=rust_tracer_amd/librt_hip_mf32.so
RT_LIB=$M timeout -k 10 300 python tools/subband_time.py 20 5 > $O/subband_mf32.txt 2>&1 || exit 1
cat $O/subband_mf32.txt
for r in 1 2; do
  RT_LIB=$M timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --seam-stats 0 > $O/k20_mf32_$r.json 2> $O/k20_mf32_$r.err || exit 2
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --seam-stats 0 > $O/k20_base_$r.json 2> $O/k20_base_$r.err || exit 3
  RT_LIB=$M timeout -k 10 300 python bench.py --cpu-baseline 0 --seam-stats 0 > $O/k64_mf32_$r.json 2> $O/k64_mf32_$r.err || exit 4
  timeout -k 10 300 python bench.py --cpu-baseline 0 --seam-stats 0 > $O/k64_base_$r.json 2> $O/k64_base_$r.err || exit 5
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4t/k*.json")):
    d = json.load(open(f))
    c = d["config"]
    print(f.split("/")[-1], d["value"], "B", c["frames_per_pass"], "S", c["sub_bands"], "check", d.get("frame_check"))
PY
