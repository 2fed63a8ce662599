set -o pipefail
bash tools/gpu_check.sh r4u || exit 1
for r in 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --seam-stats 0 > gpurun_out/r4u/bench_$r.json 2> gpurun_out/r4u/bench_$r.err || exit 2
done
timeout -k 10 300 python bench.py --cpu-baseline 0 --seam-stats 0 > gpurun_out/r4u/bench_k64.json 2> gpurun_out/r4u/bench_k64.err || exit 3
python - <<'PY'
import json
for f in ("bench", "bench_2", "bench_3", "bench_k64"):
    d = json.load(open(f"gpurun_out/r4u/{f}.json"))
    c = d["config"]
    print(f, d["value"], "B", c["frames_per_pass"], "S", c["sub_bands"], "check", d.get("frame_check"), "lat", c["pass_latency_ms"])
PY
