# sub-band slot groups: parity tests, then the driver's bench line with and without them
set -o pipefail
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "direct or sub_bands or pipeline or batch" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $O/bench_s2_$r.json 2> $O/bench_s2_$r.err || exit 2
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --seam-stats 0 --sub-bands 1 > $O/bench_s1_$r.json 2> $O/bench_s1_$r.err || exit 3
done
python - <<'PY'
import json
for f in ("s2_1", "s1_1", "s2_2", "s1_2"):
    d = json.load(open(f"gpurun_out/r4s/bench_{f}.json"))
    c = d["config"]
    print(f, d["value"], c["frames_per_pass"], c["sub_bands"], c["passes_in_flight"], "check", d.get("frame_check"), d["roofline"]["frac"])
PY
timeout -k 10 200 python tools/kernel_ops.py > $O/kernel_ops.txt 2>&1 || exit 4
RT_LIB=rust_tracer_amd/librt_hip_mf32.so timeout -k 10 300 python tools/subband_time.py 20 5 > $O/subband_mf32.txt 2>&1 || exit 5
