# band-share groups through the process-group gather (N = 2's form) on one GPU, and the default line
set -o pipefail
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --steps 20 --warmup 5 --force-gather 1 --cpu-baseline 0 > $O/bench_fg.json 2> $O/bench_fg.err || { tail -20 $O/bench_fg.err; exit 2; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $O/bench.json 2> $O/bench.err || exit 3
python - <<'PY'
import json
for f in ("bench_fg", "bench"):
    d = json.load(open(f"gpurun_out/r4g/{f}.json"))
    c = d["config"]
    print(f, d["value"], "B", c["frames_per_pass"], "S", c["sub_bands"], c["parallelism"], "check", d.get("frame_check"))
PY
