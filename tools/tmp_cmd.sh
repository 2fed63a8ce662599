set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cull_stress.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/stress.log 2>&1
echo "stress rc=$?"
for b in 1 2 4; do timeout -k 10 200 python bench.py --steps 20 --warmup 4 --batch $b --cpu-baseline 0 --seam-stats 0 --count-frame 0 > gpurun_out/b$b.json 2>/dev/null || exit 3; done
echo done
