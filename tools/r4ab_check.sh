# tuning re-check under the band-share groups (K = 20)
set -o pipefail
mkdir -p gpurun_out/r4ab5
REPS=4 bash tools/ab_env.sh "RT_X=0" "RT_TUNE=bvh_maxleaf=16" > gpurun_out/r4ab5/ab.txt 2>&1 || exit 1
cat gpurun_out/r4ab5/ab.txt
REPS=3 K=64 bash tools/ab_env.sh "RT_X=0" "RT_TUNE=bvh_maxleaf=16" > gpurun_out/r4ab5/ab64.txt 2>&1 || exit 2
cat gpurun_out/r4ab5/ab64.txt
for r in 1 2; do
  for t in "RT_X=0" "RT_TUNE=bvh_maxleaf=16"; do
    env $t timeout -k 10 200 python tools/frame_async_time.py > gpurun_out/r4ab5/fa.txt 2>&1 || exit 3
    echo "$t $(tail -1 gpurun_out/r4ab5/fa.txt)"
  done
done
