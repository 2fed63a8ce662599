# A/B of two builds of librt_hip.so at 4 frames in flight and one frame at a time:
# tools/lib_ab.sh NEW_SO OLD_SO
set -o pipefail
for v in new old new old; do
  if [ $v = new ]; then L=$1; else L=$2; fi
  echo "== $v" >> gpurun_out/libab.log
  RT_LIB=$L REPS=3 timeout -k 10 100 python -u tools/ab_inflight.py 3 24 - >> gpurun_out/libab.log 2>&1 || exit 1
  RT_LIB=$L FLIGHT=1 REPS=3 timeout -k 10 100 python -u tools/ab_inflight.py 3 12 - >> gpurun_out/libab.log 2>&1 || exit 1
done
