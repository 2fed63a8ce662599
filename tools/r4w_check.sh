# rank 0's share at N = 2 / 4 / 8 (one GPU): whole-frame slots vs band-share groups, K = 20
set -o pipefail
O=gpurun_out/r4w
mkdir -p $O
for w in 8 4 2; do
  WORLD=$w F=3 MODES="frames" timeout -k 10 200 python tools/subband_time.py 20 5 >> $O/subband.txt 2>&1 || exit 1
  WORLD=$w F=4 MODES="frames bands2 bands4" timeout -k 10 300 python tools/subband_time.py 20 5 >> $O/subband.txt 2>&1 || exit 2
done
grep K= $O/subband.txt
