#!/bin/bash
# GPU side of a round-3 profile: bench lines, kernel traces (bench defaults and one frame at
# a time) and PMC passes (HBM FETCH / WRITE, SQ), each its own run; the PMC passes once for
# one frame per pass and once for a BIG-frame pass (default 16, the headline pass size).
# usage: tools/prof3.sh TAG   -> gpurun_out/TAG/
set -o pipefail
TAG=${1:-r3p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="--cpu-baseline 0 --seam-stats 0 --check 0"
cat /sys/fs/cgroup/cpu.max > $OUT/cpu_max.txt 2>/dev/null
git rev-parse --short=12 HEAD > $OUT/commit.txt 2>/dev/null
# the bench defaults (K = 64, passes of up to 16 frames) and a PMC pass of that size
BIG=${BIG:-16}
timeout -k 10 300 python bench.py --warmup 4 --cpu-baseline 0 --seam-stats 0 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --inflight 1 --batch 1 $B > $OUT/bench1.json 2> $OUT/bench1.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python bench.py --warmup 4 $B --count-frame 0 > $OUT/trace.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o run -- \
    python bench.py --steps 6 --warmup 1 --inflight 1 --batch 1 $B --count-frame 0 > $OUT/trace1.log 2>&1 || exit 4
P1="--steps 4 --warmup 0 --inflight 1 --batch 1 $B --count-frame 0"
PB="--steps $BIG --warmup 0 --inflight 1 --batch $BIG $B --count-frame 0"
for cfg in "1:$P1" "$BIG:$PB"; do
  n=${cfg%%:*}; args=${cfg#*:}
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_b$n -o run -- \
      python bench.py $args > $OUT/pmc_fetch_b$n.log 2>&1 || exit 5
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_b$n -o run -- \
      python bench.py $args > $OUT/pmc_write_b$n.log 2>&1 || exit 6
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
      --output-format csv -d $OUT/pmc_sq_b$n -o run -- python bench.py $args > $OUT/pmc_sq_b$n.log 2>&1 || exit 7
done
echo done
