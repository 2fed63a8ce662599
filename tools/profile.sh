#!/bin/bash
# GPU side of a profile of the headline workload (config 3, 1080p, depth 8):
#   bench.json      the driver's line (--steps 20 --warmup 5)
#   trace/          rocprofv3 kernel trace of that run (kernels overlap: 4 passes in flight)
#   trace1/         kernel trace one frame at a time (--inflight 1 --batch 1): exclusive times
#   pmc_*_bN[sS]/   PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) for passes of N = 1, 5, 16 frames
#                   on one slot, and 20 frames over S = 4 band shares (PMC collection serialises
#                   the dispatches anyway)
# usage: tools/profile.sh TAG   -> gpurun_out/TAG/   (summary: tools/profile_summary.py TAG)
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="--cpu-baseline 0 --seam-stats 0 --check 0"
cat /sys/fs/cgroup/cpu.max > $OUT/cpu_max.txt 2>/dev/null
python -c "from rust_tracer_amd.provenance import sources_sha; print(sources_sha())" > $OUT/sources_sha.txt || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --seam-stats 0 > $OUT/bench.json 2> $OUT/bench.err || exit 2
echo bench; cat $OUT/bench.json | head -c 300; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python bench.py --steps 20 --warmup 5 $B --count-frame 0 > $OUT/trace.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o run -- \
    python bench.py --steps 6 --warmup 1 --inflight 1 --batch 1 $B --count-frame 0 > $OUT/trace1.log 2>&1 || exit 4
echo traces
SIZES=${SIZES:-1 5 16 20/4 32/2}  # (commas or spaces)
# a size N/S: passes of N frames over S band shares of the device (bench.py --sub-bands S; the
# driver's K = 20 runs 20/4), one group of S slots
for spec in ${SIZES//,/ }; do
  n=${spec%/*}; s=1; [ "$spec" != "$n" ] && s=${spec#*/}
  args="--steps $n --warmup 0 --inflight $s --sub-bands $s --batch $n $B --count-frame 0"
  [ "$s" = 1 ] && suf=$n || suf=${n}s$s
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_b$suf -o run -- \
      python bench.py $args > $OUT/pmc_fetch_b$suf.log 2>&1 || exit 5
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_b$suf -o run -- \
      python bench.py $args > $OUT/pmc_write_b$suf.log 2>&1 || exit 6
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
      --output-format csv -d $OUT/pmc_sq_b$suf -o run -- python bench.py $args > $OUT/pmc_sq_b$suf.log 2>&1 || exit 7
  echo pmc $spec
done
echo done
