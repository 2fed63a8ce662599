#!/bin/bash
# Run on the GPU box (via gpurun): bench line + rocprofv3 kernel trace + PMC passes.
# usage: tools/gpu_profile.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-r1}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 10 --warmup 2 "$@" > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python bench.py --steps 12 --warmup 4 --cpu-baseline 0 "$@" > $OUT/trace.log 2>&1 || exit 2
# one frame at a time: the per-kernel durations of a frame, unobscured by overlap
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --inflight 1 --batch 1 --cpu-baseline 0 "$@" > $OUT/bench1.json 2> $OUT/bench1.err || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o run -- \
    python bench.py --steps 5 --warmup 1 --inflight 1 --batch 1 --batch 1 --cpu-baseline 0 "$@" > $OUT/trace1.log 2>&1 || exit 7
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
    --output-format csv -d $OUT/pmc_sq -o run -- python bench.py --steps 4 --warmup 0 --inflight 1 --cpu-baseline 0 --count-frame 0 "$@" > $OUT/pmc_sq.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
    python bench.py --steps 4 --warmup 0 --inflight 1 --cpu-baseline 0 --count-frame 0 "$@" > $OUT/pmc_fetch.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
    python bench.py --steps 4 --warmup 0 --inflight 1 --cpu-baseline 0 --count-frame 0 "$@" > $OUT/pmc_write.log 2>&1 || exit 5
echo done
