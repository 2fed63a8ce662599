#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc1
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc1/avail.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    --output-format csv -d gpurun_out/pmc1/sq -o run -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/pmc1/sq.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SMEM SQ_INST_CYCLES_SMEM SQ_BUSY_CYCLES \
    --output-format csv -d gpurun_out/pmc1/sq2 -o run -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/pmc1/sq2.log 2>&1 || exit 4
echo done
