set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_x
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc_x -o run -- python bench.py --steps 4 --warmup 0 --inflight 1 --cpu-baseline 0 --seam-stats 0 --count-frame 0 > gpurun_out/pmc_x.log 2>&1
echo rc=$?
