#!/bin/bash
# Latency-level counters of the expansion kernels (SMEM vs VMEM in flight, scalar cache hits), 16,384 games.
OUT=gpurun_out/${TAG:-sqm}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ARGS="--workload expand --positions 16384 --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --check 0"
timeout -s KILL 90 rocprofv3 --pmc SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d $OUT/p1 -o run --output-format csv -- python bench.py $ARGS > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQ_INST_CYCLES_SMEM -d $OUT/p2 -o run --output-format csv -- python bench.py $ARGS > $OUT/p2.log 2>&1 || exit 1
echo done
