#!/bin/bash
# SQ stall/issue counters of expand_eval under each GN_ABLATE setting (16,384 games).
OUT=gpurun_out/sq
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ARGS="--workload expand --positions 16384 --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --check 0"
for a in 0 2 7; do
  GN_ABLATE=$a timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD -d $OUT/a${a}_1 -o run --output-format csv -- python bench.py $ARGS > $OUT/a${a}_1.log 2>&1 || exit 1
  GN_ABLATE=$a timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_BUSY_CU_CYCLES -d $OUT/a${a}_2 -o run --output-format csv -- python bench.py $ARGS > $OUT/a${a}_2.log 2>&1 || exit 1
  echo "a$a done"
done
