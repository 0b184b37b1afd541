#!/bin/bash
# SQ stall/issue counters of the big-net expansion kernel, 16,384 games, for each
# GN_EXPAND_LEGACY in LEGS and GN_ABLATE in ABLATE.  OUT=gpurun_out/${TAG:-sq}.
OUT=gpurun_out/${TAG:-sq}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
[ -n "$LIST" ] && { timeout -k 5 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true; }
ARGS="--workload expand --positions 16384 --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --check 0"
for leg in ${LEGS:-0}; do
for a in ${ABLATE:-0}; do
  export GN_EXPAND_LEGACY=$leg GN_ABLATE=$a
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD -d $OUT/l${leg}a${a}_1 -o run --output-format csv -- python bench.py $ARGS > $OUT/l${leg}a${a}_1.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_BUSY_CU_CYCLES -d $OUT/l${leg}a${a}_2 -o run --output-format csv -- python bench.py $ARGS > $OUT/l${leg}a${a}_2.log 2>&1 || exit 1
  echo "legacy $leg ablate $a done"
done
done
