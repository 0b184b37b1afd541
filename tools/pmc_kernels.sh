#!/bin/bash
# Per-kernel PMC passes (instruction mix, wait states, L2 requests) of one bench workload, one
# counter group per rocprofv3 run.  Usage: bash tools/pmc_kernels.sh <tag> [workload] [lib]
# (lib: a file name in fishnet_amd/lib, default the library build); then, on the CPU,
# python tools/pmc_summary.py --kernels <tag>.
TAG=${1:-pk}
WL=${2:-expand}
LIB=${3:-libgpu_nnue.so}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/$LIB
ARGS="--workload $WL --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --check 0"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  timeout -s KILL 150 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pass $i failed: $grp"; tail -5 $OUT/pmc$i.log; exit 1; }
  echo "pass $i done: $grp"
  i=$((i+1))
done
