#!/bin/bash
# Bench + rocprofv3 kernel-trace stats + PMC passes (one counter group per pass).
# Usage: bash tools/profile_round.sh <tag>
set -e
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --check 0 > $OUT/trace.log 2>&1
for wl in expand big16m; do
  ARGS="--workload $wl --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --check 0"
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$wl -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_fetch_$wl.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$wl -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_write_$wl.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d $OUT/pmc_mfma_$wl -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_mfma_$wl.log 2>&1
  echo "pmc $wl done"
done
