#!/bin/bash
# Default bench line + rocprofv3 kernel-trace stats of the same command + PMC
# passes (one counter group per pass, each its own process) for the expand and
# big16m workloads.  Usage: bash tools/profile_round.sh <tag>; then, locally,
# python tools/pmc_summary.py <tag>.
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-secondary --check 0 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
echo "trace done"
for wl in ${WLS:-expand big16m small1m}; do
  ARGS="--workload $wl --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --check 0"
  timeout -k 10 200 python bench.py $ARGS > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$wl -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_fetch_$wl.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$wl -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_write_$wl.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_l2_$wl -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_l2_$wl.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d $OUT/pmc_mfma_$wl -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_mfma_$wl.log 2>&1 || exit 1
  echo "pmc $wl done"
done
