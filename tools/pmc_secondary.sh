#!/bin/bash
# The PMC passes of profile_round.sh for the secondary workloads (big16m, small1m) into
# gpurun_out/${TAG:-r03a}/, as a call of its own.  Usage: TAG=<tag> bash tools/pmc_secondary.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r03a}
mkdir -p $OUT
for wl in big16m small1m; do
  ARGS="--workload $wl --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --check 0"
  timeout -k 10 200 python bench.py $ARGS > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$wl -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_fetch_$wl.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$wl -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_write_$wl.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum -d $OUT/pmc_l2_$wl -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_l2_$wl.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d $OUT/pmc_mfma_$wl -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_mfma_$wl.log 2>&1 || exit 1
  echo "pmc $wl done"
done
