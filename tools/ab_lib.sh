#!/bin/bash
# A/B of library builds on one box: bash tools/ab_lib.sh <tag> <lib1> <lib2> ... (interleaved twice)
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for lib in "$@"; do
  b=$(basename $lib .so)
  GPU_NNUE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-secondary --check 0 > $OUT/$b.$rep.json 2> $OUT/$b.$rep.err || { tail -5 $OUT/$b.$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$b.$rep.json'));print('$b', round(d['value']/1e6,1), 'M evals/s', d['roofline']['kernel_ms_per_launch'], 'ms')"
done; done
