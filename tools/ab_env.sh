#!/bin/bash
# A/B of environment settings on one box: bash tools/ab_env.sh <tag> "ENV=a" "ENV=b" ... (interleaved twice)
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-secondary --check 0 > $OUT/c$i.$rep.json 2> $OUT/c$i.$rep.err || { tail -5 $OUT/c$i.$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c$i.$rep.json'));print('$cfg', round(d['value']/1e6,1), 'M evals/s', d['roofline']['kernel_ms_per_launch'], 'ms')"
done; done
