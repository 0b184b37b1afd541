#!/bin/bash
# expand bench (no checks) over chain lengths K and GN_ABLATE values.  Usage: KS="-81 -27" AB="0 2" bash tools/ab_k.sh tag
TAG=${1:-abk}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for k in ${KS:--81}; do for a in ${AB:-0}; do for kc in ${KC:-1}; do
  GN_ABLATE=$a timeout -k 10 200 python -u bench.py --chain=$k --king-cache=$kc --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --check 0 > $OUT/k$k.a$a.kc$kc.json 2> $OUT/k$k.a$a.kc$kc.err || { tail -5 $OUT/k$k.a$a.kc$kc.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/k$k.a$a.kc$kc.json'));print('K $k ablate $a kc $kc', round(d['value']/1e6,1), 'M/s kernel', d['roofline']['kernel_ms_per_launch'], 'ms rows', d['config']['ft_rows_per_step_per_gpu'])"
done; done; done
