#!/bin/bash
# expand ablations (GN_ABLATE bits: 2 = every row load hits the bias row, 4 = no layer stack,
# 8 = no row stream: lists, PSQT and barriers only)
# for a kernel variant (GN_EXPAND_LEGACY=$LEG), 16,384 games.
OUT=gpurun_out/abl2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for leg in ${LEGS:-0}; do
for a in ${ABLATE:-0 2 4 6}; do
  GN_EXPAND_LEGACY=$leg GN_ABLATE=$a timeout -k 10 200 python -u bench.py --workload expand --positions ${POS:-16384} --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --check 0 > $OUT/l$leg.a$a.json 2> $OUT/l$leg.a$a.err || { tail -20 $OUT/l$leg.a$a.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/l$leg.a$a.json'));print('legacy $leg ablate $a kernel_ms', round(d['roofline']['kernel_ms_per_launch'],2))"
done
done
