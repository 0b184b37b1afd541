#!/bin/bash
# Quick GPU loop: expand/eval parity subset, then the expand bench (small) and ablations.
OUT=gpurun_out/quick
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for a in ${ABLATE:-0}; do
  GN_ABLATE=$a timeout -k 10 200 python -u bench.py --workload expand --positions 16384 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --check ${CHECK:-16} > $OUT/a$a.json 2> $OUT/a$a.err || { tail -20 $OUT/a$a.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/a$a.json'));print('ablate $a kernel_ms', round(d['roofline']['kernel_ms_per_launch'],2), 'evals/s %.4g'%d['value'], d.get('oracle_check'))"
done
