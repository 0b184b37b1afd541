#!/bin/bash
# A/B of the big-net expansion kernels: row stream (default) vs per-slot row
# programs (GN_EXPAND_LEGACY=1), expand workload, after the GPU parity tests.
OUT=gpurun_out/ab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ -z "$NOTEST" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for v in ${VARIANTS:-0 1}; do
  GN_EXPAND_LEGACY=$v timeout -k 10 200 python -u bench.py --workload expand --positions ${POS:-16384} --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --check ${CHECK:-16} > $OUT/legacy$v.json 2> $OUT/legacy$v.err || { tail -20 $OUT/legacy$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/legacy$v.json'));print('legacy=$v kernel_ms', round(d['roofline']['kernel_ms_per_launch'],2), 'evals/s %.4g'%d['value'], d.get('oracle_check'))"
done
