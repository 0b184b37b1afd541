#!/bin/bash
# Quick GPU loop: parity tests (default lib) then the expand bench (16,384 games)
# for each library variant in LIBS (default: the default build) and each GN_ABLATE in ABLATE.
OUT=gpurun_out/quick
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ -z "$NOTEST" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for lib in ${LIBS:-libgpu_nnue.so}; do
for a in ${ABLATE:-0}; do
  GPU_NNUE_LIB=$PWD/fishnet_amd/lib/$lib GN_ABLATE=$a timeout -k 10 200 python -u bench.py --workload ${WL:-expand} --positions ${POS:-16384} --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --check ${CHECK:-16} > $OUT/$lib.a$a.json 2> $OUT/$lib.a$a.err || { tail -20 $OUT/$lib.a$a.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$lib.a$a.json'));print('$lib ablate $a kernel_ms', round(d['roofline']['kernel_ms_per_launch'],2), 'evals/s %.4g'%d['value'], d.get('oracle_check'))"
done
done
