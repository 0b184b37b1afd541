#!/bin/bash
# A/B of the chained walk's block length (GN_OPT_CHAIN; -k = exactly k), expand workload,
# after the chained-walk parity tests; HEADLIB=<lib> adds a run of another build.
OUT=gpurun_out/ab_chain
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "chain or expand" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="python -u bench.py --workload expand --positions ${POS:-16384} --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --check ${CHECK:-16}"
if [ -n "$HEADLIB" ]; then
  GPU_NNUE_LIB=$HEADLIB timeout -k 10 200 $B > $OUT/head.json 2> $OUT/head.err || { tail -20 $OUT/head.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/head.json'));print('head kernel_ms', round(d['roofline']['kernel_ms_per_launch'],2), 'evals/s %.4g'%d['value'])"
fi
for v in ${VARIANTS:-1 -81:0 -81:1}; do
  ch=${v%%:*}; kc=${v#*:}; [ "$kc" = "$v" ] && kc=1
  timeout -k 10 200 $B --chain=$ch --king-cache=$kc > $OUT/chain$v.json 2> $OUT/chain$v.err || { tail -20 $OUT/chain$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/chain$v.json'));print('chain:kc=$v kernel_ms', round(d['roofline']['kernel_ms_per_launch'],2), 'evals/s %.4g'%d['value'], 'rows', d['config']['ft_rows_per_step_per_gpu'], d.get('oracle_check'))"
done
