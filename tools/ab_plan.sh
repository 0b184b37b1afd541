#!/bin/bash
# GPU suite + planned vs round-1 stream (GN_STREAM=old) on the default expand line.
# Usage: bash tools/ab_plan.sh <tag> [extra bench args]
TAG=${1:-plan}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
fi
for v in new ${OLD:+old}; do
  GN_STREAM=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --check 64 "$@" > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail -20 $OUT/bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('$v', round(d['value']/1e6,1), 'M evals/s', d['roofline']['kernel_ms_per_launch'], 'ms', d['config']['ft_rows_per_step_per_gpu'], 'rows', d['roofline']['stage_ms'], d['oracle_check']['oracle']['mismatching_parents'], d['oracle_check']['vs_plain_path']['equal'])"
done
