#!/bin/bash
# A/B: expand_eval one workgroup per parent vs persistent (GN_PERSIST WGs per CU)
OUT=gpurun_out/persist
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
GN_PERSIST=2 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "expand or incremental" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for p in 0 1 2 3 4; do
  GN_PERSIST=$p timeout -k 10 200 python -u bench.py --workload expand --positions 16384 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --check 0 > $OUT/p$p.json 2> $OUT/p$p.err || exit 1
  python -c "import json;d=json.load(open('$OUT/p$p.json'));print('persist $p', round(d['roofline']['kernel_ms_per_launch'],2), d['value'])"
done
