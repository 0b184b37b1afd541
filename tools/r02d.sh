#!/bin/bash
OUT=gpurun_out/r02d; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/dbg_plan.py > $OUT/dbg_new.txt 2>&1; cat $OUT/dbg_new.txt
GN_STREAM=old timeout -k 10 120 python -u tools/dbg_plan.py > $OUT/dbg_old.txt 2>&1; cat $OUT/dbg_old.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; grep -E "FAILED|passed|failed" $OUT/pytest.log | tail -20
