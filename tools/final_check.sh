#!/bin/bash
# Round-end check on the GPU box, in the driver's order: the GPU suite, smoke(), then the
# default bench line (N=1).  Each step has its own time limit; the first failure ends it.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_final.log 2>&1 || { tail -30 gpurun_out/pytest_final.log; exit 1; }
tail -1 gpurun_out/pytest_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/smoke_final.log 2>&1 || { tail -30 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err \
    || { tail -30 gpurun_out/bench_final.err; exit 1; }
cat gpurun_out/bench_final.json
