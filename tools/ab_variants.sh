#!/bin/bash
# A/B of kernel variants (GN_EVAL_VARIANT / GN_EXPAND_VARIANT) on one GPU.
# Each run is bounded; the script stops at the first failure.
set -e
mkdir -p gpurun_out/ab
for v in 0 1 2 3; do
  GN_EVAL_VARIANT=$v timeout -k 10 240 python -u bench.py --workload big16m --steps 3 --warmup 1 \
      --no-cpu-baseline --no-secondary --check 1024 > gpurun_out/ab/eval_v$v.json 2> gpurun_out/ab/eval_v$v.err
  python -c "import json;d=json.load(open('gpurun_out/ab/eval_v$v.json'));print('eval v$v', d['value'], d['roofline']['kernel_ms_per_launch'], d['oracle_check'])"
done
for v in 0 1 2; do
  GN_EXPAND_VARIANT=$v timeout -k 10 240 python -u bench.py --workload children --steps 3 --warmup 1 \
      --check 1 > gpurun_out/ab/exp_v$v.json 2> gpurun_out/ab/exp_v$v.err
  python -c "import json;d=json.load(open('gpurun_out/ab/exp_v$v.json'));print('expand v$v', d['value'], d['roofline']['kernel_ms_per_launch'], d['oracle_check'])"
done
GN_EVAL_VARIANT=2 GN_EXPAND_VARIANT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_stream.log 2>&1
tail -2 gpurun_out/ab/pytest_stream.log
