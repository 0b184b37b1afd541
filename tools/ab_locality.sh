#!/bin/bash
# A/B of L2-locality options on one GPU (each run bounded, stop on failure).
set -e
mkdir -p gpurun_out/ab2
run() { # name, args...
  local name=$1; shift
  timeout -k 10 240 python -u bench.py "$@" > gpurun_out/ab2/$name.json 2> gpurun_out/ab2/$name.err
  python -c "import json;d=json.load(open('gpurun_out/ab2/$name.json'));print('$name', d['value'], d['roofline']['kernel_ms_per_launch'], d.get('oracle_check'))"
}
run eval_s0_k0 --workload big16m --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --check 1024 --swizzle 0 --king-sort 0
run eval_s1_k0 --workload big16m --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --check 1024 --swizzle 1 --king-sort 0
run eval_s1_k1 --workload big16m --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --check 1024 --swizzle 1 --king-sort 1
run eval_s0_k1 --workload big16m --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --check 1024 --swizzle 0 --king-sort 1
run exp_s0 --workload children --steps 3 --warmup 1 --check 1 --swizzle 0
run exp_s1 --workload children --steps 3 --warmup 1 --check 1 --swizzle 1
