#!/bin/bash
# Timing-only ablation of expand_eval phases (GN_ABLATE bits: 1 parent refresh,
# 2 slot gathers, 4 layer stack).  Outputs are wrong under ablation; --check 0.
set -e
mkdir -p gpurun_out/abl
for a in ${ABL:-0 1 2 4 6 7}; do
  GN_ABLATE=$a timeout -k 10 200 python -u bench.py --workload expand --positions 16384 --steps 3 --warmup 1 \
     --no-cpu-baseline --no-secondary --check 0 > gpurun_out/abl/a$a.json 2> gpurun_out/abl/a$a.err
  python -c "import json;d=json.load(open('gpurun_out/abl/a$a.json'));print('ablate $a', round(d['roofline']['kernel_ms_per_launch'],2))"
done
