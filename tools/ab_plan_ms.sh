#!/bin/bash
# plan / stream / step times of the default expand line per library build (interleaved twice)
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do for lib in "$@"; do
  b=$(basename $lib .so)
  GPU_NNUE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --check 0 > $OUT/$b.$rep.json 2> $OUT/$b.$rep.err || { tail -5 $OUT/$b.$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$b.$rep.json'));r=d['roofline'];print('$b', round(d['value']/1e6,1), 'M/s step', d['ms_per_step'], 'stream', r['kernel_ms_per_launch'], 'plan', r.get('plan_kernel_ms'), 'children', r['stage_ms']['write_children'], 'fin', r['stage_ms']['finalize'])"
done; done
