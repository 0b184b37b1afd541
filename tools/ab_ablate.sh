#!/bin/bash
# kernel time of the default expand line per library and GN_ABLATE value (timing diagnostics)
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for lib in "$@"; do for a in ${ABL:-0 2 4 6}; do
  b=$(basename $lib .so)
  GN_ABLATE=$a GPU_NNUE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-secondary --check 0 > $OUT/$b.$a.json 2> $OUT/$b.$a.err || { tail -5 $OUT/$b.$a.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$b.$a.json'));print('$b ablate $a', d['roofline']['kernel_ms_per_launch'], 'ms')"
done; done
