#!/bin/bash
# Per-kernel times (rocprofv3 --kernel-trace --stats) of the default expand line for library builds.
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for lib in "$@"; do
  b=$(basename $lib .so)
  GPU_NNUE_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$b -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-secondary --check 0 > $OUT/$b.log 2>&1 || { tail -5 $OUT/$b.log; exit 1; }
  f=$(find $OUT/$b -name "*kernel_stats.csv" | head -1)
  echo "== $b"; python - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:8]: print(f"{r['Name'][:60]:60s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e6:9.3f} ms")
PY
done
