set -o pipefail
# per-slice launch durations (kernel trace) of the prefetching sliced stream
OUT=gpurun_out/r04zn
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline --check 0 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r04zn/trace/**/*kernel_trace.csv', recursive=True)[0]
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in csv.DictReader(open(f)) if 'stream_eval' in r['Kernel_Name']]
print([round(x, 2) for x in d])
PY
