#!/bin/bash
# kernel-trace stats + L2 hit / FETCH / WRITE of one expand step.  Usage: bash tools/prof_quick.sh <tag> [bench args]
TAG=${1:-pq}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-secondary --check 0 $@"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py $ARGS > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_l2 -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_l2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || exit 1
python - "$OUT" <<'PY'
import csv, glob, collections, sys
out = sys.argv[1]
ks = sorted(glob.glob(out + '/trace/**/*kernel_stats.csv', recursive=True))[-1]
for r in csv.DictReader(open(ks)):
    print('%-60s calls %4s avg_ms %.3f tot_ms %.3f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e6, float(r['TotalDurationNs'])/1e6))
for tag in ('pmc_l2', 'pmc_fetch'):
    p = sorted(glob.glob(out + f'/{tag}/**/*counter_collection.csv', recursive=True))[-1]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(p)):
        acc[r['Kernel_Name'][:40]][r['Counter_Name']] += float(r['Counter_Value'])
    for k, v in acc.items():
        if 'stream' in k or 'plan' in k or 'eval_net' in k:
            d = dict(v)
            if 'TCC_HIT_sum' in d:
                d['hit'] = d['TCC_HIT_sum'] / max(1, d['TCC_HIT_sum'] + d['TCC_MISS_sum'])
            if 'FETCH_SIZE' in d:
                d['fetch_GB_x2'] = d['FETCH_SIZE'] * 1024 * 2 / 1e9
            print(tag, k, d)
PY
