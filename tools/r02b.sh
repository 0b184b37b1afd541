#!/bin/bash
# XCC probe + quick expand bench (old kernel, relaxed tickets) + gpu tests
OUT=gpurun_out/r02b
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
hipcc --offload-arch=gfx950 -O2 tools/xcc_probe.hip -o /tmp/xcc_probe && timeout -k 5 60 /tmp/xcc_probe > $OUT/xcc.txt 2>&1; cat $OUT/xcc.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --check 64 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['roofline']['kernel_ms_per_launch'], d['oracle_check'], d['config']['chain_fallbacks'])"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_l2 -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --check 0 > $OUT/pmc_l2.log 2>&1 || exit 1
python - <<'PY'
import csv, glob, collections
p = sorted(glob.glob('gpurun_out/r02b/pmc_l2/**/*counter_collection.csv', recursive=True))[-1]
acc = collections.defaultdict(float)
for r in csv.DictReader(open(p)):
    if 'expand_stream' in r['Kernel_Name']:
        acc[r['Counter_Name']] += float(r['Counter_Value'])
print(dict(acc), 'hit rate', acc['TCC_HIT_sum'] / (acc['TCC_HIT_sum'] + acc['TCC_MISS_sum']))
PY
