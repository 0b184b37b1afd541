#!/bin/bash
# FETCH_SIZE / TCC counters against the known byte count of tools/ubench_ring (calibration of
# the HBM-side byte correction for the 16-B-lane row gather)
OUT=gpurun_out/${1:-calib}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- ./tools/ubench_ring.bin > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/l2 -o run --output-format csv -- ./tools/ubench_ring.bin > $OUT/l2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $OUT/ea -o run --output-format csv -- ./tools/ubench_ring.bin > $OUT/ea.log 2>&1 || exit 1
python - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for f in sorted(glob.glob(out + "/*/**/*counter_collection.csv", recursive=True)):
    rows = list(csv.DictReader(open(f)))
    byd = collections.OrderedDict()
    for r in rows:
        d = int(r.get("Dispatch_Id", r.get("Dispatch-Id", 0)))
        byd.setdefault(d, {})[r["Counter_Name"]] = byd.get(d, {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for d, c in list(byd.items())[:40]:
        print(f.split("/")[-3], d, {k: f"{v:.4g}" for k, v in c.items()})
PY
