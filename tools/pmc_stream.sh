#!/bin/bash
# PMC passes (one group per process) over one default expand step: HBM-side bytes and L2 hits.
TAG=${1:-r02pmc}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ARGS="--workload expand --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --check 0"
timeout -k 10 200 python bench.py $ARGS > $OUT/bench_expand.json 2> $OUT/bench_expand.err || exit 1
GPU_NNUE_LIB=$PWD/fishnet_amd/lib/libgpu_nnue_prof.so GN_EXPAND_CHUNKS=1 timeout -k 10 200 python bench.py $ARGS > $OUT/prof.json 2> $OUT/prof.err || exit 1
grep "stream prof" $OUT/prof.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_expand -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_expand -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_l2_expand -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_l2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $OUT/pmc_tcp_expand -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_tcp.log 2>&1 || exit 1
python - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for f in sorted(glob.glob(out + "/pmc_*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", r.get("Kernel-Name", ""))
        if "stream_eval" in k or "plan_kernel" in k or "write_children" in k:
            acc[(k.split("(")[0][-30:], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, c), v in sorted(acc.items()): print(f.split("/")[-3], k, c, f"{v:.4g}")
PY
