#!/bin/bash
# L2 hit rate and past-L2 bytes of stream_eval per bench variant (one --pmc pass each).
# Usage: VARIANTS="--chain=-81|--chain=-5" bash tools/pmc_ab.sh <tag>   (variants split on |)
TAG=${1:-pmcab}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
IFS='|' read -ra VS <<< "${VARIANTS:---chain=-81}"
i=0
for v in "${VS[@]}"; do
  i=$((i+1))
  ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-secondary --check 0 $v"
  timeout -k 10 200 python bench.py $ARGS > $OUT/v$i.json 2> $OUT/v$i.err || { tail -5 $OUT/v$i.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/l2_v$i -o run --output-format csv -- python bench.py $ARGS > $OUT/l2_v$i.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/f_v$i -o run --output-format csv -- python bench.py $ARGS > $OUT/f_v$i.log 2>&1 || exit 1
  python - "$OUT" "$i" "$v" <<'PY'
import csv, glob, json, sys
out, i, v = sys.argv[1:4]
acc = {}
for grp in ("l2", "f"):
    for p in glob.glob(f"{out}/{grp}_v{i}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if "stream_eval_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]] = acc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
d = json.load(open(f"{out}/v{i}.json"))
h, m = acc.get("TCC_HIT_sum", 0), acc.get("TCC_MISS_sum", 1)
print(v, "kernel_ms", d["roofline"]["kernel_ms_per_launch"], "rows", d["config"]["ft_rows_per_step_per_gpu"],
      "l2_hit %.3f" % (h / (h + m)), "past_L2_GB %.1f" % (acc.get("FETCH_SIZE", 0) * 2048 / 1e9))
PY
done
