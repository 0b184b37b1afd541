set -o pipefail
# column-sliced stream: block claiming (default XCD-local eighths, swizzle 9) vs one in-order counter (swizzle 1)
# vs static eighths (swizzle 5), and without the king block order (king-sort 0)
OUT=gpurun_out/r04zl
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="--steps 5 --no-secondary --no-cpu-baseline --check 0"
for v in "--swizzle 9" "--swizzle 1" "--swizzle 5" "--king-sort 0" "--swizzle 9"; do
  timeout -k 10 300 python -u bench.py $A $v > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$OUT/b.json'));r=d['roofline'];print(sys.argv[1:], round(d['value']/1e6,1), r['kernel_ms_per_launch'], r['plan_kernel_ms'], r.get('frac'))" $v | tee -a $OUT/sum.txt
done
