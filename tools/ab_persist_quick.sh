OUT=gpurun_out/persist2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for p in 0 3 4 6; do
  GN_PERSIST=$p timeout -k 10 200 python -u bench.py --workload expand --positions 16384 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --check 0 > $OUT/p$p.json 2> $OUT/p$p.err || exit 1
  python -c "import json;d=json.load(open('$OUT/p$p.json'));print('persist $p', round(d['roofline']['kernel_ms_per_launch'],2), d['value'])"
done
