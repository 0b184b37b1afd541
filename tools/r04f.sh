set -o pipefail
OUT=gpurun_out/r04f
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
B="--no-secondary --no-cpu-baseline --check 0"
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], round(d['value']/1e6,1), 'M/s', r['kernel'], r['kernel_ms_per_launch'], 'ms', 'plan', r.get('plan_kernel_ms'))" $1; }
for sw in 1 9 1 9; do
  timeout -k 10 300 python -u bench.py --steps 8 $B --swizzle $sw > $OUT/x_sw$sw.json 2> $OUT/x.err || { tail -20 $OUT/x.err; exit 1; }
  summ $OUT/x_sw$sw.json
done
for lib in libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_base.so libgpu_nnue.so; do
  for wl in small1m big16m; do
    GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/$lib timeout -k 10 300 python -u bench.py --workload $wl --steps 10 $B > $OUT/$wl.$lib.json 2> $OUT/e.err || { tail -20 $OUT/e.err; exit 1; }
    summ $OUT/$wl.$lib.json
  done
done
