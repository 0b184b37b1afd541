set -o pipefail
OUT=gpurun_out/r04i
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="--no-secondary --no-cpu-baseline --check 0"
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], round(d['value']/1e6,1), 'M/s', r['kernel'], r['kernel_ms_per_launch'], 'ms')" $1; }
for lib in libgpu_nnue_v0.so libgpu_nnue_tb.so libgpu_nnue_ls.so libgpu_nnue_v0.so libgpu_nnue_tb.so libgpu_nnue_ls.so; do
  for wl in small1m big16m; do
    GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/$lib timeout -k 10 300 python -u bench.py --workload $wl --steps 10 $B > $OUT/$wl.$lib.json 2> $OUT/e.err || { tail -20 $OUT/e.err; exit 1; }
    summ $OUT/$wl.$lib.json
  done
done
