set -o pipefail
# stream_eval_kernel time split (GN_STREAM_PROF diagnostics build): row stream / tile barrier / layer stack wave-cycles
OUT=gpurun_out/r04ze
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/libgpu_nnue_sprof.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-secondary --no-cpu-baseline --check 0 > $OUT/sprof.json 2> $OUT/sprof.err || { tail -20 $OUT/sprof.err; exit 1; }
grep "stream prof" $OUT/sprof.err | tail -2
