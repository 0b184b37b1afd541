set -o pipefail
# plan_kernel section cycles (GN_PLAN_PROF build) at commit d1b6c5c
OUT=gpurun_out/r04s
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/libgpu_nnue_pprof.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-secondary --no-cpu-baseline --check 0 > $OUT/pprof.json 2> $OUT/pprof.err || { tail -20 $OUT/pprof.err; exit 1; }
grep "plan prof" $OUT/pprof.err | tail -2
