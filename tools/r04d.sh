set -o pipefail
mkdir -p gpurun_out/r04d
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04d/pytest.log 2>&1 || { tail -40 gpurun_out/r04d/pytest.log; exit 1; }
tail -2 gpurun_out/r04d/pytest.log
timeout -k 10 900 python tools/ab.py --variants libgpu_nnue.so libgpu_nnue_r3s.so libgpu_nnue.so libgpu_nnue_r3s.so -- --steps 8 --check 0 || exit 1
GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/libgpu_nnue_pp.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-secondary --no-cpu-baseline --check 0 > gpurun_out/r04d/pp.json 2> gpurun_out/r04d/pp.err || { tail -30 gpurun_out/r04d/pp.err; exit 1; }
grep "plan prof" gpurun_out/r04d/pp.err | tail -3
