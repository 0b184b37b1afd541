set -o pipefail
mkdir -p gpurun_out/r04c
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04c/pytest.log 2>&1 || { tail -40 gpurun_out/r04c/pytest.log; exit 1; }
tail -2 gpurun_out/r04c/pytest.log
timeout -k 10 300 python -u bench.py --dropin > gpurun_out/r04c/dropin.json 2> gpurun_out/r04c/dropin.err || { tail -30 gpurun_out/r04c/dropin.err; exit 1; }
cat gpurun_out/r04c/dropin.json
timeout -k 10 300 python -u bench.py --abi-games 49152 --steps 3 > gpurun_out/r04c/abi.json 2> gpurun_out/r04c/abi.err || { tail -30 gpurun_out/r04c/abi.err; exit 1; }
cat gpurun_out/r04c/abi.json
timeout -k 10 600 python tools/ab.py --variants libgpu_nnue.so libgpu_nnue_kc2.so libgpu_nnue.so libgpu_nnue_kc2.so -- --steps 8 --check 0 || exit 1
GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/libgpu_nnue_pp.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-secondary --no-cpu-baseline --check 0 > gpurun_out/r04c/pp.json 2> gpurun_out/r04c/pp.err || { tail -30 gpurun_out/r04c/pp.err; exit 1; }
grep "plan prof" gpurun_out/r04c/pp.err | tail -3
