set -o pipefail
mkdir -p gpurun_out/r04e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04e/pytest.log 2>&1 || { tail -40 gpurun_out/r04e/pytest.log; exit 1; }
tail -2 gpurun_out/r04e/pytest.log
timeout -k 10 900 python tools/ab.py --variants libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_base.so libgpu_nnue.so -- --steps 8 --check 0 || exit 1
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r04e/bench.json 2> gpurun_out/r04e/bench.err || { tail -30 gpurun_out/r04e/bench.err; exit 1; }
cat gpurun_out/r04e/bench.json
