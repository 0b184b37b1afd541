# round 6: GPU suite on the new library (stream decode + small-batch graphs), the stream A/B
# against HEAD, the drop-in line, then the SALU / VALU sensitivity builds
set -o pipefail
mkdir -p gpurun_out/r06c
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "fast_batch or score_fixture or concurrent or bad_fens" > gpurun_out/r06c/pytest_fast.log 2>&1 || { tail -40 gpurun_out/r06c/pytest_fast.log; exit 1; }
tail -3 gpurun_out/r06c/pytest_fast.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06c/pytest.log 2>&1 || { tail -40 gpurun_out/r06c/pytest.log; exit 1; }
tail -3 gpurun_out/r06c/pytest.log
timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06c/dropin.json 2> gpurun_out/r06c/dropin.err || { tail -20 gpurun_out/r06c/dropin.err; exit 1; }
cat gpurun_out/r06c/dropin.json
timeout -k 10 900 python -u tools/ab.py --variants libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_salu6.so libgpu_nnue_salu12.so libgpu_nnue_valu8.so --timeout 200 -- --steps 5 > gpurun_out/r06c/ab.log 2>&1; echo ab rc=$?
cat gpurun_out/r06c/ab.log
