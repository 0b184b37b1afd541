# round 6 (re-entry): GPU suite on the committed library, the drop-in line, stream A/B vs round 5, bench
set -o pipefail
mkdir -p gpurun_out/r06d
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "fast_batch or score_fixture or concurrent or bad_fens or device_blocks" > gpurun_out/r06d/pytest_fast.log 2>&1 || { tail -40 gpurun_out/r06d/pytest_fast.log; exit 1; }
tail -3 gpurun_out/r06d/pytest_fast.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r06d/pytest.log 2>&1 || { tail -40 gpurun_out/r06d/pytest.log; exit 1; }
tail -3 gpurun_out/r06d/pytest.log
timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06d/dropin.json 2> gpurun_out/r06d/dropin.err || { tail -20 gpurun_out/r06d/dropin.err; exit 1; }
cat gpurun_out/r06d/dropin.json
timeout -k 10 700 python -u tools/ab.py --variants libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_base.so libgpu_nnue.so --timeout 160 -- --steps 5 > gpurun_out/r06d/ab.log 2>&1; echo ab rc=$?
cat gpurun_out/r06d/ab.log
