# round 6: GPU suite (fast-batch tests first), the drop-in line, then the stream A/B:
# r5 end (base), HEAD before the ring change (head), this tree (ring 4), ring 5, and the
# SALU/VALU sensitivity builds
set -o pipefail
mkdir -p gpurun_out/r06e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "fast_batch or score_fixture or concurrent or bad_fens or odd_gather" > gpurun_out/r06e/pytest_fast.log 2>&1 || { tail -40 gpurun_out/r06e/pytest_fast.log; exit 1; }
tail -3 gpurun_out/r06e/pytest_fast.log
timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06e/dropin.json 2> gpurun_out/r06e/dropin.err || { tail -20 gpurun_out/r06e/dropin.err; exit 1; }
cat gpurun_out/r06e/dropin.json
timeout -k 10 1000 python -u tools/ab.py --out gpurun_out/r06e/ab --variants libgpu_nnue_base.so libgpu_nnue_head.so libgpu_nnue.so libgpu_nnue_ring5.so libgpu_nnue_head.so libgpu_nnue_ring5.so libgpu_nnue_salu6.so libgpu_nnue_valu8.so --timeout 160 -- --steps 5 > gpurun_out/r06e/ab.log 2>&1; echo ab rc=$?
cat gpurun_out/r06e/ab.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r06e/pytest.log 2>&1 || { tail -40 gpurun_out/r06e/pytest.log; exit 1; }
tail -3 gpurun_out/r06e/pytest.log
