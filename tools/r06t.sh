# round 6: the partial sums quarter-major ([slice][quarter][position][4], one contiguous 1 KiB per
# wave load in finalize) against round 5's position-major layout (-DGN_AB_PART_POS_MAJOR), serial
# and pipelined; the sliced-stream parity tests first
set -o pipefail
mkdir -p gpurun_out/r06t
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "slice or expand or pipeline or chunk or depth" > gpurun_out/r06t/pytest.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06t/pytest.log; [ $rc -eq 0 ] || exit 1
for P in 2 0; do
  timeout -k 10 500 python -u tools/ab.py --out gpurun_out/r06t/ab$P --variants libgpu_nnue_posmajor.so libgpu_nnue.so libgpu_nnue_posmajor.so libgpu_nnue.so --timeout 150 -- --steps 5 --pipeline $P > gpurun_out/r06t/ab$P.log 2>&1; rc=$?; echo "ab$P rc=$rc"; cat gpurun_out/r06t/ab$P.log; [ $rc -eq 0 ] || exit 1
done
