# round 6: finalize reads the children's ChildInfo records (no do_move / in_check per child):
# the expansion parity tests, then A/B against HEAD's library with the pipeline on (2) and off (0),
# then kernel traces of the default bench line in both modes
set -o pipefail
mkdir -p gpurun_out/r06n
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "expand or pipeline or chunk or depth or score or slices" > gpurun_out/r06n/pytest.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r06n/pytest.log; [ $rc -eq 0 ] || exit 1
for P in 2 0; do
  timeout -k 10 500 python -u tools/ab.py --out gpurun_out/r06n/ab$P --variants libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_base.so libgpu_nnue.so --timeout 150 -- --steps 5 --pipeline $P > gpurun_out/r06n/ab$P.log 2>&1; rc=$?; echo "ab$P rc=$rc"; cat gpurun_out/r06n/ab$P.log; [ $rc -eq 0 ] || exit 1
done
for P in 2 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06n/trace$P -o run --output-format csv -- python bench.py --steps 3 --no-cpu-baseline --no-secondary --check 0 --pipeline $P > gpurun_out/r06n/trace$P.log 2>&1 || { tail -20 gpurun_out/r06n/trace$P.log; exit 1; }; echo "trace $P done"
done
