# round 6: full GPU suite on the fixed library, then the pipeline A/B (0 / 1 / 2) and the drop-in line
set -o pipefail
mkdir -p gpurun_out/r06i
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06i/pytest.log 2>&1; rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/r06i/pytest.log; [ $rc -eq 0 ] || exit 1
for P in 2 0 1 2; do
  timeout -k 10 200 python -u tools/ab.py --out gpurun_out/r06i/ab$P --variants libgpu_nnue.so --timeout 180 -- --steps 5 --pipeline $P > gpurun_out/r06i/ab_p$P.log 2>&1; echo "pipeline $P rc=$?"; cat gpurun_out/r06i/ab_p$P.log
done
timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06i/dropin.json 2> gpurun_out/r06i/dropin.err; echo "dropin rc=$?"; cat gpurun_out/r06i/dropin.json
