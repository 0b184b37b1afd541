# round 6: full GPU suite on the fixed library (stop at the first failure), the pipeline A/B, the
# drop-in line, small1m / big16m lines
set -o pipefail
mkdir -p gpurun_out/r06j
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06j/pytest.log 2>&1; rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/r06j/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06j/dropin.json 2> gpurun_out/r06j/dropin.err || exit 1; cat gpurun_out/r06j/dropin.json
for P in 2 0 1 2; do
  timeout -k 10 200 python -u tools/ab.py --out gpurun_out/r06j/ab$P --variants libgpu_nnue.so --timeout 180 -- --steps 5 --pipeline $P > gpurun_out/r06j/ab_p$P.log 2>&1 || exit 1; echo "pipeline $P"; cat gpurun_out/r06j/ab_p$P.log
done
for W in small1m big16m; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 5 --no-cpu-baseline --no-secondary > gpurun_out/r06j/$W.json 2> gpurun_out/r06j/$W.err || exit 1; python -c "import json;d=json.load(open('gpurun_out/r06j/$W.json'));print('$W',d['value'],d['ms_per_step'],d['roofline'].get('kernel_ms_per_launch'),d.get('oracle_check'))"
done
