# round 6: GPU suite, drop-in, small1m, then the default bench line (cpu baseline + secondary lines)
set -o pipefail
mkdir -p gpurun_out/r06k
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06k/pytest.log 2>&1; rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/r06k/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06k/dropin.json 2> gpurun_out/r06k/dropin.err || exit 1; cat gpurun_out/r06k/dropin.json
timeout -k 10 300 python -u bench.py --workload small1m --steps 20 --no-cpu-baseline --no-secondary > gpurun_out/r06k/small1m.json 2> gpurun_out/r06k/small1m.err || exit 1; python -c "import json;d=json.load(open('gpurun_out/r06k/small1m.json'));print('small1m',d['value'],d['roofline'].get('kernel_ms_per_launch'),d.get('oracle_check'))"
timeout -k 10 600 python -u bench.py > gpurun_out/r06k/bench.json 2> gpurun_out/r06k/bench.err || { tail -20 gpurun_out/r06k/bench.err; exit 1; }; cat gpurun_out/r06k/bench.json
