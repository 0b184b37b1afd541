# round 6, final code: the GPU suite, smoke(), the drop-in line, then the round's profile (default bench
# line, kernel-trace stats of the same command, PMC passes; tools/profile_round.sh)
set -o pipefail
mkdir -p gpurun_out/r06z
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r06z/pytest.log 2>&1; rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r06z/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06z/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r06z/smoke.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06z/dropin.json 2> gpurun_out/r06z/dropin.err || { tail -20 gpurun_out/r06z/dropin.err; exit 1; }; cat gpurun_out/r06z/dropin.json
bash tools/profile_round.sh r06z
