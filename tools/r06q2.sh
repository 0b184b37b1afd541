# round 6, last rehearsal: the default bench line as the driver runs it (secondary.dropin now with
# its native callers), smoke()
set -o pipefail
mkdir -p gpurun_out/r06q2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06q2/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r06q2/smoke.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r06q2/bench.json 2> gpurun_out/r06q2/bench.err || { tail -20 gpurun_out/r06q2/bench.err; exit 1; }; cat gpurun_out/r06q2/bench.json
