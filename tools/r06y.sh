# round 6, final code: the GPU suite, smoke(), the default bench line (CPU baseline and secondary
# lines included) and the kernel-trace stats of the same command
set -o pipefail
mkdir -p gpurun_out/r06y
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r06y/pytest.log 2>&1; rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r06y/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06y/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r06y/smoke.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r06y/bench.json 2> gpurun_out/r06y/bench.err || { tail -20 gpurun_out/r06y/bench.err; exit 1; }; cat gpurun_out/r06y/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06y/trace -o run --output-format csv -- python bench.py --no-cpu-baseline --no-secondary --check 0 > gpurun_out/r06y/trace.log 2>&1 || { tail -20 gpurun_out/r06y/trace.log; exit 1; }; echo "trace done"
