set -o pipefail
mkdir -p gpurun_out/r04b
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04b/pytest.log 2>&1 || { tail -40 gpurun_out/r04b/pytest.log; exit 1; }
tail -3 gpurun_out/r04b/pytest.log
timeout -k 10 300 python -u bench.py --dropin > gpurun_out/r04b/dropin.json 2> gpurun_out/r04b/dropin.err || { tail -30 gpurun_out/r04b/dropin.err; exit 1; }
cat gpurun_out/r04b/dropin.json
timeout -k 10 300 python -u bench.py --abi-games 49152 --steps 3 > gpurun_out/r04b/abi.json 2> gpurun_out/r04b/abi.err || { tail -30 gpurun_out/r04b/abi.err; exit 1; }
cat gpurun_out/r04b/abi.json
