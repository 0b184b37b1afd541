# round 6: the drop-in line with its native-thread callers (tools/dropin_native.c)
set -o pipefail
mkdir -p gpurun_out/r06n2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --dropin > gpurun_out/r06n2/dropin.json 2> gpurun_out/r06n2/dropin.err || { tail -20 gpurun_out/r06n2/dropin.err; exit 1; }; cat gpurun_out/r06n2/dropin.json
