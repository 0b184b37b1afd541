set -o pipefail
# round-end rehearsal in the driver's order (GPU suite, smoke, default bench line), outputs to gpurun_out/r04final/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/final_check.sh || exit 1
mkdir -p gpurun_out/r04final && cp gpurun_out/pytest_final.log gpurun_out/smoke_final.log gpurun_out/bench_final.json gpurun_out/r04final/
