# round 6: the drop-in graph with one evaluation over the batch and both reply levels (the levels
# selected from the boards first): the GPU suite, then the drop-in line against HEAD's library
set -o pipefail
mkdir -p gpurun_out/r06u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06u/pytest.log 2>&1; rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/r06u/pytest.log; [ $rc -eq 0 ] || exit 1
for L in libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_base.so libgpu_nnue.so; do
  GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/$L timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06u/dropin_$L.json 2> gpurun_out/r06u/dropin_$L.err || { tail -20 gpurun_out/r06u/dropin_$L.err; exit 1; }; echo "$L"; python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['single_caller'],d['16_callers_coalesced']['positions_per_s'],d['oracle_check']['mismatches'])" gpurun_out/r06u/dropin_$L.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06u/dropin -o run --output-format csv -- python bench.py --dropin > gpurun_out/r06u/dropin_trace.json 2> gpurun_out/r06u/dropin_trace.err || { tail -20 gpurun_out/r06u/dropin_trace.err; exit 1; }; echo "trace done"
