# round 6: drop-in A/B -- HEAD (two reply-level launches, blocking wait), this tree (both levels in
# one workgroup, a polling wait), and each change alone; the fast-batch and drop-in tests first
set -o pipefail
mkdir -p gpurun_out/r06v
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fast_batch or dropin or coalesce or batch or score" > gpurun_out/r06v/pytest.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06v/pytest.log; [ $rc -eq 0 ] || exit 1
for L in libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_blocking.so libgpu_nnue_twolevel.so libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_blocking.so libgpu_nnue_twolevel.so; do
  GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/$L timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06v/dropin_$L.json 2> gpurun_out/r06v/dropin_$L.err || { tail -20 gpurun_out/r06v/dropin_$L.err; exit 1; }; echo "$L"; python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['single_caller'],d['16_callers_coalesced']['positions_per_s'],d['16_callers_coalesced']['p50_ms'],d['oracle_check']['mismatches'])" gpurun_out/r06v/dropin_$L.json
done
