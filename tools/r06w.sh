# round 6: two merged launches in flight (two graph instances per class, the wait without the
# device lock) against one at a time (-DGN_AB_ONE_LEADER): the GPU suite, then the drop-in line
set -o pipefail
mkdir -p gpurun_out/r06w
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06w/pytest.log 2>&1; rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/r06w/pytest.log; [ $rc -eq 0 ] || exit 1
for L in libgpu_nnue_oneleader.so libgpu_nnue.so libgpu_nnue_oneleader.so libgpu_nnue.so; do
  GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/$L timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06w/dropin_$L.json 2> gpurun_out/r06w/dropin_$L.err || { tail -20 gpurun_out/r06w/dropin_$L.err; exit 1; }; echo "$L"; python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['16_callers_coalesced'];print(d['single_caller'],c['positions_per_s'],c['p50_ms'],c['launches'],d['16_callers_serial']['positions_per_s'],d['oracle_check']['mismatches'])" gpurun_out/r06w/dropin_$L.json
done
