# round 6: reply_level_kernel at 512 threads (-DGN_RL_THREADS=512, two positions per thread at the
# 1,024-position class) against 256: the fast-batch / coalesce tests on the variant, the drop-in A/B
set -o pipefail
mkdir -p gpurun_out/r06x
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/libgpu_nnue_rl512.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fast_batch or coalesce or dropin" > gpurun_out/r06x/pytest.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06x/pytest.log; [ $rc -eq 0 ] || exit 1
for L in libgpu_nnue.so libgpu_nnue_rl512.so libgpu_nnue.so libgpu_nnue_rl512.so; do
  GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/$L timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06x/dropin_$L.json 2> gpurun_out/r06x/dropin_$L.err || { tail -20 gpurun_out/r06x/dropin_$L.err; exit 1; }; echo "$L"; python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['16_callers_coalesced'];print(d['single_caller'],c['positions_per_s'],c['p50_ms'],c['launches'],d['16_callers_serial']['positions_per_s'],d['oracle_check']['mismatches'])" gpurun_out/r06x/dropin_$L.json
done
