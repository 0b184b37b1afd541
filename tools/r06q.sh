# round 6: reply_level_kernel with one move generation and the replies made in parallel, the front
# kernels at 2-wave workgroups: the whole GPU suite, the drop-in bench against HEAD's library, the
# expansion A/B (pipeline 2)
set -o pipefail
mkdir -p gpurun_out/r06q
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06q/pytest.log 2>&1; rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/r06q/pytest.log; [ $rc -eq 0 ] || exit 1
for L in libgpu_nnue_base.so libgpu_nnue.so; do
  GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/$L timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06q/dropin_$L.json 2> gpurun_out/r06q/dropin_$L.err || { tail -20 gpurun_out/r06q/dropin_$L.err; exit 1; }; echo "$L"; python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['single_caller'],d['16_callers_coalesced']['positions_per_s'],d['oracle_check']['mismatches'])" gpurun_out/r06q/dropin_$L.json
done
timeout -k 10 500 python -u tools/ab.py --out gpurun_out/r06q/ab --variants libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_base.so libgpu_nnue.so --timeout 150 -- --steps 5 > gpurun_out/r06q/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06q/ab.log; [ $rc -eq 0 ] || exit 1
