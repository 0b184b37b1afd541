# round 6 (then tools/r06t.sh's partial-sum layout A/B): drop-in A/B -- the two score reductions in one workgroup (default) against two launches
# (-DGN_AB_FAST_TWO_REDUCES), and one position per big-net workgroup (-DGN_TN_MIN=1); the GPU
# suite first (fast-batch graphs against the general path and the oracle)
set -o pipefail
mkdir -p gpurun_out/r06s gpurun_out/r06t
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06s/pytest.log 2>&1; rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/r06s/pytest.log; [ $rc -eq 0 ] || exit 1
for L in libgpu_nnue_tworeduce.so libgpu_nnue.so libgpu_nnue_tn1.so libgpu_nnue_tworeduce.so libgpu_nnue.so libgpu_nnue_tn1.so; do
  GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/$L timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06s/dropin_$L.json 2> gpurun_out/r06s/dropin_$L.err || { tail -20 gpurun_out/r06s/dropin_$L.err; exit 1; }; echo "$L"; python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['single_caller'],d['16_callers_coalesced']['positions_per_s'],d['oracle_check']['mismatches'])" gpurun_out/r06s/dropin_$L.json
done
mkdir -p gpurun_out/r06t
for P in 2 0; do
  timeout -k 10 500 python -u tools/ab.py --out gpurun_out/r06t/ab$P --variants libgpu_nnue_posmajor.so libgpu_nnue.so libgpu_nnue_posmajor.so libgpu_nnue.so --timeout 150 -- --steps 5 --pipeline $P > gpurun_out/r06t/ab$P.log 2>&1; rc=$?; echo "ab$P rc=$rc"; cat gpurun_out/r06t/ab$P.log; [ $rc -eq 0 ] || exit 1
done
