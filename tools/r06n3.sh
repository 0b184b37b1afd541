# round 6: two merged launches in flight (-DGN_MAX_LEADERS=2) against one, with the native callers
# (the drop-in line's 16_callers_native) -- the variant library is loaded by both the bench process
# and its native child (GPU_NNUE_LIB for the bench; the child links fishnet_amd/lib/libgpu_nnue.so,
# so the variant is copied over it in a scratch copy of the tree first)
set -o pipefail
mkdir -p gpurun_out/r06n3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for V in one two one two; do
  if [ $V = two ]; then cp fishnet_amd/lib/libgpu_nnue_lead2.so fishnet_amd/lib/libgpu_nnue.so; else cp fishnet_amd/lib/libgpu_nnue_one.so fishnet_amd/lib/libgpu_nnue.so; fi
  GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/libgpu_nnue.so timeout -k 10 300 python -u bench.py --dropin > gpurun_out/r06n3/dropin_$V.json 2> gpurun_out/r06n3/dropin_$V.err || { tail -20 gpurun_out/r06n3/dropin_$V.err; exit 1; }
  echo "$V"; python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['16_callers_coalesced'];n=d['16_callers_native'];print(d['single_caller']['p50_ms'],c['positions_per_s'],c['launches'],n['positions_per_s'],n['p50_ms'],n['p99_ms'],n['launches'],n['records_equal_to_single_thread'])" gpurun_out/r06n3/dropin_$V.json
done
cp fishnet_amd/lib/libgpu_nnue_one.so fishnet_amd/lib/libgpu_nnue.so
