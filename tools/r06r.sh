# round 6: the drop-in's graph -- the big net on its own branch (default) against the serial nets
# (-DGN_AB_FAST_SERIAL_NETS), p50 of one caller; then a kernel trace of the default's drop-in bench
set -o pipefail
mkdir -p gpurun_out/r06r
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in libgpu_nnue_serialnets.so libgpu_nnue.so libgpu_nnue_serialnets.so libgpu_nnue.so; do
  GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/$L timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06r/dropin_$L.json 2> gpurun_out/r06r/dropin_$L.err || { tail -20 gpurun_out/r06r/dropin_$L.err; exit 1; }; echo "$L"; python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['single_caller'],d['16_callers_coalesced']['positions_per_s'],d['oracle_check']['mismatches'])" gpurun_out/r06r/dropin_$L.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r06r/dropin -o run --output-format csv -- python bench.py --dropin > gpurun_out/r06r/dropin_trace.json 2> gpurun_out/r06r/dropin_trace.err || { tail -20 gpurun_out/r06r/dropin_trace.err; exit 1; }; echo "trace done"
