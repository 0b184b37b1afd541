# round 6: bisect test_stream_column_slices_equal_whole_rows (r5 end / HEAD~2 / ring commit / tree),
# the expansion pipeline's test, A/B pipeline on/off, then the rest of the GPU suite
set -o pipefail
mkdir -p gpurun_out/r06g
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=tests/test_gpu_parity.py::test_stream_column_slices_equal_whole_rows
for L in libgpu_nnue_base.so libgpu_nnue_head.so libgpu_nnue_ringc.so libgpu_nnue.so; do
  GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/$L timeout -k 10 200 python -u -m pytest $T -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r06g/slices_$L.log 2>&1; echo "$L rc=$?"; tail -2 gpurun_out/r06g/slices_$L.log
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py::test_expand_pipeline_equals_serial -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r06g/pipe.log 2>&1 || { tail -30 gpurun_out/r06g/pipe.log; exit 1; }
tail -2 gpurun_out/r06g/pipe.log
for P in 1 0 1 0; do
  timeout -k 10 200 python -u tools/ab.py --out gpurun_out/r06g/ab$P --variants libgpu_nnue.so --timeout 180 -- --steps 5 --pipeline $P > gpurun_out/r06g/ab_p$P.log 2>&1; echo "pipeline $P rc=$?"; cat gpurun_out/r06g/ab_p$P.log
done
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --deselect $T > gpurun_out/r06g/pytest.log 2>&1; echo "suite rc=$?"; tail -5 gpurun_out/r06g/pytest.log
timeout -k 10 200 python -u bench.py --dropin > gpurun_out/r06g/dropin.json 2> gpurun_out/r06g/dropin.err; echo "dropin rc=$?"; cat gpurun_out/r06g/dropin.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06g/dtrace -o run --output-format csv -- python bench.py --dropin > gpurun_out/r06g/dtrace.log 2>&1; echo "dtrace rc=$?"
