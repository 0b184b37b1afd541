# round 6: bisect test_stream_column_slices_equal_whole_rows (r5 end / HEAD~ / tree), the rest of the
# GPU suite, then per-kernel PMC passes of the expand workload
set -o pipefail
mkdir -p gpurun_out/r06f
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=tests/test_gpu_parity.py::test_stream_column_slices_equal_whole_rows
for L in libgpu_nnue_base.so libgpu_nnue_head.so libgpu_nnue.so; do
  GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/$L timeout -k 10 200 python -u -m pytest $T -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r06f/slices_$L.log 2>&1; echo "$L rc=$?"; tail -2 gpurun_out/r06f/slices_$L.log
done
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --deselect $T > gpurun_out/r06f/pytest.log 2>&1; echo "suite rc=$?"; tail -5 gpurun_out/r06f/pytest.log
timeout -k 10 600 bash tools/pmc_kernels.sh r06f/pk expand > gpurun_out/r06f/pk.log 2>&1; echo "pmc rc=$?"; tail -5 gpurun_out/r06f/pk.log
