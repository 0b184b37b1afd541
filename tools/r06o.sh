# round 6 (r06o, then r06p's front-workgroup A/B): finalize's child-record path as its own instantiation (92 VGPRs, no board code) and the
# 32-bit square: expansion parity tests, A/B against HEAD's library (pipeline 0 and 2), a
# kernel trace of the drop-in bench
set -o pipefail
mkdir -p gpurun_out/r06o gpurun_out/r06p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06o/pytest.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r06o/pytest.log; [ $rc -eq 0 ] || exit 1
for P in 0 2; do
  timeout -k 10 500 python -u tools/ab.py --out gpurun_out/r06o/ab$P --variants libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_base.so libgpu_nnue.so --timeout 150 -- --steps 5 --pipeline $P > gpurun_out/r06o/ab$P.log 2>&1; rc=$?; echo "ab$P rc=$rc"; cat gpurun_out/r06o/ab$P.log; [ $rc -eq 0 ] || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06o/dropin -o run --output-format csv -- python bench.py --dropin > gpurun_out/r06o/dropin.json 2> gpurun_out/r06o/dropin.err || { tail -20 gpurun_out/r06o/dropin.err; exit 1; }; echo "dropin trace done"; cat gpurun_out/r06o/dropin.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u tools/ab.py --out gpurun_out/r06p/ab --variants libgpu_nnue.so libgpu_nnue_fw64.so libgpu_nnue_fw128.so libgpu_nnue_fw64p.so libgpu_nnue.so libgpu_nnue_fw64.so libgpu_nnue_fw128.so libgpu_nnue_fw64p.so --timeout 150 -- --steps 5 --pipeline 2 > gpurun_out/r06p/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06p/ab.log; [ $rc -eq 0 ] || exit 1
GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/libgpu_nnue_fw64p.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06p/trace64p -o run --output-format csv -- python bench.py --steps 3 --no-cpu-baseline --no-secondary --check 0 --pipeline 2 > gpurun_out/r06p/trace64p.log 2>&1 || { tail -20 gpurun_out/r06p/trace64p.log; exit 1; }; echo "trace done"
