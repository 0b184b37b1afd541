# round 6: the expansion front's workgroup size (GN_FRONT_WG 256 / 128 / 64, and 64 with the front
# stream at the highest priority) with the pipeline on: does the front run beside the row stream?
set -o pipefail
mkdir -p gpurun_out/r06p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u tools/ab.py --out gpurun_out/r06p/ab --variants libgpu_nnue.so libgpu_nnue_fw64.so libgpu_nnue_fw128.so libgpu_nnue_fw64p.so libgpu_nnue.so libgpu_nnue_fw64.so libgpu_nnue_fw128.so libgpu_nnue_fw64p.so --timeout 150 -- --steps 5 --pipeline 2 > gpurun_out/r06p/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06p/ab.log; [ $rc -eq 0 ] || exit 1
GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/libgpu_nnue_fw64p.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06p/trace64p -o run --output-format csv -- python bench.py --steps 3 --no-cpu-baseline --no-secondary --check 0 --pipeline 2 > gpurun_out/r06p/trace64p.log 2>&1 || { tail -20 gpurun_out/r06p/trace64p.log; exit 1; }; echo "trace done"
