set -o pipefail
# eval_net<128>: persistent workgroups, the next tile's boards by LDS-DMA during the current tile (p8: 8 waves per
# SIMD, 13 VGPRs spilled; p7: 7 waves, no spill) vs one tile per workgroup (base, commit bd81357); small1m 20 steps
OUT=gpurun_out/r04w
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -u tools/ab.py --timeout 240 --out gpurun_out/ab_small --variants libgpu_nnue_base.so libgpu_nnue_p8.so libgpu_nnue_p7.so libgpu_nnue_base.so libgpu_nnue_p8.so libgpu_nnue_p7.so -- --workload small1m --steps 20 > $OUT/ab_small.log 2>&1 || { tail -30 $OUT/ab_small.log; exit 1; }
grep -v "^\s*$" $OUT/ab_small.log | tail -6
for v in p8 p7; do GPU_NNUE_LIB=$GRAFT_REPO_ROOT/fishnet_amd/lib/libgpu_nnue_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "small or batch or eval" > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }; tail -1 $OUT/pytest_$v.log; done
