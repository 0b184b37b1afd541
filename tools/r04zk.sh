set -o pipefail
# column-sliced stream: row ring of 4 entries (default, libgpu_nnue.so) vs 8 (-DGN_RING=8, _r8; 140 VGPRs, 3 waves per SIMD)
OUT=gpurun_out/r04zk
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -u tools/ab.py --timeout 240 --variants libgpu_nnue_r8.so libgpu_nnue.so libgpu_nnue_r8.so libgpu_nnue.so -- --steps 5 > $OUT/ab.log 2>&1 || { tail -30 $OUT/ab.log; exit 1; }
grep -v "^\s*$" $OUT/ab.log | tail -4
