set -o pipefail
# column-sliced stream: 4 waves per SIMD (GN_SLICE_WPE 4, 109 VGPRs; libgpu_nnue.so) vs 3 (125 VGPRs; _w3)
OUT=gpurun_out/r04zi
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -u tools/ab.py --timeout 240 --variants libgpu_nnue_w3.so libgpu_nnue.so libgpu_nnue_w3.so libgpu_nnue.so -- --steps 5 --check 0 > $OUT/ab.log 2>&1 || { tail -30 $OUT/ab.log; exit 1; }
grep -v "^\s*$" $OUT/ab.log | tail -4
