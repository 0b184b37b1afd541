set -o pipefail
# column-sliced stream: the other slices' fc_0 sums loaded at the tile start (libgpu_nnue.so) vs in the
# finishing step (libgpu_nnue_old.so, the previous commit); then the slice-equality test on the new one
OUT=gpurun_out/r04zm
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -u tools/ab.py --timeout 240 --variants libgpu_nnue_old.so libgpu_nnue.so libgpu_nnue_old.so libgpu_nnue.so -- --steps 5 > $OUT/ab.log 2>&1 || { tail -30 $OUT/ab.log; exit 1; }
grep -v "^\s*$" $OUT/ab.log | tail -4
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "slices" -x -q --timeout 300 --timeout-method thread > $OUT/test.log 2>&1 || { tail -40 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
