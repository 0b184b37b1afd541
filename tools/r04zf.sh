set -o pipefail
# chained-walk link found per parent in child_moves_kernel (libgpu_nnue.so) vs per child by packing
# (libgpu_nnue_old.so, built from the previous commit): A/B (same pads = same links) and the GPU suite
OUT=gpurun_out/r04zf
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -u tools/ab.py --timeout 240 --variants libgpu_nnue_old.so libgpu_nnue.so -- --steps 5 > $OUT/ab.log 2>&1 || { tail -30 $OUT/ab.log; exit 1; }
grep -v "^\s*$" $OUT/ab.log | tail -2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
