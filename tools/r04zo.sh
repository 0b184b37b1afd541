set -o pipefail
# column-sliced stream: the finish in slice_finish_kernel (libgpu_nnue.so; fc_1 by sdot4, weights in LDS; earlier: _xp 192 B of LDS
# padding per tile row -> 3 waves per SIMD) vs in the last slice's launch (_old, the previous commit);
# the slice-equality test and the games tests first
OUT=gpurun_out/r04zo
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_games.py -k "slices or chained or king_walk" -x -q --timeout 300 --timeout-method thread > $OUT/test.log 2>&1 || { tail -40 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
python -u tools/ab.py --timeout 240 --variants libgpu_nnue_old.so libgpu_nnue.so libgpu_nnue_old.so libgpu_nnue.so -- --steps 5 > $OUT/ab.log 2>&1 || { tail -30 $OUT/ab.log; exit 1; }
grep -v "^\s*$" $OUT/ab.log | tail -4
