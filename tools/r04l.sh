set -o pipefail
# plan_kernel: jps = the king-move jobs' PSQT loads batched; waves per SIMD 3 (lib) / 4 / 5, and the plan without PSQT loads (timing only: wrong PSQT, checks fail)
OUT=gpurun_out/r04l
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -u tools/ab.py --timeout 240 --variants libgpu_nnue.so libgpu_nnue_wpe4.so libgpu_nnue_wpe5.so libgpu_nnue_nopsqt.so libgpu_nnue_jps.so libgpu_nnue.so libgpu_nnue_jps.so -- --steps 3 > $OUT/ab.log 2>&1 || { tail -30 $OUT/ab.log; exit 1; }
grep -v "^\s*$" $OUT/ab.log | tail -8
