set -o pipefail
# plan_kernel: job PSQT stored with the slots + packed job descriptor (np) vs commit bbe8305 (base)
OUT=gpurun_out/r04q
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -u tools/ab.py --timeout 240 --variants libgpu_nnue_base.so libgpu_nnue_np.so libgpu_nnue_base.so libgpu_nnue_np.so -- --steps 3 > $OUT/ab.log 2>&1 || { tail -30 $OUT/ab.log; exit 1; }
grep -v "^\s*$" $OUT/ab.log | tail -4
