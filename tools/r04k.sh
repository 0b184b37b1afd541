set -o pipefail
# plan_kernel entries built pre-decoded at each put site (lib) vs the committed build (base): A/B, then the GPU suite
OUT=gpurun_out/r04k
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -u tools/ab.py --timeout 240 --variants libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_base.so libgpu_nnue.so -- --steps 3 > $OUT/ab.log 2>&1 || { tail -30 $OUT/ab.log; exit 1; }
cat $OUT/ab.log | grep -v "^\s*$" | tail -8
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
