set -o pipefail
# eval_net<128>: fc_1 weights loaded with no branch around them (one round trip for the layer stack's loads) (lib) vs base; GPU suite
OUT=gpurun_out/r04z
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -u tools/ab.py --timeout 240 --out gpurun_out/ab_small --variants libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_base.so libgpu_nnue.so -- --workload small1m --steps 20 > $OUT/ab_small.log 2>&1 || { tail -30 $OUT/ab_small.log; exit 1; }
grep -v "^\s*$" $OUT/ab_small.log | tail -4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
