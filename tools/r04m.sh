set -o pipefail
# plan_kernel: inputs prefetched one parent ahead, PSQT loads before any wait, DPP scans, uniform wave index
# (lib, 3 waves per SIMD; pf4: 4) vs the committed build (base): GPU suite, then A/B; then eval_net<128> variants
OUT=gpurun_out/r04m
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
python -u tools/ab.py --timeout 240 --variants libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_pf4.so libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_pf4.so -- --steps 3 > $OUT/ab.log 2>&1 || { tail -30 $OUT/ab.log; exit 1; }
grep -v "^\s*$" $OUT/ab.log | tail -8
# eval_net<128>: FT rows in flight per thread / waves per SIMD (lib: 8 / 5; s48 = round-3 shape)
python -u tools/ab.py --timeout 240 --out gpurun_out/ab_small --variants libgpu_nnue_s48.so libgpu_nnue.so libgpu_nnue_s66.so libgpu_nnue_s84.so libgpu_nnue_s48.so libgpu_nnue.so -- --workload small1m --steps 20 > $OUT/ab_small.log 2>&1 || { tail -30 $OUT/ab_small.log; exit 1; }
grep -v "^\s*$" $OUT/ab_small.log | tail -8
# block size (parents per chained block): L2 hits against chain breaks
for k in 41 27; do timeout -k 10 300 python -u bench.py --steps 3 --no-secondary --no-cpu-baseline --chain -$k > $OUT/chain$k.json 2> $OUT/chain$k.err || { tail -20 $OUT/chain$k.err; exit 1; }; python3 -c "
import json,sys; d=json.load(open('$OUT/chain$k.json')); r=d['roofline']
print('chain $k', d['value'], d['ms_per_step'], r['kernel_ms_per_launch'], r.get('plan_kernel_ms'), d['config'].get('ft_rows_per_step_per_gpu'), d['oracle_check']['vs_plain_path'])"; done
