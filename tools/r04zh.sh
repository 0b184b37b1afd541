set -o pipefail
# column-sliced stream (GN_OPT_STREAM_SLICES 3, three launches over 1,024 columns) vs whole rows:
# the equality test, then the default bench line without secondaries
OUT=gpurun_out/r04zh
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "slices" -x -v --timeout 300 --timeout-method thread > $OUT/test.log 2>&1 || { tail -40 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
timeout -k 10 400 python -u bench.py --steps 5 --no-cpu-baseline --no-secondary > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value']/1e6, d['ms_per_step'], r['kernel_ms_per_launch'], r['plan_kernel_ms'], r['stage_ms'], d.get('oracle_check'))"
