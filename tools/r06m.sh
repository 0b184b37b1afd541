# round 6: kernel traces of the default bench line with the pipeline (mode 2) and without (0), to see
# what runs beside finalize
set -o pipefail
mkdir -p gpurun_out/r06m
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for P in 2 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06m/trace$P -o run --output-format csv -- python bench.py --steps 3 --no-cpu-baseline --no-secondary --check 0 --pipeline $P > gpurun_out/r06m/trace$P.log 2>&1 || { tail -20 gpurun_out/r06m/trace$P.log; exit 1; }; echo "trace $P done"
done
