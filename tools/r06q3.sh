# round 6: kernel-trace stats of the drop-in line on the final code (evidence for DESIGN §8 item 4)
set -o pipefail
mkdir -p gpurun_out/r06q3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06q3/dropin -o run --output-format csv -- python bench.py --dropin > gpurun_out/r06q3/dropin.json 2> gpurun_out/r06q3/dropin.err || { tail -20 gpurun_out/r06q3/dropin.err; exit 1; }; echo "trace done"
