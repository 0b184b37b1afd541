# round 6: the front stream's priority A/B, then per-kernel PMC passes of the expand workload
set -o pipefail
mkdir -p gpurun_out/r06l
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 800 python -u tools/ab.py --out gpurun_out/r06l/ab --variants libgpu_nnue_prio.so libgpu_nnue.so libgpu_nnue_prio.so libgpu_nnue.so --timeout 180 -- --steps 5 > gpurun_out/r06l/ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/r06l/ab.log
timeout -k 10 600 bash tools/pmc_kernels.sh r06l/pk expand > gpurun_out/r06l/pk.log 2>&1; echo "pmc rc=$?"; tail -5 gpurun_out/r06l/pk.log
