set -o pipefail
OUT=gpurun_out/r04g
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python tools/ab.py --variants libgpu_nnue.so libgpu_nnue_early.so libgpu_nnue.so libgpu_nnue_early.so -- --steps 6 --check 0 || exit 1
