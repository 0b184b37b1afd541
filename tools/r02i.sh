#!/bin/bash
OUT=gpurun_out/r02i; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for a in 0 2 4; do export GN_EXPAND_CHUNKS=1
GN_ABLATE=$a GPU_NNUE_LIB=$PWD/fishnet_amd/lib/libgpu_nnue_prof.so timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --check 0 > $OUT/b$a.json 2> $OUT/b$a.err || { tail -5 $OUT/b$a.err; exit 1; }
echo "ablate $a"; grep "stream prof" $OUT/b$a.err | tail -1
done
