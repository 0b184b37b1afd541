#!/bin/bash
# Round-end check on the GPU box: an A/B line, the GPU suite and smoke()
python tools/ab.py --variants libgpu_nnue.so libgpu_nnue_kcnt.so libgpu_nnue_entnt.so -- --steps 5 --check 32 || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_final.log 2>&1; tail -2 gpurun_out/pytest_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
