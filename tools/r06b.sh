mkdir -p gpurun_out/r06b
timeout -k 10 900 python -u tools/ab.py --variants libgpu_nnue_base.so libgpu_nnue.so libgpu_nnue_salu6.so libgpu_nnue_salu12.so libgpu_nnue_valu8.so libgpu_nnue.so libgpu_nnue_base.so --timeout 240 -- --steps 5 > gpurun_out/r06b/ab.log 2>&1; echo ab rc=$?
cat gpurun_out/r06b/ab.log
