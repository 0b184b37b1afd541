// xcc_probe.hip — which XCD runs which workgroup: hwreg XCC_ID per block vs blockIdx % 8.
// Build + run on the GPU box: hipcc --offload-arch=gfx950 -O2 tools/xcc_probe.hip -o /tmp/xcc_probe && /tmp/xcc_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
__global__ void probe(unsigned *o) {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (threadIdx.x == 0) o[blockIdx.x] = x;
}
int main() {
  const int n = 8192;
  unsigned *d;
  if (hipMalloc(&d, n * 4) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(n), dim3(384), 0, 0, d);
  std::vector<unsigned> h(n);
  if (hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int hist[16] = {0}, agree = 0, maxv = 0;
  for (int i = 0; i < n; ++i) {
    hist[h[i] & 15]++;
    agree += (int)(h[i] & 7) == (i & 7);
    if ((int)h[i] > maxv) maxv = (int)h[i];
  }
  printf("xcc_id max %d; histogram:", maxv);
  for (int k = 0; k < 16; ++k) printf(" %d", hist[k]);
  printf("\nblocks with xcc_id == blockIdx %% 8: %d of %d\n", agree, n);
  return 0;
}
