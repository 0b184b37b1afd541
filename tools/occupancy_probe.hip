// occupancy_probe.hip — diagnostic: how many workgroups of a given shape are
// co-resident on one CU of this MI355X.  Each workgroup records (XCC, SE, CU)
// and s_memtime at start and end of a fixed spin; the host reports the maximum
// and average number of overlapping workgroups per CU.
// Build: hipcc --offload-arch=gfx950 -O3 tools/occupancy_probe.hip -o tools/occupancy_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <vector>

struct Rec {
  unsigned long long t0, t1;
  unsigned hwid, xcc;
};

template <int LDS, int VG>
__global__ void __launch_bounds__(512) probe(Rec *out, int spin) {
  __shared__ volatile char lds[LDS];
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID, 32 bits
  unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)); // HW_REG_XCC_ID
  if (VG > 0) { // hold VG VGPRs live across the spin
    float v[VG > 0 ? VG : 1];
#pragma unroll
    for (int i = 0; i < VG; ++i) v[i] = (float)(threadIdx.x + i);
    for (int k = 0; k < spin; ++k) {
#pragma unroll
      for (int i = 0; i < VG; ++i) v[i] = v[i] * 1.0001f + 0.5f;
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < VG; ++i) s += v[i];
    if (s == 12345.f) lds[threadIdx.x] = 1;
  } else {
    for (int k = 0; k < spin; ++k) __builtin_amdgcn_s_sleep(10);
  }
  lds[threadIdx.x % LDS] = 0;
  __syncthreads();
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = {t0, t1, hw, xcc};
}

template <int LDS, int VG>
static void run(const char *name, int blocks, int threads, int spin) {
  Rec *d;
  (void)hipMalloc(&d, blocks * sizeof(Rec));
  hipLaunchKernelGGL((probe<LDS, VG>), dim3(blocks), dim3(threads), 0, 0, d, spin); // warm
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL((probe<LDS, VG>), dim3(blocks), dim3(threads), 0, 0, d, spin);
  (void)hipDeviceSynchronize();
  std::vector<Rec> h(blocks);
  (void)hipMemcpy(h.data(), d, blocks * sizeof(Rec), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  // per CU key = xcc, se, sh, cu
  std::map<unsigned, std::vector<std::pair<unsigned long long, int>>> ev;
  unsigned long long lo = ~0ull, hi = 0;
  for (auto &r : h) {
    unsigned cu = (r.hwid >> 8) & 15, sh = (r.hwid >> 12) & 1, se = (r.hwid >> 13) & 7;
    unsigned key = (r.xcc & 15) << 16 | se << 8 | sh << 4 | cu;
    ev[key].push_back({r.t0, +1});
    ev[key].push_back({r.t1, -1});
    lo = std::min(lo, r.t0), hi = std::max(hi, r.t1);
  }
  int maxc = 0;
  double area = 0, dur_sum = 0;
  for (auto &r : h) dur_sum += (double)(r.t1 - r.t0);
  for (auto &kv : ev) {
    auto &v = kv.second;
    std::sort(v.begin(), v.end(), [](auto &a, auto &b) { return a.first < b.first || (a.first == b.first && a.second < b.second); });
    int c = 0;
    for (auto &e : v) c += e.second, maxc = std::max(maxc, c);
  }
  area = dur_sum / (double)(hi - lo);
  printf("%-34s blocks %6d threads %4d  CUs seen %4zu  max WGs/CU %d  avg resident WGs/CU %.2f  span %.1f kcyc  mean WG %.1f kcyc\n",
         name, blocks, threads, ev.size(), maxc, area / ev.size(), (hi - lo) / 1000.0, dur_sum / blocks / 1000.0);
}

int main(int argc, char **argv) {
  int spin = argc > 1 ? atoi(argv[1]) : 200;
  run<52656, 0>("lds52656 sleep", 4096, 384, spin);
  run<26000, 0>("lds26000 sleep", 4096, 384, spin);
  run<1024, 0>("lds1024 sleep", 4096, 384, spin);
#define V(vg)                                                              \
  run<1024, vg>("vg" #vg " 256thr", 4096, 256, spin / 20 + 1);            \
  run<1024, vg>("vg" #vg " 384thr", 4096, 384, spin / 20 + 1);            \
  run<1024, vg>("vg" #vg " 512thr", 4096, 512, spin / 20 + 1);
  V(40) V(56) V(72) V(88) V(100) V(116) V(124) V(150)
  return 0;
}
