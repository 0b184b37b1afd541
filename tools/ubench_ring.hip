// Microbenchmark: the ceiling of the expansion's row stream on one MI355X.
// Each workgroup of NT threads streams rows of RS bytes (2 x 16 B per thread and
// row, as stream_eval_kernel does: lo half at 16 jt, hi half at 16 jt + L1) with a
// register ring of DEPTH rows in flight per wave, adding them into an int16
// accumulator.  Rows: random over the FT table (mode 0), one row (mode 1, L1-hit),
// or random over the first 2048 rows (mode 2, L2-resident).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_ring.hip -o /tmp/ubench_ring
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

typedef unsigned short ushort8 __attribute__((ext_vector_type(8)));
constexpr int L1 = 3072;
constexpr uint32_t RS = 2 * L1 + 32;
constexpr int ROWS = 22529;

template <int NT, int DEPTH>
__global__ void __launch_bounds__(NT) ring(const uint8_t *ft, const uint32_t *rows, int per_block, uint32_t *out) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)ft, 0, (int)(ROWS * RS), 0x00020000);
  const int tid = threadIdx.x;
  const uint32_t j16 = 16 * (tid % (L1 / 16));
  typedef const __attribute__((address_space(4))) uint32_t cu32;
  cu32 *rw = (cu32 *)(rows + (size_t)blockIdx.x * per_block); // entries by scalar loads, as the stream
  ushort8 lo = {}, hi = {}, rl[DEPTH], rh[DEPTH];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) {
    const uint32_t o = rw[d] * RS;
    rl[d] = __builtin_bit_cast(ushort8, __builtin_amdgcn_raw_buffer_load_b128(r, j16, o, 0));
    rh[d] = __builtin_bit_cast(ushort8, __builtin_amdgcn_raw_buffer_load_b128(r, j16 + L1, o, 0));
  }
  for (int i = DEPTH; i < per_block; i += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      lo += rl[d], hi += rh[d];
      const uint32_t o = rw[i + d] * RS;
      rl[d] = __builtin_bit_cast(ushort8, __builtin_amdgcn_raw_buffer_load_b128(r, j16, o, 0));
      rh[d] = __builtin_bit_cast(ushort8, __builtin_amdgcn_raw_buffer_load_b128(r, j16 + L1, o, 0));
    }
  }
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) lo += rl[d], hi += rh[d];
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) x += lo[k] ^ hi[k];
  if (x == (uint32_t)per_block + 1000000u) out[tid] = x; // keep the work (never true: x < 2^19)
}

template <int NT, int DEPTH>
static void run(const char *name, const uint8_t *ft, const uint32_t *rows, int nblk, int per_block, uint32_t *out,
                size_t lds) {
  hipEvent_t a, b;
  hipEventCreate(&a), hipEventCreate(&b);
  auto k = ring<NT, DEPTH>;
  hipLaunchKernelGGL(k, dim3(nblk), dim3(NT), lds, 0, ft, rows, per_block, out);
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess || hipGetLastError() != hipSuccess) printf("launch error %s\n", hipGetErrorString(e));
  hipEventRecord(a);
  for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k, dim3(nblk), dim3(NT), lds, 0, ft, rows, per_block, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  ms /= 5;
  const double bytes = (double)nblk * per_block * 2.0 * L1 * (NT / (L1 / 16));
  printf("%-28s NT %4d depth %d lds %6zu: %8.3f ms  %7.2f TB/s (row bytes)\n", name, NT, DEPTH, lds, ms,
         bytes / ms / 1e9);
}

int main() {
  uint8_t *ft;
  uint32_t *rows, *out;
  const int nblk = 256 * 3 * 8, per_block = 4096;
  hipMalloc(&ft, (size_t)ROWS * RS);
  hipMemset(ft, 1, (size_t)ROWS * RS);
  hipMalloc(&rows, (size_t)nblk * per_block * 4);
  hipMalloc(&out, 4096 * 4);
  std::vector<uint32_t> h((size_t)nblk * per_block);
  for (int mode = 0; mode < 3; ++mode) {
    srand(1);
    for (auto &v : h) v = mode == 0 ? (uint32_t)(rand() % ROWS) : mode == 1 ? 22528u : (uint32_t)(rand() % 2048);
    hipMemcpy(rows, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    const char *nm = mode == 0 ? "random rows (IC/HBM)" : mode == 1 ? "one row (L1)" : "2048 rows (L2)";
    for (size_t lds : {size_t(0), size_t(54000)}) {
      run<192, 4>(nm, ft, rows, nblk, per_block, out, lds);
      run<192, 8>(nm, ft, rows, nblk, per_block, out, lds);
      run<384, 4>(nm, ft, rows, nblk, per_block, out, lds);
    }
  }
  printf("err %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
