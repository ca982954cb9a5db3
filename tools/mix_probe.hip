// Diagnostic probe (not part of the product): achievable HBM rate of K4's traffic mix — every row
// read once (16-B non-temporal loads) and written back twice as large (dequantized copy + a
// quarter-size packed copy), rows of 8 KB, 10k rows (cfg3's kept K and V rows).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <bool NT_ST>
__global__ __launch_bounds__(256) void mix(const u4* __restrict__ src, u4* __restrict__ dq, u4* __restrict__ pk,
                                           int rows, int row_u4) {
  // one wave per row, 8 x 1 KiB loads per wave
  const int w = (blockIdx.x * 4 + (threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  if (w >= rows) return;
  const u4* s = src + (size_t)w * row_u4;
  u4 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(s + k * 64 + lane);
  u4* d = dq + (size_t)w * row_u4;
  u4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (NT_ST) __builtin_nontemporal_store(v[k], d + k * 64 + lane);
    else d[k * 64 + lane] = v[k];
    acc ^= v[k];
  }
  // packed: a quarter of the row (2 x 16 B per lane... 1/4 of 8 KB = 2 KB = 2 stores per lane)
  u4* p = pk + (size_t)w * (row_u4 / 4);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (NT_ST) __builtin_nontemporal_store(acc + (unsigned)k, p + k * 64 + lane);
    else p[k * 64 + lane] = acc + (unsigned)k;
  }
}

__global__ void rd(const u4* __restrict__ src, u4* out, size_t n) {
  u4 acc = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= __builtin_nontemporal_load(src + i);
  if (acc.x == 0x12345) out[0] = acc;
}

int main() {
  const int rows = 2 * 9831, row_u4 = 8192 / 16, NB = 4;
  const size_t rb = (size_t)rows * row_u4 * 16;
  std::vector<u4*> S(NB), D(NB), P(NB);
  for (int i = 0; i < NB; ++i) {
    (void)hipMalloc(&S[i], rb); (void)hipMalloc(&D[i], rb); (void)hipMalloc(&P[i], rb / 4);
    (void)hipMemset(S[i], 1, rb);
  }
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  auto run = [&](const char* nm, double bytes, auto launch) {
    for (int i = 0; i < NB; ++i) launch(i);
    (void)hipEventRecord(a);
    const int n = 20;
    for (int k = 0; k < n; ++k) launch(k % NB);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("%-36s %8.2f us  %7.1f GB/s\n", nm, ms * 1e3 / n, bytes / (ms / n * 1e-3) / 1e9);
  };
  const double mixb = rb * 2.25;
  run("mix 1R:1.25W nt stores", mixb, [&](int i) { hipLaunchKernelGGL(mix<true>, dim3((rows + 3) / 4), dim3(256), 0, 0, S[i], D[i], P[i], rows, row_u4); });
  run("mix 1R:1.25W plain stores", mixb, [&](int i) { hipLaunchKernelGGL(mix<false>, dim3((rows + 3) / 4), dim3(256), 0, 0, S[i], D[i], P[i], rows, row_u4); });
  run("read only", (double)rb, [&](int i) { hipLaunchKernelGGL(rd, dim3(4096), dim3(256), 0, 0, S[i], P[i], rb / 16); });
  return 0;
}
