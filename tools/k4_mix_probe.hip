// Diagnostic probe (not part of the product): what HBM rate K4's fp32 traffic shape can reach.
// cfg3 fp32: ~27.7k kept row-tasks (K and V) of 16 KB each, read once (16-B non-temporal loads),
// written back as a 16 KB dequantized row + a ~2 KB packed row (average 3.96 bits/element).
// Variants: rows per wave / waves per row, and loads in flight, with a register-only "transform".
//   hipcc -O3 --offload-arch=gfx950 tools/k4_mix_probe.hip -o tools/k4_mix_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

// WPR waves cooperate on one row of ROW_U4 16-byte chunks (each wave: ROW_U4 / WPR / 64 loads per lane).
template <int ROW_U4, int WPR, bool NT = true, bool DQ = true, int PKW = 8>
__global__ __launch_bounds__(256) void mix(const u4* __restrict__ src, const int* __restrict__ idx, u4* __restrict__ dq,
                                           u4* __restrict__ pk, int rows) {
  constexpr int PER = ROW_U4 / WPR / 64;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int r = wave / WPR, part = wave % WPR;
  if (r >= rows) return;
  const u4* s = src + (size_t)idx[r] * ROW_U4 + part * PER * 64;
  u4 v[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) v[k] = __builtin_nontemporal_load(s + k * 64 + lane);
  u4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < PER; ++k) acc ^= v[k];
  u4* d = dq + (size_t)r * ROW_U4 + part * PER * 64;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (!DQ) break;
    if (NT) __builtin_nontemporal_store(v[k] ^ acc, d + k * 64 + lane);
    else d[k * 64 + lane] = v[k] ^ acc;
  }
  // packed: 1/8 of the row bytes (4 bits per fp32 element); PKW-byte stores (0: none)
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  if constexpr (PKW == 8) {
    u2* p = reinterpret_cast<u2*>(pk + (size_t)r * (ROW_U4 / 8)) + part * PER * 64;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (NT) __builtin_nontemporal_store(u2{acc.x + k, acc.y}, p + k * 64 + lane);
      else p[k * 64 + lane] = u2{acc.x + k, acc.y};
    }
  } else if constexpr (PKW == 16) {  // the same bytes as whole 16-B lanes (codes staged per lane)
    u4* p = pk + (size_t)r * (ROW_U4 / 8) + part * (PER / 2) * 64;
#pragma unroll
    for (int k = 0; k < PER / 2; ++k) __builtin_nontemporal_store(acc + (unsigned)k, p + k * 64 + lane);
  } else if constexpr (PKW == 1) {  // sink so the loads stay live, no stores worth counting
    if (acc.x == 0x12345u) pk[0] = acc;
  }
}

__global__ void wr(u4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(u4{(unsigned)i, 1u, 2u, 3u}, dst + i);
}

__global__ void rd(const u4* __restrict__ src, u4* out, size_t n) {
  u4 acc = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= __builtin_nontemporal_load(src + i);
  if (acc.x == 0x12345) out[0] = acc;
}

int main() {
  constexpr int ROW_U4 = 16384 / 16;     // fp32 row of 4096
  const int S = 16384, rows = 2 * 13000;  // kept K and V rows of one layer
  const int NB = 3;                       // rotate buffers so nothing stays in the 256 MB cache
  const size_t srcb = (size_t)2 * S * ROW_U4 * 16, dqb = (size_t)rows * ROW_U4 * 16, pkb = dqb / 8;
  std::vector<u4*> Sx(NB), D(NB), P(NB);
  for (int i = 0; i < NB; ++i) {
    (void)hipMalloc(&Sx[i], srcb); (void)hipMalloc(&D[i], dqb); (void)hipMalloc(&P[i], pkb);
    (void)hipMemset(Sx[i], 1, srcb);
  }
  // kept rows: ~80 % of the tokens of each tensor, ascending (K rows then V rows interleaved per task)
  std::vector<int> h(rows);
  unsigned x = 12345;
  int n = 0;
  for (int t = 0; t < S && n < rows; ++t) {
    x = x * 1664525u + 1013904223u;
    if ((x >> 8) % 100 < 80) { h[n++] = t; if (n < rows) h[n++] = S + t; }
  }
  for (; n < rows; ++n) h[n] = n % (2 * S);
  int* idx;
  (void)hipMalloc(&idx, rows * sizeof(int));
  (void)hipMemcpy(idx, h.data(), rows * sizeof(int), hipMemcpyHostToDevice);
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  auto run = [&](const char* nm, double bytes, auto launch) {
    for (int i = 0; i < NB; ++i) launch(i);
    (void)hipEventRecord(a);
    const int reps = 30;
    for (int k = 0; k < reps; ++k) launch(k % NB);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("%-44s %8.2f us  %7.1f GB/s\n", nm, ms * 1e3 / reps, bytes / (ms / reps * 1e-3) / 1e9);
  };
  const double mixb = (double)rows * ROW_U4 * 16 * (2.0 + 1.0 / 8);
#define V(WPR)                                                                                                   \
  run("rows 16KB, " #WPR " wave(s)/row", mixb, [&](int i) {                                                      \
    hipLaunchKernelGGL((mix<ROW_U4, WPR>), dim3((rows * WPR + 3) / 4), dim3(256), 0, 0, Sx[i], idx, D[i], P[i], \
                       rows);                                                                                    \
  });
  V(1) V(2) V(4) V(8)
#undef V
  run("rows 16KB, 4 waves/row, plain stores", mixb, [&](int i) {
    hipLaunchKernelGGL((mix<ROW_U4, 4, false>), dim3((rows * 4 + 3) / 4), dim3(256), 0, 0, Sx[i], idx, D[i], P[i], rows);
  });
  run("rows 8KB (fp16), 1 wave/row", (double)rows * 512 * 16 * (2.0 + 1.0 / 8), [&](int i) {
    hipLaunchKernelGGL((mix<512, 1>), dim3((rows + 3) / 4), dim3(256), 0, 0, Sx[i], idx, D[i], P[i], rows);
  });
  run("rows 16KB, packed only (read + 1/8 write)", (double)rows * ROW_U4 * 16 * (1.0 + 1.0 / 8), [&](int i) {
    hipLaunchKernelGGL((mix<ROW_U4, 4, true, false>), dim3((rows * 4 + 3) / 4), dim3(256), 0, 0, Sx[i], idx, D[i], P[i], rows);
  });
  run("rows 16KB, packed only, 16-B code stores", (double)rows * ROW_U4 * 16 * (1.0 + 1.0 / 8), [&](int i) {
    hipLaunchKernelGGL((mix<ROW_U4, 4, true, false, 16>), dim3((rows * 4 + 3) / 4), dim3(256), 0, 0, Sx[i], idx, D[i], P[i], rows);
  });
  run("rows 16KB, packed only, plain 8-B code stores", (double)rows * ROW_U4 * 16 * (1.0 + 1.0 / 8), [&](int i) {
    hipLaunchKernelGGL((mix<ROW_U4, 4, false, false, 8>), dim3((rows * 4 + 3) / 4), dim3(256), 0, 0, Sx[i], idx, D[i], P[i], rows);
  });
  run("rows 16KB, packed only, 1 wave/row", (double)rows * ROW_U4 * 16 * (1.0 + 1.0 / 8), [&](int i) {
    hipLaunchKernelGGL((mix<ROW_U4, 1, true, false, 8>), dim3((rows + 3) / 4), dim3(256), 0, 0, Sx[i], idx, D[i], P[i], rows);
  });
  run("rows 16KB gathered, read only, 4 waves/row", (double)rows * ROW_U4 * 16, [&](int i) {
    hipLaunchKernelGGL((mix<ROW_U4, 4, true, false, 1>), dim3((rows * 4 + 3) / 4), dim3(256), 0, 0, Sx[i], idx, D[i], P[i], rows);
  });
  run("rows 16KB gathered, read only, 1 wave/row", (double)rows * ROW_U4 * 16, [&](int i) {
    hipLaunchKernelGGL((mix<ROW_U4, 1, true, false, 1>), dim3((rows + 3) / 4), dim3(256), 0, 0, Sx[i], idx, D[i], P[i], rows);
  });
  run("write only (streaming)", (double)dqb, [&](int i) {
    hipLaunchKernelGGL(wr, dim3(8192), dim3(256), 0, 0, D[i], dqb / 16);
  });
  run("read only (streaming)", (double)dqb, [&](int i) {
    hipLaunchKernelGGL(rd, dim3(8192), dim3(256), 0, 0, Sx[i], P[i], dqb / 16);
  });
  return 0;
}
