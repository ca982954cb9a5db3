// Diagnostic probe (not part of the product): achievable HBM read rate of K1's access pattern.
// W prompt slice [H, S, P] fp16 (P = 128): a block owns TT consecutive tokens, each thread a 16-byte
// chunk of one token row, looping over the H head slabs (4 MB apart at S = 16k).
//   variant 0: plain sum of every loaded element (no LDS, no reduction tail)      — pattern ceiling
//   variant 1: same, heads unrolled 8 at a time with all loads issued first
//   variant 2: one block per 64 tokens, thread = (token, chunk), heads split in two halves
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void v0(const uint4* __restrict__ W, int H, long S, int TT, float* out) {
  const int cpr = 16;  // 16-byte chunks per 128-col fp16 row
  const long i0 = (long)blockIdx.x * TT;
  float acc = 0.f;
  for (int e = threadIdx.x; e < TT * cpr; e += blockDim.x) {
    const long i = i0 + e / cpr;
    const int ch = e % cpr;
    for (int h = 0; h < H; ++h) {
      const uint4 v = W[((long)h * S + i) * cpr + ch];
      acc += __uint_as_float(v.x) + __uint_as_float(v.y) + __uint_as_float(v.z) + __uint_as_float(v.w);
    }
  }
  if (acc == 12345.f) out[0] = acc;
}

template <int U>
__global__ __launch_bounds__(256) void v1(const uint4* __restrict__ W, int H, long S, int TT, float* out) {
  const int cpr = 16;
  const long i0 = (long)blockIdx.x * TT;
  float acc = 0.f;
  for (int e = threadIdx.x; e < TT * cpr; e += blockDim.x) {
    const long i = i0 + e / cpr;
    const int ch = e % cpr;
    for (int h = 0; h < H; h += U) {
      uint4 v[U];
#pragma unroll
      for (int j = 0; j < U; ++j) v[j] = W[((long)(h + j) * S + i) * cpr + ch];
#pragma unroll
      for (int j = 0; j < U; ++j)
        acc += __uint_as_float(v[j].x) + __uint_as_float(v[j].y) + __uint_as_float(v[j].z) + __uint_as_float(v[j].w);
    }
  }
  if (acc == 12345.f) out[0] = acc;
}

int main() {
  const int H = 32, P = 128;
  const long S = 16384;
  const size_t bytes = (size_t)H * S * P * 2;
  uint4* W;
  float* out;
  hipMalloc(&W, bytes);
  hipMalloc(&out, 4);
  hipMemset(W, 0, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    hipEventRecord(a);
    const int n = 20;
    for (int k = 0; k < n; ++k) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-40s %8.2f us  %7.1f GB/s\n", name, ms * 1e3 / n, bytes / (ms / n * 1e-3) / 1e9);
  };
  for (int TT : {16, 32, 64}) {
    char nm[64];
    snprintf(nm, 64, "v0 TT=%d", TT);
    run(nm, [&] { hipLaunchKernelGGL(v0, dim3(S / TT), dim3(256), 0, 0, W, H, S, TT, out); });
    snprintf(nm, 64, "v1<8> TT=%d", TT);
    run(nm, [&] { hipLaunchKernelGGL(v1<8>, dim3(S / TT), dim3(256), 0, 0, W, H, S, TT, out); });
    snprintf(nm, 64, "v1<16> TT=%d", TT);
    run(nm, [&] { hipLaunchKernelGGL(v1<16>, dim3(S / TT), dim3(256), 0, 0, W, H, S, TT, out); });
    snprintf(nm, 64, "v1<32> TT=%d", TT);
    run(nm, [&] { hipLaunchKernelGGL(v1<32>, dim3(S / TT), dim3(256), 0, 0, W, H, S, TT, out); });
  }
  // contiguous streaming reference: same bytes, flat
  run("flat stream (v1<8>, H=1, S*32)", [&] { hipLaunchKernelGGL(v1<8>, dim3(S * 32 / 16 / 8), dim3(256), 0, 0, W, 8, S * 32 / 8, 16, out); });
  return 0;
}
