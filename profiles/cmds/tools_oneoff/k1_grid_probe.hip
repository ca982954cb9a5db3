// Diagnostic probe (not part of the product): K1's read pattern — W prompt slice [H][S][P] streamed
// once, thread (token, 16-byte chunk) summing its chunk over the heads — at cfg3 sizes, for head
// batch HB (loads in flight per thread), grid size (one pass, or a persistent loop over token
// blocks) and element size (fp32 268 MB, fp16 134 MB).  Sums are kept so the loads are live.
//   hipcc -O3 --offload-arch=gfx950 tools/k1_grid_probe.hip -o tools/k1_grid_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int CPR, int HB, bool PF>
__global__ __launch_bounds__(256) void k1(const u4* __restrict__ W, int H, int S, int nblk, float* __restrict__ out) {
  constexpr int TT = 256 / CPR;
  const int tok = threadIdx.x / CPR, ch = threadIdx.x % CPR;
  const size_t sh = (size_t)S * CPR;  // u4 per head
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int i = blk * TT + tok;
    const u4* base = W + (size_t)i * CPR + ch;
    float a = 0.f;
    if constexpr (!PF) {
      for (int h = 0; h < H; h += HB) {
        u4 v[HB];
#pragma unroll
        for (int j = 0; j < HB; ++j) v[j] = __builtin_nontemporal_load(base + (size_t)(h + j) * sh);
#pragma unroll
        for (int j = 0; j < HB; ++j)
          a += __uint_as_float(v[j].x) + __uint_as_float(v[j].y) + __uint_as_float(v[j].z) + __uint_as_float(v[j].w);
      }
    } else {
      u4 v0[HB], v1[HB];
#pragma unroll
      for (int j = 0; j < HB; ++j) v0[j] = __builtin_nontemporal_load(base + (size_t)j * sh);
      for (int h = 0; h < H; h += 2 * HB) {
#pragma unroll
        for (int j = 0; j < HB; ++j) v1[j] = __builtin_nontemporal_load(base + (size_t)(h + HB + j) * sh);
#pragma unroll
        for (int j = 0; j < HB; ++j)
          a += __uint_as_float(v0[j].x) + __uint_as_float(v0[j].y) + __uint_as_float(v0[j].z) + __uint_as_float(v0[j].w);
        if (h + 2 * HB < H) {
#pragma unroll
          for (int j = 0; j < HB; ++j) v0[j] = __builtin_nontemporal_load(base + (size_t)(h + 2 * HB + j) * sh);
        }
#pragma unroll
        for (int j = 0; j < HB; ++j)
          a += __uint_as_float(v1[j].x) + __uint_as_float(v1[j].y) + __uint_as_float(v1[j].z) + __uint_as_float(v1[j].w);
      }
    }
    a += __shfl_xor(a, 1);
    if (ch == 0) out[i] = a;
  }
}

int main() {
  const int H = 32, S = 16384, NB = 3;
  std::vector<u4*> Wb(NB);
  const size_t bytes32 = (size_t)H * S * 128 * 4;
  for (int i = 0; i < NB; ++i) { (void)hipMalloc(&Wb[i], bytes32); (void)hipMemset(Wb[i], 0, bytes32); }
  float* out;
  (void)hipMalloc(&out, S * sizeof(float));
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
    printf("%-48s %8.2f us  %7.1f GB/s\n", nm, ms * 1e3 / reps, bytes / (ms / reps * 1e-3) / 1e9);
  };
  char nm[128];
#define RUN(CPR, HB, PF, GRID)                                                                             \
  {                                                                                                        \
    const int nblk = S / (256 / CPR);                                                                      \
    const int grid = GRID ? GRID : nblk;                                                                   \
    snprintf(nm, sizeof nm, "%s HB=%d PF=%d grid=%d (%d blocks)", CPR == 32 ? "fp32" : "fp16", HB, PF, grid, \
             nblk);                                                                                        \
    run(nm, (double)H * S * CPR * 16, [&](int i) {                                                         \
      hipLaunchKernelGGL((k1<CPR, HB, PF>), dim3(grid), dim3(256), 0, 0, Wb[i], H, S, nblk, out);          \
    });                                                                                                    \
  }
  RUN(32, 16, false, 0) RUN(32, 8, false, 0) RUN(32, 4, false, 0) RUN(32, 8, true, 0) RUN(32, 4, true, 0)
  RUN(32, 16, false, 1024) RUN(32, 8, false, 1024) RUN(32, 8, true, 1024) RUN(32, 8, false, 512)
  RUN(32, 16, false, 1280) RUN(32, 8, true, 2048)
  RUN(16, 16, false, 0) RUN(16, 8, false, 0) RUN(16, 8, true, 0) RUN(16, 4, true, 0) RUN(16, 16, false, 512)
  RUN(16, 8, true, 512) RUN(16, 8, false, 256)
#undef RUN
  return 0;
}
