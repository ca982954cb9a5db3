// Diagnostic probe (not part of the product): K1 (launch_aggregation) against the raw read rate of
// its access pattern, with the W slices rotated over more than the 256 MB Infinity Cache so every
// launch reads from HBM.   hipcc -O3 --offload-arch=gfx950 -I../include -I../realtime-kv-cache-compression_amd/csrc
#include "../realtime-kv-cache-compression_amd/csrc/importance.hip"

#include <cstdio>
#include <vector>

namespace rtkv {
void set_error(const std::string& m) { fprintf(stderr, "%s\n", m.c_str()); }
}  // namespace rtkv

__global__ __launch_bounds__(256) void raw_pattern(const uint4* __restrict__ W, int H, long S, int TT, float* out) {
  const int cpr = 16;
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

int main() {
  const int H = 32, P = 128, NB = 6;
  const long S = 16384;
  const size_t bytes = (size_t)H * S * P * 2;
  std::vector<uint16_t*> W(NB);
  for (auto& w : W) { (void)hipMalloc(&w, bytes); (void)hipMemset(w, 0x3c, bytes); }
  float *A, *out;
  (void)hipMalloc(&A, S * 4 * 2);
  (void)hipMalloc(&out, 64);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < NB; ++w) launch(w);
    (void)hipEventRecord(a);
    const int n = 24;
    for (int k = 0; k < n; ++k) launch(k % NB);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("%-44s %8.2f us  %7.1f GB/s\n", name, ms * 1e3 / n, bytes / (ms / n * 1e-3) / 1e9);
  };
  run("raw pattern TT=16", [&](int k) {
    hipLaunchKernelGGL(raw_pattern, dim3(S / 16), dim3(256), 0, 0, (const uint4*)W[k], H, S, 16, out);
  });
  run("raw pattern TT=32", [&](int k) {
    hipLaunchKernelGGL(raw_pattern, dim3(S / 32), dim3(256), 0, 0, (const uint4*)W[k], H, S, 32, out);
  });
  rtkv_attn_desc d{};
  d.dtype = RTKV_F16;
  d.B = 1; d.H = H; d.S = S; d.cols = P;
  d.stride_b = (int64_t)H * S * P; d.stride_h = S * P; d.stride_s = P;
  run("K1 launch_aggregation (no extras)", [&](int k) {
    d.w_dev = W[k];
    rtkv::launch_aggregation(d, P, A, 0);
  });
  rtkv::AggExtras x;
  x.t2 = A + S;
  x.beta = 0.1f;
  x.logS = 9.7f;
  int np = 0;
  x.part = out;  // only the first blocks' partials fit: probe timing only
  x.nparts = &np;
  run("K1 launch_aggregation (t2)", [&](int k) {
    d.w_dev = W[k];
    rtkv::AggExtras y = x;
    y.part = nullptr;
    rtkv::launch_aggregation(d, P, A, 0, y);
  });
  return 0;
}
