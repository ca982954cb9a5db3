// Diagnostic probe (not part of the product): K1 register-path variants (heads per load batch,
// prefetch of the next batch) at cfg3 shape, W slices rotated over more than the 256 MB Infinity
// Cache so every launch reads from HBM; with and without the β·pos side output.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         -I../include -I../realtime-kv-cache-compression_amd/csrc k1_variants.hip -o k1_variants_probe
#include "../realtime-kv-cache-compression_amd/csrc/importance.hip"

#include <cstdio>
#include <vector>

namespace rtkv {
void set_error(const std::string& m) { fprintf(stderr, "%s\n", m.c_str()); }
}  // namespace rtkv

int main() {
  const int H = 32, P = 128, NB = 6;
  const long S = 16384;
  const size_t bytes = (size_t)H * S * P * 2;
  std::vector<uint16_t*> W(NB);
  for (auto& w : W) { (void)hipMalloc(&w, bytes); (void)hipMemset(w, 0x3c, bytes); }
  float *A, *part, *t2;
  (void)hipMalloc(&A, S * 4);
  (void)hipMalloc(&t2, S * 4);
  (void)hipMalloc(&part, S * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < NB; ++w) launch(w);
    (void)hipEventRecord(a);
    const int n = 30;
    for (int k = 0; k < n; ++k) launch(k % NB);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("%-40s %8.2f us  %7.1f GB/s\n", name, ms * 1e3 / n, bytes / (ms / n * 1e-3) / 1e9);
  };
  const int64_t lim = rtkv::cascade_limit(RTKV_F16, S * (int64_t)P);
  dim3 grid((unsigned)(S / 16), 1);
  for (int extras = 0; extras < 2; ++extras) {
    rtkv::AggExtras x;
    int np = 0;
    if (extras) { x.t2 = t2; x.beta = 0.1f; x.logS = 9.7f; x.part = part; x.nparts = &np; }
    const char* sfx = extras ? " +t2+part" : "";
    char nm[64];
#define VAR(HB, PF)                                                                                          \
    snprintf(nm, sizeof nm, "HB=%d PF=%d%s", HB, (int)PF, sfx);                                             \
    run(nm, [&](int k) {                                                                                    \
      hipLaunchKernelGGL((rtkv::aggregation_shfl_kernel<RTKV_F16, 16, HB, PF>), grid, dim3(256), 0, 0,      \
                         (const uint16_t*)W[k], H, S, (int64_t)H * S * P, S * P, (int64_t)P, lim, A, x);    \
    });
    VAR(16, false) VAR(32, false) VAR(8, true) VAR(4, true) VAR(16, true)
  }
  return 0;
}
