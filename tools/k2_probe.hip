// Diagnostic probe (not part of the product): K2 (selection) timing at cfg3 shape (B = 1, S = 16384),
// the one-launch fast path (select_fast.hip; per-phase timestamps of its workgroups and of the
// selecting one, s_memrealtime at 100 MHz) against the four-launch pipeline (select.hip), both timed with HIP events.
//   hipcc -O3 --offload-arch=gfx950 -DRTKV_SELECT_PROBE -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         -I../include -I../realtime-kv-cache-compression_amd/csrc k2_probe.hip -o k2_probe
#include "../realtime-kv-cache-compression_amd/csrc/select_fast.hip"
#include "../realtime-kv-cache-compression_amd/csrc/select.hip"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

namespace rtkv {
void set_error(const std::string& m) { fprintf(stderr, "%s\n", m.c_str()); }
}  // namespace rtkv

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
  const int64_t S = argc > 1 ? atol(argv[1]) : 16384;
  const double ratio = argc > 2 ? atof(argv[2]) : 0.6;
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  std::vector<float> A(S), T2(S);
  const float logS = (float)std::log((double)S), beta = 0.1f;
  const bool skew = argc > 3 && std::string(argv[3]) == "skew";  // attention-like: mass ~ P/(i+1)
  for (int64_t i = 0; i < S; ++i) {
    float m = 0.f;  // bench-like: head mean of 32 row masses ~ U(0, 1)
    for (int h = 0; h < 32; ++h) m += U(rng);
    A[i] = skew ? (float)std::fmin(1.0, 128.0 / (double)(i + 1)) * (0.9f + 0.2f * U(rng)) : (float)(_Float16)(m / 32.f);
    T2[i] = beta * ((float)std::log((double)(i + 1)) / logS);
  }
  float *dA, *dT2, *dsc;
  uint8_t *dlab, *dmask;
  int32_t* dki;
  int64_t* dro;
  void* dst;
  void* ws;
  const size_t wsb = rtkv::select_workspace_bytes(1, S) + 4096;
  CK(hipMalloc(&dA, (S + 64) * 4));
  CK(hipMalloc(&dT2, (S + 64) * 4));
  CK(hipMalloc(&dsc, S * 4));
  CK(hipMalloc(&dlab, S));
  CK(hipMalloc(&dmask, S));
  CK(hipMalloc(&dki, S * 4));
  CK(hipMalloc(&dro, S * 8));
  CK(hipMalloc(&dst, rtkv_stats_bytes(1)));  // header + batch row + rtkv_layer_times (the memset covers it all)
  CK(hipMalloc(&ws, wsb));
  CK(hipMemcpy(dA, A.data(), S * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dT2, T2.data(), S * 4, hipMemcpyHostToDevice));
  rtkv::FinalizeArgs a;
  std::memset(&a, 0, sizeof(a));
  a.p.alpha = 0.8f; a.p.beta = beta; a.p.gamma = 0.1f; a.p.layer_weight = 1.f;
  a.p.theta_h = 0.4f; a.p.theta_m = 0.25f;
  a.p.bits[0] = 2; a.p.bits[1] = 4; a.p.bits[2] = 8;
  a.p.prompt_len = 128; a.p.propagation_ratio = ratio; a.p.flags = RTKV_EMIT_DEQUANT | RTKV_EMIT_PACKED;
  a.B = 1; a.S = S; a.F = 4096; a.kv_dtype = RTKV_F16; a.a_dtype = RTKV_F16;
  a.logS = logS; a.ctx = 128.f / (float)S;
  a.A = dA; a.T2 = dT2;
  if (!(argc > 4 && std::string(argv[4]) == "row")) {  // K1's per-block (min, max) partials, as in the pipeline
    const int nparts = (int)((S + 15) / 16);
    std::vector<float> part(2 * nparts);
    for (int k = 0; k < nparts; ++k) {
      float mn = INFINITY, mx = -INFINITY;
      for (int64_t j = 16 * k; j < S && j < 16 * (k + 1); ++j) { mn = std::fmin(mn, A[j]); mx = std::fmax(mx, A[j]); }
      part[2 * k] = mn; part[2 * k + 1] = mx;
    }
    float* dp;
    CK(hipMalloc(&dp, part.size() * 4));
    CK(hipMemcpy(dp, part.data(), part.size() * 4, hipMemcpyHostToDevice));
    a.A_part = dp; a.A_nparts = nparts;
  }
  a.scores = dsc; a.labels = dlab; a.mask = dmask; a.kept_index = dki; a.row_offset = dro; a.row_capacity = S;
  a.stats = (rtkv_layer_stats*)dst;
  a.mode_scores = a.mode_labels = 1; a.mode_select = 1;
  if (argc > 5 && std::string(argv[5]) == "twice") {
    const int one = 1;
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_k2_twice), &one, sizeof(one)));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int variant = 0; variant < 2; ++variant) {
    rtkv::FinalizeArgs v = a;
    if (variant == 1) v.p.flags |= RTKV_SELECT_PIPELINE;
    const int reps = 50;
    double tot = 0.0;
    double ph[16] = {0}, tl[11] = {0};
    for (int r = 0; r < reps + 5; ++r) {
      CK(hipEventRecord(e0, 0));
      if (rtkv::launch_select(v, ws, false, 0)) { printf("launch failed\n"); return 1; }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 5) {
        tot += ms;
        if (variant == 0) {
          unsigned long long pr[16];
          CK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_k2_probe), sizeof(pr)));
          unsigned long long ck[16];
          CK(hipMemcpyFromSymbol(ck, HIP_SYMBOL(g_k2_clock), sizeof(ck)));
          if (r == reps + 4) printf("  shader clock over the selecting workgroup: %.0f MHz\n", (double)(ck[3] - ck[0]) / ((double)(pr[3] - pr[0]) * 0.01));
          for (int k = 1; k < 16; ++k) { const unsigned long long b0 = k >= 8 ? pr[8] : pr[0]; if (k != 8) ph[k] += (pr[k] > b0 ? (double)(pr[k] - b0) : 0.0) * 0.01; }  // µs
          unsigned long long wg[64][10];
          CK(hipMemcpyFromSymbol(wg, HIP_SYMBOL(g_k2_wg), sizeof(wg)));
          const int G = (int)((S + 1023) / 1024);
          unsigned long long t0 = wg[0][0], mx[10] = {0};
          for (int w = 0; w < G; ++w) t0 = wg[w][0] < t0 ? wg[w][0] : t0;
          for (int w = 0; w < G; ++w)
            for (int k = 0; k < 10; ++k) mx[k] = wg[w][k] > mx[k] ? wg[w][k] : mx[k];
          for (int k = 0; k < 10; ++k) tl[k] += (double)(mx[k] - t0) * 0.01;
          tl[10] += (double)(pr[0] - t0) * 0.01;
        }
      }
    }
    printf("%s: %.2f us/launch (events, incl. the memset of the zeroed scratch)\n", variant ? "pipeline" : "fast", tot / reps * 1e3);
    if (variant == 0) {
      const char* nm[8] = {"start", "counts + partials (+ ready) seen", "threshold bins", "selection published", "histogram loaded", "stats published", "bin scan", "bin pick"};
      for (int k = 1; k < 8; ++k) printf("  t(%s) = %.2f us (from the selecting workgroup's phase-2 start)\n", nm[k], ph[k] / reps);
      for (int k = 9; k < 16; ++k) if (ph[k] != 0.0) printf("  cold pass: t(%s) = %.2f us\n", nm[k - 8], ph[k] / reps);
      const char* tn[11] = {"entry", "A min/max", "scores", "histogram slots", "partials", "selection seen",
                            "aggregates published", "look-back done", "exit", "kept ranks", "selector phase-2 start"};
      for (int k = 0; k < 11; ++k) printf("  last %-22s %.2f us after the first workgroup's entry\n", tn[k], tl[k] / reps);
    }
    rtkv_layer_stats st;
    CK(hipMemcpy(&st, dst, sizeof(st), hipMemcpyDeviceToHost));
    printf("  max_kept %lld packed %lld\n", (long long)st.max_kept, (long long)st.total_packed_bytes);
    {
      std::vector<int32_t> ki(S);
      CK(hipMemcpy(ki.data(), dki, S * 4, hipMemcpyDeviceToHost));
      long long h = 0;
      for (int64_t r = 0; r < st.max_kept; ++r) h = h * 1000003 + ki[r];
      printf("  kept_index hash %lld\n", h);
    }
  }
  return 0;
}
