// select_one.h — K2 in ONE workgroup for one batch row of S <= 8192 tokens (kOneMaxS).
//
// The multi-workgroup K2 (select_fast.h) spends most of its time in cross-workgroup hand-offs (class
// counts → quotas, histograms → thresholds, kept counts → ranks: ≈1–2 µs each), and at S = 4096 its 4
// workgroups pay the same chain as 16 do at S = 16384.  Below 8192 tokens one 1024-thread workgroup
// holds every token (TPT = 4 or 8 per thread, consecutive indices) and every exchange is an LDS
// barrier.  Same outputs bit for bit (scores, classes, mask, kept_index, row_label, row_offset,
// counts; the double statistics to rounding):
//   1  scores and classes (token_importance.py:134-176, dynamic_quantization.py:41-45), block counts
//   2  quotas: the greedy in closed form (selective_propagation.py:93-131), fallback (:205-211)
//   3  per partially kept group, the exact threshold key T by an LDS radix select over the group's keys
//      (4 passes of 8 bits, all groups at once), and the tie cutoff: the index of the last kept token
//      at T (ties go in token order), from a block scan of per-thread tie counts
//   4  keep decisions, ranks per class from a block scan (tokens are in index order across threads),
//      mask, kept_index, row_label, row_offset, statistics
// The early host mirror is published after phase 2, as the multi-workgroup K2 does after its phase 2.
#pragma once
#include "select_fast.h"

namespace rtkv {

namespace {

constexpr int kOneMaxTPT = 8;
constexpr int kOneMaxS = kST * kOneMaxTPT;

template <int TPT, bool HAS_T2, int DT>
__global__ __launch_bounds__(kST) void fsel1_kernel(FastArgs g) {
  const FinalizeArgs& a = g.f;
  __shared__ uint32_t s_hist[kGrp][256];
  __shared__ uint32_t s_red[8][kSW];
  __shared__ double s_dred[2][kSW];
  __shared__ uint64_t s_scan[kSW];
  __shared__ int s_q[2 * kGrp];         // [q] mode, [kGrp + q] quota (tokens to keep)
  __shared__ uint32_t s_pref[kGrp], s_need[kGrp], s_cut[kGrp];
  __shared__ double s_mean;
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const int S = (int)a.S;
  const int i0 = t * TPT;
  // ---- phase 1: scores and classes of this thread's TPT consecutive tokens
  float Av[TPT], T2v[TPT];
#pragma unroll
  for (int k = 0; k < TPT; ++k) {
    const bool v = i0 + k < S;
    Av[k] = v ? a.A[i0 + k] : 0.f;
    T2v[k] = (HAS_T2 && v) ? a.T2[i0 + k] : 0.f;
  }
  float mn, mx;
  amin_amax(a, mn, mx);
  const float den = Dt<DT>::rnd(mx - mn), eps = Dt<DT>::rnd(1e-8f);
  float sv[TPT];
  uint32_t key[TPT];
  uint32_t lab = 0;  // 2 bits per token: its class (3 = no token)
  uint32_t c3[3] = {0u, 0u, 0u};
  double ssum = 0.0;
  uint32_t kmn = 0xffffffffu, kmx = 0u;
#pragma unroll
  for (int k = 0; k < TPT; ++k) {
    const int i = i0 + k;
    sv[k] = 0.f;
    key[k] = 0u;
    if (i < S) {
      const float s = token_score<DT, HAS_T2>(a, i, Av[k], T2v[k], mn, den, eps);
      const int l = class_of(s, a.p);
      a.scores[i] = s;
      a.labels[i] = (uint8_t)l;
      sv[k] = s;
      key[k] = score_key(s);
      lab |= (uint32_t)l << (2 * k);
      c3[0] += l == 0 ? 1u : 0u;  // (no dynamic register indexing)
      c3[1] += l == 1 ? 1u : 0u;
      c3[2] += l == 2 ? 1u : 0u;
      ssum += (double)s;
      kmn = min(kmn, key[k]);
      kmx = max(kmx, key[k]);
    } else {
      lab |= 3u << (2 * k);
    }
  }
  {  // block sums: class counts, score sum, key range
    uint32_t r0 = c3[0], r1 = c3[1], r2 = c3[2];
    double ss = ssum;
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
      r0 += __shfl_xor(r0, o, kWave);
      r1 += __shfl_xor(r1, o, kWave);
      r2 += __shfl_xor(r2, o, kWave);
      ss += __shfl_xor(ss, o, kWave);
      kmn = min(kmn, (uint32_t)__shfl_xor((int)kmn, o, kWave));
      kmx = max(kmx, (uint32_t)__shfl_xor((int)kmx, o, kWave));
    }
    if (lane == 0) {
      s_red[0][wid] = r0; s_red[1][wid] = r1; s_red[2][wid] = r2; s_red[3][wid] = kmn; s_red[4][wid] = kmx;
      s_dred[0][wid] = ss;
    }
  }
  __syncthreads();
  // ---- phase 2 (wave 0): quotas, statistics known here, the early host mirror
  if (wid == 0) {
    const int src = lane & (kSW - 1);
    uint32_t r0 = s_red[0][src], r1 = s_red[1][src], r2 = s_red[2][src], m0 = s_red[3][src], m1 = s_red[4][src];
    double ss = s_dred[0][src];
#pragma unroll
    for (int o = kSW / 2; o > 0; o >>= 1) {
      r0 += __shfl_xor(r0, o, kWave);
      r1 += __shfl_xor(r1, o, kWave);
      r2 += __shfl_xor(r2, o, kWave);
      ss += __shfl_xor(ss, o, kWave);
      m0 = min(m0, (uint32_t)__shfl_xor((int)m0, o, kWave));
      m1 = max(m1, (uint32_t)__shfl_xor((int)m1, o, kWave));
    }
    if (lane == 0) {
      const int64_t ccount[3] = {r0, r1, r2};
      // the greedy in closed form, as select_fast.h phase 2 (32-bit integer math; U compared as a double)
      const double u8 = 8.0 * ((double)S * a.p.propagation_ratio);
      const double Ud = u8 >= 9.0e18 ? 9.0e18 : floor(u8);
      int used = 0, kept = 0;
      int md[kGrp];
      int64_t quota[3];
      for (int k = 2; k >= 0; --k) {
        const int N = (int)ccount[k], bb = a.p.bits[k];
        int n;
        if (a.mode_select == 2) n = N;
        else if (!(u8 >= 0.0)) n = 0;
        else if (bb <= 0) n = N;
        else {
          const double x = Ud - (double)used;
          n = x >= (double)bb * (double)N ? N : (int)((uint32_t)x / (uint32_t)bb);
        }
        used += n * (bb > 0 ? bb : 0);
        kept += n;
        s_q[kGrp + k] = n;
        quota[k] = n;
        md[k] = (n == 0) ? M_NONE : (n == N ? M_ALL : M_PART);
        s_q[k] = md[k];
      }
      int64_t kf = (int64_t)((double)S * 0.1);
      if (kf < 1) kf = 1;
      const bool fb = a.mode_select == 1 && !(a.p.flags & RTKV_NO_FALLBACK) && kept == 0;
      s_q[kGrp + 3] = (int)kf;
      s_q[3] = !fb ? M_NONE : (kf >= S ? M_ALL : M_PART);
      s_mean = ss / (double)S;
      rtkv_layer_stats* hs = a.stats;
      rtkv_batch_stats* bs = reinterpret_cast<rtkv_batch_stats*>(hs + 1);
      for (int q = 0; q < 3; ++q) bs->class_count[q] = ccount[q];
      bs->fallback = fb ? 1 : 0;
      hs->score_sum = ss;
      hs->score_min = key_score(m0);
      hs->score_max = key_score(m1);
      int flags = 0;
      if (a.kv_dtype == RTKV_F16)
        for (int q = 0; q < 3; ++q)
          if (ccount[q] > 0 && a.p.bits[q] >= 16) flags |= RTKV_FLAG_F16_QMAX_OVERFLOW;
      hs->error_flags = flags;
      hs->B = 1;
      int64_t n = 0, units = 0, bytes = 0;
      if (!fb) {  // the kept counts are the quotas (the fallback's come after its selection)
        for (int q = 0; q < 3; ++q) {
          bs->kept_class[q] = quota[q];
          n += quota[q];
          units += quota[q] * (int64_t)a.p.bits[q];
          bytes += quota[q] * row_bytes(a, q);
        }
        bs->kept = n;
        bs->cost_units = units;
        bs->packed_bytes = bytes;
        hs->max_kept = n;
        hs->total_packed_bytes = bytes;
      }
      if (g.early) {  // host-mapped mirror for the caller's early return (as select_fast.h)
        rtkv_early_stats* e = g.early;
        auto put64 = [](void* dst, uint64_t v) {
          __hip_atomic_store(reinterpret_cast<uint64_t*>(dst), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        };
        auto put32 = [](void* dst, uint32_t v) {
          __hip_atomic_store(reinterpret_cast<uint32_t*>(dst), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        };
        put32(&e->complete, fb ? 0u : 1u);
        if (!fb) {
          put64(&e->stats.max_kept, (uint64_t)n);
          put64(&e->stats.total_packed_bytes, (uint64_t)bytes);
          put64(&e->stats.score_sum, __builtin_bit_cast(uint64_t, ss));
          put32(&e->stats.score_min, __builtin_bit_cast(uint32_t, hs->score_min));
          put32(&e->stats.score_max, __builtin_bit_cast(uint32_t, hs->score_max));
          put32(&e->stats.error_flags, (uint32_t)flags);
          put32(&e->stats.B, 1u);
          for (int q = 0; q < 3; ++q) {
            put64(&e->batch.class_count[q], (uint64_t)ccount[q]);
            put64(&e->batch.kept_class[q], (uint64_t)quota[q]);
          }
          put64(&e->batch.kept, (uint64_t)n);
          put64(&e->batch.cost_units, (uint64_t)units);
          put64(&e->batch.packed_bytes, (uint64_t)bytes);
          put32(&e->batch.fallback, 0u);
        }
        __hip_atomic_store(&e->seq, g.early_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  __syncthreads();
  const bool fallback = s_q[3] != M_NONE;
  int part = 0;
#pragma unroll
  for (int q = 0; q < kGrp; ++q) part |= (s_q[q] == M_PART) << q;
  // a token's group: its class, or 3 (every token) when the fallback runs; 4 = no token
  auto grp_of = [&](int k) -> int {
    const int l = (int)((lab >> (2 * k)) & 3u);
    return l == 3 ? 4 : (fallback ? 3 : l);
  };
  // ---- phase 3: exact thresholds of the partially kept groups (radix select, 8 bits per pass)
  if (part) {
    if (t < kGrp) { s_pref[t] = 0u; s_need[t] = (uint32_t)s_q[kGrp + t]; }
    uint32_t pmask = 0u;
#pragma unroll 1
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
      s_hist[t >> 8][t & 255] = 0u;
      __syncthreads();
#pragma unroll
      for (int k = 0; k < TPT; ++k) {
        // wave-aggregated: lanes with the same (group, digit) share one LDS atomic by the lowest of them
        // (heavily tied or clustered scores would otherwise serialise on a few addresses)
        const int e = grp_of(k);
        const bool in = e < kGrp && ((part >> e) & 1) && (key[k] & pmask) == s_pref[e < kGrp ? e : 0];
        const uint32_t v = ((uint32_t)(e & 3) << 8) | ((key[k] >> shift) & 255u);
        uint64_t peers = __ballot(in);
        if (peers) {
#pragma unroll
          for (int bit = 0; bit < 10; ++bit) {
            const uint64_t bk = __ballot((v >> bit) & 1u);
            peers &= ((v >> bit) & 1u) ? bk : ~bk;
          }
          if (in && (peers & ((1ull << lane) - 1ull)) == 0ull)
            atomicAdd(&s_hist[v >> 8][v & 255u], (uint32_t)__popcll(peers));
        }
      }
      __syncthreads();
      // wave q: the digit of group q's need-th key from the top.  Lane l owns digits 255-4l .. 252-4l.
      if (wid < kGrp && ((part >> wid) & 1)) {
        const int q = wid;
        const uint32_t need = s_need[q];
        uint32_t c[4], sum = 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) { c[j] = s_hist[q][255 - 4 * lane - j]; sum += c[j]; }
        const uint32_t incl = wave_scan_dpp(sum);
        uint32_t run = incl - sum;  // tokens of the group with a higher digit
        if (run < need && need <= incl) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (run < need && need <= run + c[j]) {
              s_pref[q] |= (uint32_t)(255 - 4 * lane - j) << shift;
              s_need[q] = need - run;
            }
            run += c[j];
          }
        }
      }
      pmask |= 255u << shift;
      __syncthreads();
    }
    // tie cutoff: the s_need[q]-th token at T (in index order) is the last one kept
    uint64_t tie = 0;
#pragma unroll
    for (int k = 0; k < TPT; ++k) {
      const int e = grp_of(k);
      if (e < kGrp && ((part >> e) & 1) && key[k] == s_pref[e]) tie += 1ull << (16 * e);
    }
    uint64_t tot;
    const uint64_t before = block_excl_scan(tie, s_scan, &tot);
#pragma unroll
    for (int q = 0; q < kGrp; ++q) {
      if (!((part >> q) & 1)) continue;
      const uint32_t T = s_pref[q], r = s_need[q];
      uint32_t run = fld(before, q);
      if (run < r && r <= run + fld(tie, q)) {
#pragma unroll
        for (int k = 0; k < TPT; ++k) {
          if (grp_of(k) == q && key[k] == T) {
            ++run;
            if (run == r) s_cut[q] = (uint32_t)(i0 + k);
          }
        }
      }
    }
    __syncthreads();
  }
  // ---- phase 4: keep decisions, ranks per class in index order, outputs
  uint32_t keptbits = 0;
  uint64_t kc = 0;  // kept tokens of this thread per class (16-bit fields)
  double ks = 0.0, m2 = 0.0;
  const double mean = s_mean;
#pragma unroll
  for (int k = 0; k < TPT; ++k) {
    const int e = grp_of(k);
    if (e == 4) continue;
    const int md = s_q[e];
    bool kept = md == M_ALL;
    if (md == M_PART) kept = key[k] > s_pref[e] || (key[k] == s_pref[e] && (uint32_t)(i0 + k) <= s_cut[e]);
    const int l = (int)((lab >> (2 * k)) & 3u);
    if (kept) {
      keptbits |= 1u << k;
      kc += 1ull << (16 * l);
      ks += (double)sv[k];
    }
    const double d = (double)sv[k] - mean;
    m2 += d * d;
  }
  uint64_t ktot;
  const uint64_t kbefore = block_excl_scan(kc, s_scan, &ktot);
  int64_t rb[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) rb[q] = row_bytes(a, q);
  int64_t k0 = fld(kbefore, 0), k1 = fld(kbefore, 1), k2 = fld(kbefore, 2);
#pragma unroll
  for (int k = 0; k < TPT; ++k) {
    const int i = i0 + k;
    if (i >= S) continue;
    const bool kept = (keptbits >> k) & 1u;
    a.mask[i] = kept ? 1 : 0;
    if (kept) {
      const int l = (int)((lab >> (2 * k)) & 3u);
      const int64_t row = k0 + k1 + k2;
      if (row < a.row_capacity) {
        a.kept_index[row] = i;
        if (a.row_label) a.row_label[row] = (uint8_t)l;
        if (a.row_offset) a.row_offset[row] = k0 * rb[0] + k1 * rb[1] + k2 * rb[2];
      }
      k0 += l == 0;
      k1 += l == 1;
      k2 += l == 2;
    }
  }
  // ---- statistics: Σ kept scores, Σ (s - mean)^2; the fallback's kept counts
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) { ks += __shfl_xor(ks, o, kWave); m2 += __shfl_xor(m2, o, kWave); }
  if (lane == 0) { s_dred[0][wid] = ks; s_dred[1][wid] = m2; }
  __syncthreads();
  if (wid == 0) {
    double x = s_dred[0][lane & (kSW - 1)], y = s_dred[1][lane & (kSW - 1)];
#pragma unroll
    for (int o = kSW / 2; o > 0; o >>= 1) { x += __shfl_xor(x, o, kWave); y += __shfl_xor(y, o, kWave); }
    if (lane == 0) {
      rtkv_layer_stats* hs = a.stats;
      rtkv_batch_stats* bs = reinterpret_cast<rtkv_batch_stats*>(hs + 1);
      if (fallback) {
        int64_t n = 0, units = 0, bytes = 0;
        for (int q = 0; q < 3; ++q) {
          const int64_t nq = fld(ktot, q);
          bs->kept_class[q] = nq;
          n += nq;
          units += nq * (int64_t)a.p.bits[q];
          bytes += nq * rb[q];
        }
        bs->kept = n;
        bs->cost_units = units;
        bs->packed_bytes = bytes;
        hs->max_kept = n;
        hs->total_packed_bytes = bytes;
      }
      bs->kept_score_sum = x;
      hs->score_m2 = y;
    }
  }
}

}  // namespace

}  // namespace rtkv
