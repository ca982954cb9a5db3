// finalize.hip — K2: importance scores, precision classes, budgeted selection and the ordered
// compaction map, in ONE workgroup (1024 threads) per layer.
//
// Reference (all per batch row):
//   scores      token_importance.py:134-176   s = α·N·w_l + β·log(i+1)/log(S) + γ·min(1, P/S)
//   min-max     token_importance.py:49-85
//   classes     dynamic_quantization.py:21-60  2 if s ≥ θh, 1 if θm ≤ s < θh, else 0
//   selection   selective_propagation.py:68-161  argsort(desc) + greedy knapsack on costs bits/8
//   fallback    selective_propagation.py:205-211  topk(max(1, int(0.1·S))) if nothing selected
//   compaction  selective_propagation.py:214-232  kept rows in ascending original index
//
// The greedy needs no sort.  Classes are monotone in the score, so the descending order visits all
// HIGH tokens, then MEDIUM, then LOW, and inside a class every cost is equal: once one token of a
// class is rejected, every later token of that class is too.  With costs in units of 1/8 (exact),
// the greedy keeps the top n_g tokens of class g for
//     n_g = min(N_g, floor((U - used)/bits_g)),   U = floor(8·S·ratio),  g = HIGH, MEDIUM, LOW.
// "Top n_g of class g" is a radix select (4 passes of 8 bits over the order-preserving key) plus an
// index-ordered rank among the tokens equal to the threshold key (ties: score desc, index asc).
//
// One layer's selection state is 5 bytes per token, so for S ≤ kLdsMaxS the scores and classes
// live in LDS for the whole kernel (one HBM read of A and β·pos, one write of scores/classes/mask/
// index); larger S (the sharded global selection) streams them through L2.  Histogram updates are
// aggregated per wave with a ballot-built match-any, so a bin shared by many lanes costs one LDS
// atomic per wave instead of one per lane.
#include "common.h"

namespace rtkv {

constexpr int kFT = 1024;           // threads
constexpr int kFW = kFT / kWave;    // waves
constexpr int64_t kLdsMaxS = 24576; // 5 B/token in LDS (120 KiB) + static state

enum { SEL_NONE = 0, SEL_ALL = 1, SEL_PARTIAL = 2 };

struct FinShared {
  uint32_t hist[3][256];
  int64_t wscan[kFW][4];
  int64_t wtot[4];
  float fred[2][kFW];
  double dred[kFW];
  int64_t ired[kFW][3];
  int sel_mode[3];
  uint32_t prefix[3];
  int64_t need[3];
  int64_t count[3];
  int64_t max_kept;
  int64_t off_base;        // packed byte offset where this batch row starts
  float mn, mx;
};

// Block-wide exclusive scan of 4 int64 counters.
__device__ void block_scan4(FinShared& sh, const int64_t v[4], int64_t excl[4], int64_t tot[4]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t inc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) inc[k] = wave_inclusive_scan(v[k]);
  if (lane == 63) {
#pragma unroll
    for (int k = 0; k < 4; ++k) sh.wscan[wid][k] = inc[k];
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int k = threadIdx.x;
    int64_t run = 0;
    for (int w = 0; w < kFW; ++w) {
      const int64_t t = sh.wscan[w][k];
      sh.wscan[w][k] = run;
      run += t;
    }
    sh.wtot[k] = run;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    excl[k] = sh.wscan[wid][k] + inc[k] - v[k];
    tot[k] = sh.wtot[k];
  }
  __syncthreads();
}

__device__ void block_minmax(FinShared& sh, float& mn, float& mx) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  mn = wave_min(mn);
  mx = wave_max(mx);
  if (lane == 0) { sh.fred[0][wid] = mn; sh.fred[1][wid] = mx; }
  __syncthreads();
  if (threadIdx.x < 64) {
    float a = lane < kFW ? sh.fred[0][lane] : INFINITY;
    float c = lane < kFW ? sh.fred[1][lane] : -INFINITY;
    a = wave_min(a);
    c = wave_max(c);
    if (lane == 0) { sh.mn = a; sh.mx = c; }
  }
  __syncthreads();
  mn = sh.mn;
  mx = sh.mx;
}

__device__ double block_sum_d(FinShared& sh, double v) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) sh.dred[wid] = v;
  __syncthreads();
  double r = 0.0;
  for (int w = 0; w < kFW; ++w) r += sh.dred[w];
  __syncthreads();
  return r;
}

__device__ void block_sum3(FinShared& sh, int64_t v[3]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 3; ++k) v[k] = wave_sum(v[k]);
  if (lane == 0)
    for (int k = 0; k < 3; ++k) sh.ired[wid][k] = v[k];
  __syncthreads();
  for (int k = 0; k < 3; ++k) {
    int64_t r = 0;
    for (int w = 0; w < kFW; ++w) r += sh.ired[w][k];
    v[k] = r;
  }
  __syncthreads();
}

// Lanes (among those with `part` set) holding the same 10-bit value: wave64 match-any from ballots.
__device__ __forceinline__ uint64_t match_any10(uint32_t v, bool part) {
  uint64_t m = __ballot(part);
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const uint64_t bk = __ballot((v >> k) & 1u);
    m &= ((v >> k) & 1u) ? bk : ~bk;
  }
  return m;
}

// Radix select: for each group g with sel_mode PARTIAL, find the need[g]-th largest key among the
// tokens of that group (merge = all tokens form group 0).  On return prefix[g] = threshold key and
// need[g] = how many tokens equal to it are taken (in index order).
__device__ void radix_select(FinShared& sh, const float* sc, const uint8_t* lb, int64_t S, bool merge) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t Sr = (S + kFT - 1) / kFT * kFT;  // every lane of a wave runs the same trip count
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int k = threadIdx.x; k < 3 * 256; k += kFT) (&sh.hist[0][0])[k] = 0u;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < Sr; i += kFT) {
      bool part = false;
      uint32_t v = 0;
      if (i < S) {
        const int g = merge ? 0 : lb[i];
        const uint32_t key = score_key(sc[i]);
        part = sh.sel_mode[g] == SEL_PARTIAL && (pass == 0 || ((key ^ sh.prefix[g]) >> (shift + 8)) == 0u);
        v = ((uint32_t)g << 8) | ((key >> shift) & 255u);
      }
      const uint64_t peers = match_any10(v, part);
      if (part && (peers & ((1ull << lane) - 1ull)) == 0ull)  // lowest lane of its peer group
        atomicAdd(&sh.hist[v >> 8][v & 255u], (uint32_t)__popcll(peers));
    }
    __syncthreads();
    if (wid < 3 && sh.sel_mode[wid] == SEL_PARTIAL) {
      const int g = wid;
      uint32_t c[4];
      int64_t lsum = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // lane l owns descending bins 4l..4l+3 (digit 255 - j)
        c[q] = sh.hist[g][255 - (4 * lane + q)];
        lsum += c[q];
      }
      const int64_t incl = wave_inclusive_scan(lsum);
      const int64_t excl = incl - lsum;
      const int64_t need = sh.need[g];
      if (excl < need && incl >= need) {
        int64_t run = excl;
        for (int q = 0; q < 4; ++q) {
          if (run + (int64_t)c[q] >= need) {
            sh.prefix[g] |= (255u - (uint32_t)(4 * lane + q)) << shift;
            sh.need[g] = need - run;
            break;
          }
          run += c[q];
        }
      }
    }
    __syncthreads();
  }
}

// Ordered compaction of batch row b (sc/lb: this row's scores/classes, LDS or global).
__device__ void compact_row(FinShared& sh, const FinalizeArgs& a, int64_t b, bool merge, const float* sc,
                            const uint8_t* lb, int64_t class_counts_b[3], int fallback) {
  const int64_t S = a.S;
  uint8_t* mk = a.mask + b * S;
  const int64_t chunk = (S + kFT - 1) / kFT;
  const int64_t lo = (int64_t)threadIdx.x * chunk;
  const int64_t hi = lo + chunk < S ? lo + chunk : S;
  int64_t rowbytes[3];
  for (int g = 0; g < 3; ++g)
    rowbytes[g] = (a.F * field_width(a.kv_dtype < 0 ? RTKV_F32 : a.kv_dtype, a.p.bits[g]) + 7) / 8;
  const bool any_partial = sh.sel_mode[0] == SEL_PARTIAL || sh.sel_mode[1] == SEL_PARTIAL || sh.sel_mode[2] == SEL_PARTIAL;
  // pass A: ties at the threshold, per group, in index order
  int64_t tie_base[3] = {0, 0, 0};
  if (any_partial) {
    int64_t v[4] = {0, 0, 0, 0}, ex[4], tot[4];
    for (int64_t i = lo; i < hi; ++i) {
      const int g = merge ? 0 : lb[i];
      if (sh.sel_mode[g] == SEL_PARTIAL && score_key(sc[i]) == sh.prefix[g]) v[g]++;
    }
    block_scan4(sh, v, ex, tot);
    for (int g = 0; g < 3; ++g) tie_base[g] = ex[g];
  }
  // pass B: selection decision, counts
  int64_t cnt = 0, bytes = 0, kc[3] = {0, 0, 0}, units = 0;
  double ssum = 0.0;
  for (int64_t i = lo; i < hi; ++i) {
    const int lab = lb[i];
    const int g = merge ? 0 : lab;
    bool sel;
    if (sh.sel_mode[g] == SEL_ALL) sel = true;
    else if (sh.sel_mode[g] == SEL_NONE) sel = false;
    else {
      const uint32_t key = score_key(sc[i]);
      if (key > sh.prefix[g]) sel = true;
      else if (key == sh.prefix[g]) sel = (tie_base[g]++ < sh.need[g]);
      else sel = false;
    }
    mk[i] = sel ? 1 : 0;
    if (sel) {
      cnt++;
      bytes += rowbytes[lab];
      kc[lab]++;
      units += a.p.bits[lab];
      ssum += (double)sc[i];
    }
  }
  int64_t v[4] = {cnt, bytes, 0, 0}, ex[4], tot[4];
  block_scan4(sh, v, ex, tot);
  const int64_t kept = tot[0], row_bytes_total = tot[1];
  // pass C: write the compaction map (this thread's rows are contiguous)
  int64_t row = ex[0], off = sh.off_base + ex[1];
  const int64_t cap = a.row_capacity;
  for (int64_t i = lo; i < hi; ++i) {
    if (!mk[i]) continue;
    if (a.kept_index && row < cap) a.kept_index[b * cap + row] = (int32_t)i;
    if (a.row_offset && row < cap) a.row_offset[b * cap + row] = off;
    row++;
    off += rowbytes[lb[i]];
  }
  for (int64_t r = kept + threadIdx.x; r < cap; r += kFT) {
    if (a.kept_index) a.kept_index[b * cap + r] = -1;
    if (a.row_offset) a.row_offset[b * cap + r] = sh.off_base + row_bytes_total;
  }
  block_sum3(sh, kc);
  int64_t u3[3] = {units, 0, 0};
  block_sum3(sh, u3);
  const double ksum = block_sum_d(sh, ssum);
  if (threadIdx.x == 0) {
    rtkv_batch_stats* bs = reinterpret_cast<rtkv_batch_stats*>(a.stats + 1) + b;
    for (int g = 0; g < 3; ++g) { bs->class_count[g] = class_counts_b[g]; bs->kept_class[g] = kc[g]; }
    bs->kept = kept;
    bs->cost_units = u3[0];
    bs->packed_bytes = row_bytes_total;
    bs->fallback = fallback;
    bs->reserved = 0;
    bs->kept_score_sum = ksum;
    sh.off_base += row_bytes_total;
    if (kept > sh.max_kept) sh.max_kept = kept;
  }
  __syncthreads();
}

// Per-class counts of this wave's labels (ballot + popcount; lane 0 accumulates).
__device__ __forceinline__ void count_label(int l, bool valid, int64_t cc[3]) {
  const uint64_t m0 = __ballot(valid && l == 0), m1 = __ballot(valid && l == 1), m2 = __ballot(valid && l == 2);
  if ((threadIdx.x & 63) == 0) { cc[0] += __popcll(m0); cc[1] += __popcll(m1); cc[2] += __popcll(m2); }
}

template <bool LDS>
__global__ __launch_bounds__(kFT) void finalize_kernel(FinalizeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
  __shared__ FinShared sh;
  const int64_t S = a.S, B = a.B;
  const int64_t Sr = (S + kFT - 1) / kFT * kFT;
  if (threadIdx.x == 0) { sh.max_kept = 0; sh.off_base = 0; }
  double score_sum = 0.0;
  float gmn = INFINITY, gmx = -INFINITY;
  int64_t total_class[3] = {0, 0, 0};
  __syncthreads();
  for (int64_t b = 0; b < B; ++b) {
    float* sc = LDS ? reinterpret_cast<float*>(dyn) : a.scores + b * S;
    uint8_t* lb = LDS ? dyn + 4 * S : a.labels + b * S;
    float* sc_g = a.scores + b * S;
    uint8_t* lb_g = a.labels + b * S;
    // ---- scores (token_importance.py:134-176)
    if (a.mode_scores) {
      const float* A = a.A + b * S;
      float mn = INFINITY, mx = -INFINITY;
      for (int64_t i = threadIdx.x; i < S; i += kFT) {
        const float v = A[i];
        if (LDS) sc[i] = v;
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
      }
      block_minmax(sh, mn, mx);
      const int dt = a.a_dtype;
      const float den = rnd_dt(dt, mx - mn);
      const float eps = rnd_dt(dt, 1e-8f);
      const float t3 = a.p.gamma * a.ctx;
      for (int64_t i = threadIdx.x; i < S; i += kFT) {
        const float Ai = LDS ? sc[i] : A[i];
        const float N = (den > eps) ? rnd_dt(dt, rnd_dt(dt, Ai - mn) / den) : 0.f;
        const float t1 = rnd_dt(dt, rnd_dt(dt, N * a.p.alpha) * a.p.layer_weight);
        const float t2 = a.T2 ? a.T2[i] : a.p.beta * ((S > 1) ? torch_logf((uint32_t)(i + 1)) / a.logS : 0.f);
        float s = t1 + t2;
        s = s + t3;
        sc[i] = s;
        if (LDS) sc_g[i] = s;
      }
    } else if (LDS) {
      for (int64_t i = threadIdx.x; i < S; i += kFT) sc[i] = sc_g[i];
    }
    // ---- precision classes (dynamic_quantization.py:41-45)
    int64_t cc[3] = {0, 0, 0};
    for (int64_t i = threadIdx.x; i < Sr; i += kFT) {
      const bool valid = i < S;
      int l = 0;
      if (valid) {
        const float s = sc[i];
        if (a.mode_labels) {
          if (s >= a.p.theta_h) l = 2;
          else if (s >= a.p.theta_m && s < a.p.theta_h) l = 1;
          lb[i] = (uint8_t)l;
          if (LDS) lb_g[i] = (uint8_t)l;
        } else {
          l = lb_g[i];
          if (LDS) lb[i] = (uint8_t)l;
        }
        score_sum += (double)s;
        gmn = fminf(gmn, s);
        gmx = fmaxf(gmx, s);
      }
      count_label(l, valid, cc);
    }
    block_sum3(sh, cc);
    for (int g = 0; g < 3; ++g) total_class[g] += cc[g];
    if (!a.mode_select) {
      if (threadIdx.x == 0) {
        rtkv_batch_stats* bs = reinterpret_cast<rtkv_batch_stats*>(a.stats + 1) + b;
        for (int g = 0; g < 3; ++g) { bs->class_count[g] = cc[g]; bs->kept_class[g] = cc[g]; }
        bs->kept = S;
        bs->cost_units = 0;
        bs->packed_bytes = 0;
        bs->fallback = 0;
        bs->kept_score_sum = 0.0;
      }
      __syncthreads();
      continue;
    }
    // ---- budget quotas (selective_propagation.py:93-131 in closed form)
    if (threadIdx.x == 0) {
      const double budget = (double)S * a.p.propagation_ratio;
      const double u8 = 8.0 * budget;
      int64_t U = (u8 >= 0.0) ? (u8 >= 9.0e18 ? (int64_t)9000000000000000000LL : (int64_t)floor(u8)) : -1;
      int64_t used = 0;
      for (int g = 2; g >= 0; --g) {
        const int64_t N = cc[g];
        const int64_t bb = a.p.bits[g];
        int64_t n;
        if (a.mode_select == 2) n = N;  // RTKV_NO_SELECTION: keep every token
        else if (U < 0) n = 0;
        else if (bb <= 0) n = N;
        else {
          const int64_t fit = (U - used) / bb;
          n = fit < N ? fit : N;
        }
        used += n * (bb > 0 ? bb : 0);
        sh.count[g] = N;
        sh.sel_mode[g] = (n == 0) ? SEL_NONE : (n == N ? SEL_ALL : SEL_PARTIAL);
        sh.prefix[g] = 0u;
        sh.need[g] = n;
      }
    }
    __syncthreads();
    if (sh.sel_mode[0] == SEL_PARTIAL || sh.sel_mode[1] == SEL_PARTIAL || sh.sel_mode[2] == SEL_PARTIAL)
      radix_select(sh, sc, lb, S, false);
    compact_row(sh, a, b, false, sc, lb, cc, 0);
  }
  // ---- emergency fallback: nothing selected in any batch row (selective_propagation.py:205-211)
  if (a.mode_select && !(a.p.flags & RTKV_NO_FALLBACK) && sh.max_kept == 0 && S > 0) {
    if (threadIdx.x == 0) sh.off_base = 0;
    __syncthreads();
    int64_t k = (int64_t)((double)S * 0.1);
    if (k < 1) k = 1;
    for (int64_t b = 0; b < B; ++b) {
      float* sc = LDS ? reinterpret_cast<float*>(dyn) : a.scores + b * S;
      uint8_t* lb = LDS ? dyn + 4 * S : a.labels + b * S;
      if (LDS && B > 1) {  // reload this row (the LDS copy holds the last row)
        for (int64_t i = threadIdx.x; i < S; i += kFT) { sc[i] = a.scores[b * S + i]; lb[i] = a.labels[b * S + i]; }
        __syncthreads();
      }
      if (threadIdx.x == 0) {
        sh.sel_mode[0] = (k >= S) ? SEL_ALL : SEL_PARTIAL;
        sh.sel_mode[1] = sh.sel_mode[2] = SEL_NONE;
        sh.prefix[0] = 0u;
        sh.need[0] = k;
      }
      __syncthreads();
      if (sh.sel_mode[0] == SEL_PARTIAL) radix_select(sh, sc, lb, S, true);
      rtkv_batch_stats* bs = reinterpret_cast<rtkv_batch_stats*>(a.stats + 1) + b;
      int64_t ccb[3] = {bs->class_count[0], bs->class_count[1], bs->class_count[2]};
      __syncthreads();
      compact_row(sh, a, b, true, sc, lb, ccb, 1);
    }
  }
  // ---- layer statistics (unified_compressor.py:144-163)
  {
    const double tot = block_sum_d(sh, score_sum);
    float mn = gmn, mx = gmx;
    block_minmax(sh, mn, mx);
    const double n = (double)(B * S);
    const double mean = n > 0 ? tot / n : 0.0;
    double m2 = 0.0;
    for (int64_t b = 0; b < B; ++b) {
      const float* scs = a.scores + b * S;
      for (int64_t i = threadIdx.x; i < S; i += kFT) {
        const double d = (double)scs[i] - mean;
        m2 += d * d;
      }
    }
    m2 = block_sum_d(sh, m2);
    if (threadIdx.x == 0) {
      rtkv_layer_stats* st = a.stats;
      st->max_kept = a.mode_select ? sh.max_kept : S;
      st->total_packed_bytes = sh.off_base;
      st->score_sum = tot;
      st->score_m2 = m2;
      st->score_min = mn;
      st->score_max = mx;
      int flags = 0;
      if (a.kv_dtype == RTKV_F16)
        for (int g = 0; g < 3; ++g)
          if (total_class[g] > 0 && a.p.bits[g] >= 16) flags |= RTKV_FLAG_F16_QMAX_OVERFLOW;
      st->error_flags = flags;
      st->B = (int32_t)B;
    }
  }
}

int launch_finalize(const FinalizeArgs& a, hipStream_t st) {
  RTKV_REQUIRE(a.scores && a.labels && a.stats, "finalize: null scores/labels/stats");
  RTKV_REQUIRE(a.B >= 1 && a.S >= 1, "finalize: empty shape");
  RTKV_REQUIRE(!a.mode_scores || a.A, "finalize: null aggregation input");
  RTKV_REQUIRE(a.S < ((int64_t)1 << 31), "finalize: S must be < 2^31");
  RTKV_REQUIRE(!a.mode_select || a.mask, "finalize: selection needs a mask buffer");
  if (a.S <= kLdsMaxS) {
    static bool attr_set = false;
    if (!attr_set) {
      RTKV_HIP_CHECK(hipFuncSetAttribute((const void*)finalize_kernel<true>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsMaxS * 5)));
      attr_set = true;
    }
    hipLaunchKernelGGL(finalize_kernel<true>, dim3(1), dim3(kFT), (size_t)a.S * 5, st, a);
  } else {
    hipLaunchKernelGGL(finalize_kernel<false>, dim3(1), dim3(kFT), 0, st, a);
  }
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

}  // namespace rtkv
