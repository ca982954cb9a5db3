// select.hip — K2 as a multi-workgroup pipeline: importance scores, precision classes, budgeted
// selection and the ordered compaction map.  Scales to the 100k+ token global selection of the
// sequence-sharded path, where one workgroup would be the bottleneck.
//
// Reference (per batch row):
//   scores      token_importance.py:134-176   s = α·N·w_l + β·log(i+1)/log(S) + γ·min(1, P/S)
//   min-max     token_importance.py:49-85     (global min/max of A: K1 per-block partials)
//   classes     dynamic_quantization.py:21-60  2 if s ≥ θh, 1 if θm ≤ s < θh, else 0
//   selection   selective_propagation.py:68-161  argsort(desc) + greedy knapsack on costs bits/8
//   fallback    selective_propagation.py:205-211  topk(max(1, int(0.1·S))) if nothing selected
//   compaction  selective_propagation.py:214-232  kept rows in ascending original index
//
// Greedy in closed form (no sort): classes are monotone in the score, so the descending order visits
// all HIGH, then MEDIUM, then LOW tokens; inside a class every cost is equal, so the greedy keeps the
// top n_g of class g, n_g = min(N_g, floor((U - used)/bits_g)), U = floor(8·S·ratio).  The top-n_g
// threshold key is found by a 2-round radix select over the order-preserving 32-bit key (16-bit
// digits, each with a 256-bin coarse histogram for a fast scan); ties at the threshold are taken in
// ascending index order.  Group 3 ("all tokens", k = max(1, int(0.1·S))) is selected alongside so
// the rare emergency fallback costs no extra round.
//
// Kernels (grid = (NB blocks of kBT tokens, B)):
//   K2a  scores, classes, class counts, score sum/min/max, round-1 histograms; last block per row:
//        quotas + round-1 digit
//   K2b  round-2 histograms of the tokens in the threshold bin; last block: threshold + tie quota
//   C1   per-block counts (rows/bytes above the threshold, ties per group), Σ(s-mean)²; last block
//        (all rows): fallback decision and the per-row / per-layer statistics
//   C2   ordered compaction: each block derives its row/byte/tie bases from the C1 partials of the
//        blocks before it, then ranks its tokens with wave ballots: mask, kept_index, row_offset
// Cross-workgroup hand-offs follow MI355X_MICROARCH.md "Valid forms": sc1 (agent-scope relaxed
// atomic) stores of every handed-off word, every storing wave drains with s_waitcnt vmcnt(0), one
// lane signals with an agent-scope atomic add, the last arriver reads with sc1 atomic loads.
#include "common.h"

namespace rtkv {

constexpr int kBT = 512;          // tokens per block
constexpr int kNT = 256;          // threads per block
constexpr int kG = 4;             // groups: 3 classes + all tokens (fallback)
constexpr int kFine = 65536;      // 16-bit digit
constexpr int kCoarse = 256;      // top 8 bits of the digit

enum { SEL_NONE = 0, SEL_ALL = 1, SEL_PARTIAL = 2 };

struct SelState {                 // per batch row (zeroed by K1 / the stage launcher)
  uint32_t done_a, done_b, pad0, pad1;
  int32_t sel_mode[kG];
  uint32_t prefix[kG];            // round-1 digit << 16, then the full threshold key
  int64_t need[kG];               // tokens still to take at/below the current prefix
  int64_t quota[kG];
  int64_t class_count[3];         // atomics (K2a)
  uint32_t smin_key, smax_key;    // ~min key, max key of the scores (atomic max)
  uint32_t cls_key[3][2];         // per class: ~min key, max key (atomic max): monotone classes?
  double ssum;                    // score sum (atomics)
};

struct SelGlobal {                // one per call
  uint32_t done_c1;
  int32_t fallback;
  int64_t max_kept;
  int32_t general;                // classes interleave in score order: exact sort + greedy path
};

struct SelPartial {               // per (batch row, block), written by C1 with sc1 stores
  int64_t gt_rows[2];             // [class mode, fallback mode]
  int64_t gt_bytes[2];
  int64_t ties[kG];
  int64_t ties_bytes3;            // fallback-mode tie bytes are resolved serially (rare path)
};

struct SelLayout {                // workspace carve for the selection pipeline
  SelGlobal* glob;
  SelState* state;                // [B]
  uint32_t* hist;                 // [B][2 rounds][kG][kCoarse + kFine]
  SelPartial* part;               // [B][NB]
  int nb;
};

__host__ __device__ inline size_t sel_hist_words(int64_t B) { return (size_t)B * 2 * kG * (kCoarse + kFine); }
__host__ __device__ inline int sel_nb(int64_t S) { return (int)((S + kBT - 1) / kBT); }

// ------------------------------------------------------------------------------------ helpers
__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << (threadIdx.x & 63)) - 1ull; }


// Every wave drains its stores, the block meets, one lane counts in; true in every thread of the
// last block to arrive (which then acquires).
__device__ bool arrive_last(uint32_t* counter, uint32_t expected, int* sh_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *sh_flag = (old + 1 == expected);
    if (*sh_flag) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  return *sh_flag != 0;
}

// Lanes with the same value (up to 20 bits) among those with `part`: wave64 match-any from ballots.
template <int NBITS> __device__ __forceinline__ uint64_t match_any(uint32_t v, bool part) {
  uint64_t m = __ballot(part);
#pragma unroll
  for (int k = 0; k < NBITS; ++k) {
    const uint64_t bk = __ballot((v >> k) & 1u);
    m &= ((v >> k) & 1u) ? bk : ~bk;
  }
  return m;
}

// Aggregated histogram increment of one (group, 16-bit digit) per lane: the 256-bin coarse histogram
// goes to the block's LDS copy (flushed once per block: its few hot bins would otherwise serialise
// thousands of global atomics on one address), the fine bin to global memory, one atomic per
// distinct (group, digit) per wave.
__device__ __forceinline__ void hist_add(uint32_t* base, uint32_t (*lcoarse)[kCoarse], int g, uint32_t bin16, bool part) {
  const uint32_t v = ((uint32_t)g << 16) | bin16;
  const uint64_t peers = match_any<18>(v, part);
  if (part && (peers & lanemask_lt()) == 0ull)
    atomicAdd(base + (size_t)g * (kCoarse + kFine) + kCoarse + bin16, (uint32_t)__popcll(peers));
  const uint32_t vc = ((uint32_t)g << 8) | (bin16 >> 8);
  const uint64_t cpeers = match_any<10>(vc, part);
  if (part && (cpeers & lanemask_lt()) == 0ull) atomicAdd(&lcoarse[g][bin16 >> 8], (uint32_t)__popcll(cpeers));
}

__device__ __forceinline__ void coarse_clear(uint32_t (*lcoarse)[kCoarse]) {
  for (int k = threadIdx.x; k < kG * kCoarse; k += blockDim.x) (&lcoarse[0][0])[k] = 0u;
  __syncthreads();
}
__device__ __forceinline__ void coarse_flush(uint32_t* base, uint32_t (*lcoarse)[kCoarse]) {
  __syncthreads();
  for (int k = threadIdx.x; k < kG * kCoarse; k += blockDim.x) {
    const uint32_t c = (&lcoarse[0][0])[k];
    if (c) atomicAdd(base + (size_t)(k / kCoarse) * (kCoarse + kFine) + (k % kCoarse), c);
  }
}

// In the last block: for every group g with want[g] (one wave per group, all four concurrently),
// find in its (coarse, fine) histogram the 16-bit digit where the count from the top reaches
// need[g]; digit[g] / above[g] = that digit and the count strictly above it.  Two dependent L2
// reads per group.  Defaults keep every index in range even if a histogram holds fewer tokens.
__device__ void find_digits(const uint32_t* h_rows, const bool want[kG], const int64_t need[kG], uint32_t digit[kG],
                            int64_t above[kG]) {
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;  // kNT = 256: wave g ↔ group g
  if (lane == 0) { digit[g] = 0; above[g] = 0; }
  __syncthreads();
  if (want[g]) {
    const uint32_t* h = h_rows + (size_t)g * (kCoarse + kFine);
    const int64_t nd = need[g];
    // coarse: lane l owns descending bins 4l..4l+3 (bin index 255 - j)
    uint32_t c[4];
    int64_t lsum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) { c[q] = ld_sc1(h + (kCoarse - 1 - (4 * lane + q))); lsum += c[q]; }
    int64_t incl = wave_inclusive_scan(lsum), excl = incl - lsum;
    const bool hit = excl < nd && incl >= nd;  // exactly one lane when the histogram holds nd tokens
    uint32_t my_coarse = 0;
    int64_t my_ac = 0;
    if (hit) {
      int64_t run = excl;
      for (int q = 0; q < 4; ++q) {
        if (run + (int64_t)c[q] >= nd) { my_coarse = (uint32_t)(kCoarse - 1 - (4 * lane + q)); my_ac = run; break; }
        run += c[q];
      }
    }
    const uint64_t hm = __ballot(hit);
    const int src = hm ? (__ffsll((unsigned long long)hm) - 1) : 0;  // wave-uniform
    const uint32_t coarse = (uint32_t)__shfl((int)my_coarse, src, 64) & (kCoarse - 1);
    const int64_t ac = __shfl(my_ac, src, 64);
    // fine bins of that coarse bin: lane l owns digits (coarse << 8) | (255 - 4l - q)
    uint32_t f[4];
    lsum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) { f[q] = ld_sc1(h + kCoarse + ((coarse << 8) | (uint32_t)(255 - (4 * lane + q)))); lsum += f[q]; }
    incl = ac + wave_inclusive_scan(lsum);
    excl = incl - lsum;
    if (excl < nd && incl >= nd) {
      int64_t run = excl;
      for (int q = 0; q < 4; ++q) {
        if (run + (int64_t)f[q] >= nd) { digit[g] = (coarse << 8) | (uint32_t)(255 - (4 * lane + q)); above[g] = run; break; }
        run += f[q];
      }
    }
  }
  __syncthreads();
}

struct SelArgs {
  FinalizeArgs f;
  SelLayout L;
};

__device__ __forceinline__ int64_t rowbytes_of(const FinalizeArgs& a, int lab) {
  return (a.F * field_width(a.kv_dtype < 0 ? RTKV_F32 : a.kv_dtype, a.p.bits[lab]) + 7) / 8;
}

// ------------------------------------------------------------------------------------ K2a
__global__ __launch_bounds__(kNT) void sel_scores_kernel(SelArgs g) {
  const FinalizeArgs& a = g.f;
  __shared__ float s_mm[2][4];
  __shared__ unsigned long long s_cnt[3];
  __shared__ double s_sum;
  __shared__ uint32_t s_key[2];
  __shared__ uint32_t s_ckey[3][2];
  __shared__ int s_flag;
  const int b = blockIdx.y, blk = blockIdx.x;
  const int64_t S = a.S;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  SelState* st = g.L.state + b;
  float* sc = a.scores + (int64_t)b * S;
  uint8_t* lb = a.labels + (int64_t)b * S;
  if (threadIdx.x < 3) s_cnt[threadIdx.x] = 0;
  if (threadIdx.x == 0) { s_sum = 0.0; s_key[0] = 0xffffffffu; s_key[1] = 0u; }
  if (threadIdx.x < 3) { s_ckey[threadIdx.x][0] = 0xffffffffu; s_ckey[threadIdx.x][1] = 0u; }
  // ---- global min/max of A (K1 per-block partials, or the whole row)
  float mn = INFINITY, mx = -INFINITY, den = 0.f, eps = 0.f;
  if (a.mode_scores) {
    if (a.A_part) {
      const float* pp = a.A_part + (int64_t)b * 2 * a.A_nparts;
      for (int k = threadIdx.x; k < a.A_nparts; k += kNT) { mn = fminf(mn, pp[2 * k]); mx = fmaxf(mx, pp[2 * k + 1]); }
    } else {
      const float* A = a.A + (int64_t)b * S;
      for (int64_t i = threadIdx.x; i < S; i += kNT) { mn = fminf(mn, A[i]); mx = fmaxf(mx, A[i]); }
    }
    mn = wave_min(mn);
    mx = wave_max(mx);
    if (lane == 0) { s_mm[0][wid] = mn; s_mm[1][wid] = mx; }
  }
  __syncthreads();
  if (a.mode_scores) {
    mn = fminf(fminf(s_mm[0][0], s_mm[0][1]), fminf(s_mm[0][2], s_mm[0][3]));
    mx = fmaxf(fmaxf(s_mm[1][0], s_mm[1][1]), fmaxf(s_mm[1][2], s_mm[1][3]));
    den = rnd_dt(a.a_dtype, mx - mn);
    eps = rnd_dt(a.a_dtype, 1e-8f);
  }
  uint32_t* h1 = g.L.hist + ((size_t)b * 2 + 0) * kG * (kCoarse + kFine);
  __shared__ uint32_t lcoarse[kG][kCoarse];
  if (a.mode_select) coarse_clear(lcoarse);
  // ---- scores, classes, round-1 histograms
  const int64_t i0 = (int64_t)blk * kBT;
  double lsum = 0.0;
  uint32_t kmin = 0xffffffffu, kmax = 0u;
  uint32_t ckmin[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, ckmax[3] = {0u, 0u, 0u};
  int64_t cnt[3] = {0, 0, 0};
  for (int j = threadIdx.x; j < kBT; j += kNT) {
    const int64_t i = i0 + j;
    const bool valid = i < S;
    float s = 0.f;
    int l = 0;
    if (valid) {
      if (a.mode_scores) {
        const float Ai = a.A[(int64_t)b * S + i];
        const int dt = a.a_dtype;
        const float N = (den > eps) ? rnd_dt(dt, rnd_dt(dt, Ai - mn) / den) : 0.f;
        const float t1 = rnd_dt(dt, rnd_dt(dt, N * a.p.alpha) * a.p.layer_weight);
        const float t2 = a.T2 ? a.T2[i] : a.p.beta * ((S > 1) ? torch_logf((uint32_t)(i + 1)) / a.logS : 0.f);
        s = t1 + t2;
        s = s + a.p.gamma * a.ctx;
        sc[i] = s;
      } else {
        s = sc[i];
      }
      if (a.mode_labels) {
        if (s >= a.p.theta_h) l = 2;
        else if (s >= a.p.theta_m && s < a.p.theta_h) l = 1;
        lb[i] = (uint8_t)l;
      } else {
        l = lb[i];
        if (l > 2) l = 0;
      }
      lsum += (double)s;
      const uint32_t key = score_key(s);
      kmin = key < kmin ? key : kmin;
      kmax = key > kmax ? key : kmax;
      ckmin[l] = key < ckmin[l] ? key : ckmin[l];
      ckmax[l] = key > ckmax[l] ? key : ckmax[l];
    }
    const uint64_t m0 = __ballot(valid && l == 0), m1 = __ballot(valid && l == 1), m2 = __ballot(valid && l == 2);
    cnt[0] += __popcll(m0);
    cnt[1] += __popcll(m1);
    cnt[2] += __popcll(m2);
    if (a.mode_select) {
      const uint32_t key = score_key(s);
      hist_add(h1, lcoarse, l, key >> 16, valid);
      if (a.fb_group) hist_add(h1, lcoarse, 3, key >> 16, valid);
    }
  }
  if (a.mode_select) coarse_flush(h1, lcoarse);
  // block reductions → row accumulators
  lsum = wave_sum(lsum);
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t a1 = __shfl_xor(kmin, o, 64), a2 = __shfl_xor(kmax, o, 64);
    kmin = a1 < kmin ? a1 : kmin;
    kmax = a2 > kmax ? a2 : kmax;
    for (int k = 0; k < 3; ++k) {
      const uint32_t c1 = __shfl_xor(ckmin[k], o, 64), c2 = __shfl_xor(ckmax[k], o, 64);
      ckmin[k] = c1 < ckmin[k] ? c1 : ckmin[k];
      ckmax[k] = c2 > ckmax[k] ? c2 : ckmax[k];
    }
  }
  if (lane == 0) {
    atomicAdd(&s_cnt[0], (unsigned long long)cnt[0]);
    atomicAdd(&s_cnt[1], (unsigned long long)cnt[1]);
    atomicAdd(&s_cnt[2], (unsigned long long)cnt[2]);
    for (int k = 0; k < 3; ++k) {
      atomicMin(&s_ckey[k][0], ckmin[k]);
      atomicMax(&s_ckey[k][1], ckmax[k]);
    }
    atomicMin(&s_key[0], kmin);
    atomicMax(&s_key[1], kmax);
  }
  __syncthreads();
  if (lane == 0) atomicAdd(&s_sum, lsum);
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 0; k < 3; ++k) atomicAdd((unsigned long long*)&st->class_count[k], (unsigned long long)s_cnt[k]);
    atomicAdd(&st->ssum, s_sum);
    atomicMax(&st->smin_key, ~s_key[0]);  // minima stored complemented: the state starts at 0
    atomicMax(&st->smax_key, s_key[1]);
    for (int k = 0; k < 3; ++k) {
      atomicMax(&st->cls_key[k][0], ~s_ckey[k][0]);
      atomicMax(&st->cls_key[k][1], s_ckey[k][1]);
    }
  }
  if (!arrive_last(&st->done_a, gridDim.x, &s_flag)) return;
  // ---- last block of this row: quotas (selective_propagation.py:93-131) + round-1 digits
  __shared__ int64_t q_need[kG];
  __shared__ int q_mode[kG];
  if (threadIdx.x == 0) {
    int64_t cc[3];
    for (int k = 0; k < 3; ++k) cc[k] = (int64_t)ld_sc1((unsigned long long*)&st->class_count[k]);
    rtkv_batch_stats* bs = reinterpret_cast<rtkv_batch_stats*>(a.stats + 1) + b;
    for (int k = 0; k < 3; ++k) bs->class_count[k] = cc[k];
    const double budget = (double)S * a.p.propagation_ratio;
    const double u8 = 8.0 * budget;
    const int64_t U = (u8 >= 0.0) ? (u8 >= 9.0e18 ? (int64_t)9000000000000000000LL : (int64_t)floor(u8)) : -1;
    int64_t used = 0;
    for (int k = 2; k >= 0; --k) {
      const int64_t N = cc[k];
      const int64_t bb = a.p.bits[k];
      int64_t n;
      if (a.mode_select == 2) n = N;  // RTKV_NO_SELECTION
      else if (U < 0) n = 0;
      else if (bb <= 0) n = N;
      else {
        const int64_t fit = (U - used) / bb;
        n = fit < N ? fit : N;
      }
      used += n * (bb > 0 ? bb : 0);
      q_need[k] = n;
      q_mode[k] = (n == 0) ? SEL_NONE : (n == N ? SEL_ALL : SEL_PARTIAL);
      st->quota[k] = n;
    }
    int64_t kf = (int64_t)((double)S * 0.1);  // topk(max(1, int(S * 0.1)))
    if (kf < 1) kf = 1;
    q_need[3] = kf;
    q_mode[3] = !a.fb_group ? SEL_NONE : (kf >= S ? SEL_ALL : SEL_PARTIAL);
    st->quota[3] = kf;
  }
  __syncthreads();
  __shared__ uint32_t q_digit[kG];
  __shared__ int64_t q_above[kG];
  __shared__ bool q_want[kG];
  if (threadIdx.x < kG) q_want[threadIdx.x] = a.mode_select && q_mode[threadIdx.x] == SEL_PARTIAL;
  __syncthreads();
  find_digits(h1, q_want, q_need, q_digit, q_above);
  if (threadIdx.x < kG) {
    const int k = threadIdx.x;
    st->sel_mode[k] = q_mode[k];
    st->prefix[k] = q_digit[k] << 16;
    st->need[k] = q_need[k] - q_above[k];
  }
}

// ------------------------------------------------------------------------------------ K2b
__global__ __launch_bounds__(kNT) void sel_refine_kernel(SelArgs g) {
  const FinalizeArgs& a = g.f;
  __shared__ int s_flag;
  const int b = blockIdx.y, blk = blockIdx.x;
  const int64_t S = a.S;
  SelState* st = g.L.state + b;
  const float* sc = a.scores + (int64_t)b * S;
  const uint8_t* lb = a.labels + (int64_t)b * S;
  uint32_t* h2 = g.L.hist + ((size_t)b * 2 + 1) * kG * (kCoarse + kFine);
  __shared__ uint32_t lcoarse[kG][kCoarse];
  coarse_clear(lcoarse);
  const int mode_l = st->sel_mode[0] | (st->sel_mode[1] << 2) | (st->sel_mode[2] << 4) | (st->sel_mode[3] << 6);
  uint32_t pre[kG];
  for (int k = 0; k < kG; ++k) pre[k] = st->prefix[k] >> 16;
  const int64_t i0 = (int64_t)blk * kBT;
  for (int j = threadIdx.x; j < kBT; j += kNT) {
    const int64_t i = i0 + j;
    const bool valid = i < S;
    uint32_t key = 0;
    int l = 0;
    if (valid) {
      key = score_key(sc[i]);
      l = lb[i];
      if (l > 2) l = 0;
    }
    const bool pc = valid && ((mode_l >> (2 * l)) & 3) == SEL_PARTIAL && (key >> 16) == pre[l];
    const bool pa = valid && ((mode_l >> 6) & 3) == SEL_PARTIAL && (key >> 16) == pre[3];
    hist_add(h2, lcoarse, l, key & 0xffffu, pc);
    if (a.fb_group) hist_add(h2, lcoarse, 3, key & 0xffffu, pa);
  }
  coarse_flush(h2, lcoarse);
  if (!arrive_last(&st->done_b, gridDim.x, &s_flag)) return;
  __shared__ uint32_t q_digit[kG];
  __shared__ int64_t q_above[kG], q_need[kG];
  __shared__ bool q_want[kG];
  if (threadIdx.x < kG) {
    q_want[threadIdx.x] = ((mode_l >> (2 * threadIdx.x)) & 3) == SEL_PARTIAL;
    q_need[threadIdx.x] = st->need[threadIdx.x];
  }
  __syncthreads();
  find_digits(h2, q_want, q_need, q_digit, q_above);
  if (threadIdx.x < kG && q_want[threadIdx.x]) {
    const int k = threadIdx.x;
    st->prefix[k] = (st->prefix[k] & 0xffff0000u) | q_digit[k];
    st->need[k] = q_need[k] - q_above[k];  // ties at the threshold key to take, in index order
  }
}

// ------------------------------------------------------------------------------------ C1
__global__ __launch_bounds__(kNT) void sel_count_kernel(SelArgs g) {
  const FinalizeArgs& a = g.f;
  __shared__ int64_t s_v[10];
  __shared__ double s_m2;
  __shared__ int s_flag;
  const int b = blockIdx.y, blk = blockIdx.x;
  const int64_t S = a.S;
  const SelState* st = g.L.state + b;
  const float* sc = a.scores + (int64_t)b * S;
  const uint8_t* lb = a.labels + (int64_t)b * S;
  int mode[kG];
  uint32_t thr[kG];
  for (int k = 0; k < kG; ++k) { mode[k] = st->sel_mode[k]; thr[k] = st->prefix[k]; }
  int64_t rb[3];
  for (int k = 0; k < 3; ++k) rb[k] = rowbytes_of(a, k);
  if (threadIdx.x < 10) s_v[threadIdx.x] = 0;
  if (threadIdx.x == 0) s_m2 = 0.0;
  __syncthreads();
  // Σ (s - mean)² over the whole layer (all rows): the mean needs every row's sum (K2a done)
  double tot = 0.0;
  for (int bb = 0; bb < a.B; ++bb) tot += g.L.state[bb].ssum;
  const double mean = tot / (double)(a.B * S);
  int64_t v[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // gt_rows[2], gt_bytes[2], ties[4], -, -
  double m2 = 0.0;
  const int64_t i0 = (int64_t)blk * kBT;
  for (int j = threadIdx.x; j < kBT; j += kNT) {
    const int64_t i = i0 + j;
    if (i >= S) break;
    const float s = sc[i];
    const double d = (double)s - mean;
    m2 += d * d;
    const uint32_t key = score_key(s);
    int l = lb[i];
    if (l > 2) l = 0;
    // class mode
    if (mode[l] == SEL_ALL || (mode[l] == SEL_PARTIAL && key > thr[l])) { v[0]++; v[2] += rb[l]; }
    else if (mode[l] == SEL_PARTIAL && key == thr[l]) v[4 + l]++;
    // fallback mode (all tokens)
    if (mode[3] == SEL_ALL || (mode[3] == SEL_PARTIAL && key > thr[3])) { v[1]++; v[3] += rb[l]; }
    else if (mode[3] == SEL_PARTIAL && key == thr[3]) { v[7]++; v[8] += rb[l]; }
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) v[k] = wave_sum(v[k]);
  m2 = wave_sum(m2);
  if ((threadIdx.x & 63) == 0) {
    for (int k = 0; k < 9; ++k) atomicAdd((unsigned long long*)&s_v[k], (unsigned long long)v[k]);
    atomicAdd(&s_m2, m2);
  }
  __syncthreads();
  SelPartial* pp = g.L.part + (size_t)b * g.L.nb + blk;
  if (threadIdx.x == 0) {
    st_sc1(&pp->gt_rows[0], s_v[0]);
    st_sc1(&pp->gt_rows[1], s_v[1]);
    st_sc1(&pp->gt_bytes[0], s_v[2]);
    st_sc1(&pp->gt_bytes[1], s_v[3]);
    for (int k = 0; k < kG; ++k) st_sc1(&pp->ties[k], s_v[4 + k]);
    st_sc1(&pp->ties_bytes3, s_v[8]);
    atomicAdd(&a.stats->score_m2, s_m2);
  }
  if (!arrive_last(&g.L.glob->done_c1, gridDim.x * gridDim.y, &s_flag)) return;
  // ---- last block of the whole call: fallback decision + statistics
  if (threadIdx.x != 0) return;
  int64_t max_kept = 0;
  for (int bb = 0; bb < a.B; ++bb) {
    const SelState* sb = g.L.state + bb;
    const int64_t kept = (a.mode_select == 2) ? S : sb->quota[0] + sb->quota[1] + sb->quota[2];
    if (kept > max_kept) max_kept = kept;
  }
  const int fallback = (a.mode_select == 1 && !(a.p.flags & RTKV_NO_FALLBACK) && max_kept == 0 && S > 0) ? 1 : 0;
  int64_t total_bytes = 0;
  for (int bb = 0; bb < a.B; ++bb) {
    const SelState* sb = g.L.state + bb;
    rtkv_batch_stats* bs = reinterpret_cast<rtkv_batch_stats*>(a.stats + 1) + bb;
    if (!fallback) {
      int64_t kept = 0, units = 0, bytes = 0;
      for (int k = 0; k < 3; ++k) {
        const int64_t n = sb->quota[k];
        bs->kept_class[k] = n;
        kept += n;
        units += n * a.p.bits[k];
        bytes += n * rowbytes_of(a, k);
      }
      bs->kept = kept;
      bs->cost_units = units;
      bs->packed_bytes = bytes;
      bs->fallback = 0;
      total_bytes += bytes;
    } else {
      bs->kept = sb->quota[3] < S ? sb->quota[3] : S;
      bs->fallback = 1;  // kept_class / cost_units / packed_bytes / score sum: C2 (serial path)
    }
  }
  if (fallback) max_kept = g.L.state[0].quota[3] < S ? g.L.state[0].quota[3] : S;
  g.L.glob->fallback = fallback;
  g.L.glob->max_kept = max_kept;
  rtkv_layer_stats* hs = a.stats;
  hs->max_kept = max_kept;
  hs->total_packed_bytes = total_bytes;  // fallback: C2 adds per row
  double ssum = 0.0;
  uint32_t kmin = 0xffffffffu, kmax = 0u;
  int64_t tc[3] = {0, 0, 0};
  int general = 0;
  for (int bb = 0; bb < a.B; ++bb) {
    const SelState* sb = g.L.state + bb;
    ssum += sb->ssum;
    const uint32_t mnk = ~sb->smin_key;
    kmin = mnk < kmin ? mnk : kmin;
    kmax = sb->smax_key > kmax ? sb->smax_key : kmax;
    for (int k = 0; k < 3; ++k) tc[k] += sb->class_count[k];
    // classes monotone in the score (always true when the classes come from the thresholds)?
    uint32_t lo_bound = 0xffffffffu;  // min key of the higher nonempty classes
    bool first = true;
    for (int k = 2; k >= 0; --k) {
      if (sb->class_count[k] == 0) continue;
      const uint32_t cmn = ~sb->cls_key[k][0], cmx = sb->cls_key[k][1];
      if (!first && !(cmx < lo_bound)) general = 1;
      lo_bound = first ? cmn : (cmn < lo_bound ? cmn : lo_bound);
      first = false;
    }
  }
  g.L.glob->general = (a.mode_select != 0) ? general : 0;
  auto unkey = [](uint32_t k) {
    const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    return __builtin_bit_cast(float, u);
  };
  hs->score_sum = ssum;
  hs->score_min = unkey(kmin);
  hs->score_max = unkey(kmax);
  int flags = 0;
  if (a.kv_dtype == RTKV_F16)
    for (int k = 0; k < 3; ++k)
      if (tc[k] > 0 && a.p.bits[k] >= 16) flags |= RTKV_FLAG_F16_QMAX_OVERFLOW;
  hs->error_flags = flags;
  hs->B = (int32_t)a.B;
}

// ------------------------------------------------------------------------------------ C2
__global__ __launch_bounds__(kNT) void sel_compact_kernel(SelArgs g) {
  const FinalizeArgs& a = g.f;
  __shared__ int64_t s_wv[4][8];
  const int b = blockIdx.y, blk = blockIdx.x;
  const int64_t S = a.S, cap = a.row_capacity;
  const SelState* st = g.L.state + b;
  const float* sc = a.scores + (int64_t)b * S;
  const uint8_t* lb = a.labels + (int64_t)b * S;
  uint8_t* mk = a.mask + (int64_t)b * S;
  if (g.L.glob->general) return;  // sel_general_kernel handles interleaved classes
  const int fallback = g.L.glob->fallback;
  const int64_t max_kept = g.L.glob->max_kept;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t rb[3];
  for (int k = 0; k < 3; ++k) rb[k] = rowbytes_of(a, k);
  // byte base of this batch row: packed bytes of the rows before it
  int64_t row_off_base = 0;
  for (int bb = 0; bb < b; ++bb) row_off_base += reinterpret_cast<const rtkv_batch_stats*>(a.stats + 1)[bb].packed_bytes;
  if (fallback) {
    // rare emergency path: block 0 of every row ranks the whole row (top-k over all tokens)
    if (blk != 0) return;
    // (row byte base needs every previous row's fallback bytes: rows run one after another)
    __shared__ int64_t s_base;
    if (b > 0) {
      if (threadIdx.x == 0) {
        // wait-free: recompute previous rows' bytes serially from their masks is costly; fallback rows
        // each keep the same k tokens, bytes differ by class, so recompute from labels here.
        int64_t base = 0;
        for (int bb = 0; bb < b; ++bb) {
          const SelState* sb = g.L.state + bb;
          const float* scb = a.scores + (int64_t)bb * S;
          const uint8_t* lbb = a.labels + (int64_t)bb * S;
          int64_t ties = 0;
          for (int64_t i = 0; i < S; ++i) {
            const uint32_t key = score_key(scb[i]);
            int l = lbb[i];
            if (l > 2) l = 0;
            bool sel = sb->sel_mode[3] == SEL_ALL || key > sb->prefix[3] ||
                       (key == sb->prefix[3] && ties++ < sb->need[3]);
            if (sel) base += rb[l];
          }
        }
        s_base = base;
      }
      __syncthreads();
      row_off_base = s_base;
    }
    int64_t row = 0, bytes = 0, ties = 0, kc[3] = {0, 0, 0}, units = 0;
    double ksum = 0.0;
    for (int64_t t0 = 0; t0 < S; t0 += kNT) {
      const int64_t i = t0 + threadIdx.x;
      const bool valid = i < S;
      uint32_t key = 0;
      int l = 0;
      if (valid) { key = score_key(sc[i]); l = lb[i]; if (l > 2) l = 0; }
      const bool tie = valid && st->sel_mode[3] == SEL_PARTIAL && key == st->prefix[3];
      const uint64_t tb = __ballot(tie);
      if (lane == 0) s_wv[0][wid] = __popcll(tb);
      __syncthreads();
      int64_t tbase = ties;
      for (int w = 0; w < wid; ++w) tbase += s_wv[0][w];
      const int64_t trank = tbase + __popcll(tb & lanemask_lt());
      const bool sel = valid && (st->sel_mode[3] == SEL_ALL || key > st->prefix[3] || (tie && trank < st->need[3]));
      uint64_t sl[3];
      for (int k = 0; k < 3; ++k) sl[k] = __ballot(sel && l == k);
      if (lane == 0) for (int k = 0; k < 3; ++k) s_wv[1 + k][wid] = __popcll(sl[k]);
      __syncthreads();
      int64_t r0 = row, by0 = bytes;
      for (int w = 0; w < wid; ++w)
        for (int k = 0; k < 3; ++k) { r0 += s_wv[1 + k][w]; by0 += s_wv[1 + k][w] * rb[k]; }
      for (int k = 0; k < 3; ++k) {
        const int64_t before = __popcll(sl[k] & lanemask_lt());
        r0 += before;
        by0 += before * rb[k];
      }
      if (valid) mk[i] = sel ? 1 : 0;
      if (sel && r0 < cap) {
        a.kept_index[(int64_t)b * cap + r0] = (int32_t)i;
        if (a.row_offset) a.row_offset[(int64_t)b * cap + r0] = row_off_base + by0;
      }
      for (int w = 0; w < 4; ++w) {
        ties += s_wv[0][w];
        for (int k = 0; k < 3; ++k) { row += s_wv[1 + k][w]; bytes += s_wv[1 + k][w] * rb[k]; kc[k] += s_wv[1 + k][w]; units += s_wv[1 + k][w] * a.p.bits[k]; }
      }
      if (sel) ksum += (double)sc[i];
      __syncthreads();
    }
    ksum = wave_sum(ksum);
    __shared__ double s_ks;
    if (threadIdx.x == 0) s_ks = 0.0;
    __syncthreads();
    if (lane == 0) atomicAdd(&s_ks, ksum);
    __syncthreads();
    if (threadIdx.x == 0) {
      rtkv_batch_stats* bs = reinterpret_cast<rtkv_batch_stats*>(a.stats + 1) + b;
      for (int k = 0; k < 3; ++k) bs->kept_class[k] = kc[k];
      bs->cost_units = units;
      bs->packed_bytes = bytes;
      bs->kept_score_sum = s_ks;
      atomicAdd((unsigned long long*)&a.stats->total_packed_bytes, (unsigned long long)bytes);
    }
    for (int64_t r = row + threadIdx.x; r < max_kept && r < cap; r += kNT) {
      a.kept_index[(int64_t)b * cap + r] = -1;
      if (a.row_offset) a.row_offset[(int64_t)b * cap + r] = row_off_base + bytes;
    }
    return;
  }
  // ---- class mode: bases from the C1 partials of the blocks before this one
  int mode[3];
  uint32_t thr[3];
  int64_t need[3];
  for (int k = 0; k < 3; ++k) { mode[k] = st->sel_mode[k]; thr[k] = st->prefix[k]; need[k] = st->need[k]; }
  const SelPartial* pp = g.L.part + (size_t)b * g.L.nb;
  // bases = sums over the earlier blocks' C1 partials: wave 0 loads 64 partials per step (lane q
  // ↔ block q), scans ties per group to know how many each earlier block takes, reduces rows/bytes
  __shared__ int64_t s_base[5];
  if (wid == 0) {
    int64_t row_acc = 0, byte_acc = 0, tie_acc[3] = {0, 0, 0};
    for (int q0 = 0; q0 < blk; q0 += 64) {
      const int q = q0 + lane;
      const bool in = q < blk;
      const int64_t gr = in ? pp[q].gt_rows[0] : 0, gb = in ? pp[q].gt_bytes[0] : 0;
      int64_t r_here = gr, b_here = gb;
      for (int k = 0; k < 3; ++k) {
        const int64_t t = in ? pp[q].ties[k] : 0;
        const int64_t before = tie_acc[k] + wave_inclusive_scan(t) - t;  // ties of blocks before q
        int64_t take = need[k] - before;
        take = take < 0 ? 0 : (take > t ? t : take);
        r_here += take;
        b_here += take * rb[k];
        tie_acc[k] += wave_sum(t);
      }
      row_acc += wave_sum(r_here);
      byte_acc += wave_sum(b_here);
    }
    if (lane == 0) {
      s_base[0] = row_acc;
      s_base[1] = byte_acc;
      for (int k = 0; k < 3; ++k) s_base[2 + k] = tie_acc[k];
    }
  }
  __syncthreads();
  int64_t row = s_base[0], bytes = s_base[1], tb[3] = {s_base[2], s_base[3], s_base[4]};
  double ksum = 0.0;
  const int64_t i0 = (int64_t)blk * kBT;
  for (int j0 = 0; j0 < kBT; j0 += kNT) {
    const int64_t i = i0 + j0 + threadIdx.x;
    const bool valid = i < S;
    uint32_t key = 0;
    int l = 0;
    if (valid) { key = score_key(sc[i]); l = lb[i]; if (l > 2) l = 0; }
    const bool part = valid && mode[l] == SEL_PARTIAL;
    const bool tie = part && key == thr[l];
    uint64_t tm[3];
    for (int k = 0; k < 3; ++k) tm[k] = __ballot(tie && l == k);
    if (lane == 0) for (int k = 0; k < 3; ++k) s_wv[k][wid] = __popcll(tm[k]);
    __syncthreads();
    int64_t trank = tb[l];
    for (int w = 0; w < wid; ++w) trank += s_wv[l][w];
    trank += __popcll(tm[l] & lanemask_lt());
    const bool sel = valid && (mode[l] == SEL_ALL || (part && (key > thr[l] || (tie && trank < need[l]))));
    uint64_t sl[3];
    for (int k = 0; k < 3; ++k) sl[k] = __ballot(sel && l == k);
    if (lane == 0) for (int k = 0; k < 3; ++k) s_wv[k][4 + wid] = __popcll(sl[k]);
    __syncthreads();
    int64_t r0 = row, by0 = bytes;
    for (int w = 0; w < wid; ++w)
      for (int k = 0; k < 3; ++k) { r0 += s_wv[k][4 + w]; by0 += s_wv[k][4 + w] * rb[k]; }
    for (int k = 0; k < 3; ++k) {
      const int64_t before = __popcll(sl[k] & lanemask_lt());
      r0 += before;
      by0 += before * rb[k];
    }
    if (valid) mk[i] = sel ? 1 : 0;
    if (sel && r0 < cap) {
      a.kept_index[(int64_t)b * cap + r0] = (int32_t)i;
      if (a.row_offset) a.row_offset[(int64_t)b * cap + r0] = row_off_base + by0;
    }
    if (sel) ksum += (double)sc[i];
    for (int w = 0; w < 4; ++w)
      for (int k = 0; k < 3; ++k) {
        tb[k] += s_wv[k][w];
        row += s_wv[k][4 + w];
        bytes += s_wv[k][4 + w] * rb[k];
      }
    __syncthreads();
  }
  ksum = wave_sum(ksum);
  if (lane == 0) atomicAdd(&(reinterpret_cast<rtkv_batch_stats*>(a.stats + 1) + b)->kept_score_sum, ksum);
  // padding rows of shorter batch rows: kept_index = -1 up to S'_max (the last block of the row)
  if (blk == (int)gridDim.x - 1) {
    const rtkv_batch_stats* bs = reinterpret_cast<const rtkv_batch_stats*>(a.stats + 1) + b;
    const int64_t kept = bs->kept;
    for (int64_t r = kept + threadIdx.x; r < max_kept && r < cap; r += kNT) {
      a.kept_index[(int64_t)b * cap + r] = -1;
      if (a.row_offset) a.row_offset[(int64_t)b * cap + r] = row_off_base + bs->packed_bytes;
    }
  }
}


// ------------------------------------------------------------------------------------ general path
// Classes given by the caller that interleave in score order (select_tokens_with_budget with
// arbitrary labels): the literal greedy over the stable (score desc, index asc) order.  One
// workgroup, bitonic sort in LDS (S ≤ kGenMaxS), then ≤ 4 phases of block scans: in sorted order
// every eligible token is accepted until the first one that does not fit; that token's cost (and every
// larger cost) is then excluded for the rest of the order (the remaining budget only shrinks).
constexpr int kGT = 1024;
constexpr int64_t kGenMaxS = 16384;

__device__ int64_t block_scan_excl(int64_t v, int64_t* sh, int64_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t inc = wave_inclusive_scan(v);
  if (lane == 63) sh[wid] = inc;
  __syncthreads();
  int64_t base = 0, tot = 0;
  for (int w = 0; w < kGT / 64; ++w) {
    if (w < wid) base += sh[w];
    tot += sh[w];
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

__global__ __launch_bounds__(kGT) void sel_general_kernel(SelArgs g) {
  const FinalizeArgs& a = g.f;
  if (!g.L.glob->general) return;
  extern __shared__ __attribute__((aligned(16))) uint64_t items[];
  __shared__ int64_t s_red[kGT / 64 + 2];
  __shared__ int64_t s_fail;
  const int64_t S = a.S, B = a.B, cap = a.row_capacity;
  int n = 1;
  while (n < S) n <<= 1;
  int64_t rb[3];
  for (int k = 0; k < 3; ++k) rb[k] = rowbytes_of(a, k);
  const double budget = (double)S * a.p.propagation_ratio;
  const double u8 = 8.0 * budget;
  const int64_t U = (u8 >= 0.0) ? (u8 >= 9.0e18 ? (int64_t)9000000000000000000LL : (int64_t)floor(u8)) : -1;
  auto cost_of = [&](int64_t idx, const uint8_t* lb) -> int64_t {
    const int l = lb[idx];
    return l <= 2 ? a.p.bits[l] : 0;  // classes outside {0,1,2} cost 0 (selective_propagation.py:54-66)
  };
  auto sort_row = [&](int64_t b) {
    const float* sc = a.scores + b * S;
    for (int t = threadIdx.x; t < n; t += kGT)
      items[t] = t < S ? (((uint64_t)score_key(sc[t]) << 32) | (uint64_t)(0xffffffffu - (uint32_t)t)) : 0ull;
    __syncthreads();
    for (int k = 2; k <= n; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int t = threadIdx.x; t < n; t += kGT) {
          const int p = t ^ j;
          if (p > t) {
            const uint64_t x = items[t], y = items[p];
            const bool desc = (t & k) == 0;
            if (desc ? (x < y) : (x > y)) { items[t] = y; items[p] = x; }
          }
        }
        __syncthreads();
      }
  };
  // pass 1: greedy per row
  int64_t max_sel = 0;
  for (int64_t b = 0; b < B; ++b) {
    const uint8_t* lb = a.labels + b * S;
    uint8_t* mk = a.mask + b * S;
    for (int64_t i = threadIdx.x; i < S; i += kGT) mk[i] = 0;
    sort_row(b);
    int64_t pos = 0, cur = 0, cmax = INT64_MAX, nsel = 0;
    if (U >= 0) {
      while (true) {
        // eligible costs from pos onward, per-thread contiguous chunks of the sorted order
        const int64_t chunk = (n - pos + kGT - 1) / kGT;
        const int64_t lo = pos + (int64_t)threadIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
        int64_t mine = 0;
        for (int64_t t = lo; t < hi; ++t) {
          const uint64_t it = items[t];
          if (t >= S || it == 0ull) continue;
          const int64_t idx = 0xffffffffu - (uint32_t)it;
          const int64_t c = cost_of(idx, lb);
          if (c < cmax) mine += c;
        }
        int64_t tot;
        int64_t run = cur + block_scan_excl(mine, s_red, &tot);
        if (threadIdx.x == 0) s_fail = INT64_MAX;
        __syncthreads();
        for (int64_t t = lo; t < hi; ++t) {
          const uint64_t it = items[t];
          if (t >= S || it == 0ull) continue;
          const int64_t idx = 0xffffffffu - (uint32_t)it;
          const int64_t c = cost_of(idx, lb);
          if (c >= cmax) continue;
          if (run + c > U) { atomicMin((unsigned long long*)&s_fail, (unsigned long long)t); break; }
          run += c;
        }
        __syncthreads();
        const int64_t fail = s_fail;
        // accept every eligible token in [pos, fail)
        int64_t acc = 0, accb = 0;
        for (int64_t t = lo; t < hi && t < fail; ++t) {
          const uint64_t it = items[t];
          if (t >= S || it == 0ull) continue;
          const int64_t idx = 0xffffffffu - (uint32_t)it;
          const int64_t c = cost_of(idx, lb);
          if (c < cmax) { mk[idx] = 1; acc++; accb += c; }
        }
        int64_t tot_acc, tot_c;
        block_scan_excl(acc, s_red, &tot_acc);
        block_scan_excl(accb, s_red, &tot_c);
        nsel += tot_acc;
        cur += tot_c;
        if (fail == INT64_MAX) break;
        const uint64_t it = items[fail];
        cmax = cost_of(0xffffffffu - (uint32_t)it, lb);
        pos = fail + 1;
        __syncthreads();
      }
    }
    if (nsel > max_sel) max_sel = nsel;
    __syncthreads();
  }
  // pass 2: emergency fallback (selective_propagation.py:205-211)
  const int fallback = (!(a.p.flags & RTKV_NO_FALLBACK) && max_sel == 0 && S > 0) ? 1 : 0;
  if (fallback) {
    int64_t k = (int64_t)((double)S * 0.1);
    if (k < 1) k = 1;
    for (int64_t b = 0; b < B; ++b) {
      uint8_t* mk = a.mask + b * S;
      sort_row(b);
      for (int64_t t = threadIdx.x; t < S; t += kGT) mk[0xffffffffu - (uint32_t)items[t]] = t < k ? 1 : 0;
      __syncthreads();
    }
  }
  // compaction in index order + statistics
  int64_t off_base = 0, max_kept = 0;
  for (int64_t b = 0; b < B; ++b) {
    const float* sc = a.scores + b * S;
    const uint8_t* lb = a.labels + b * S;
    const uint8_t* mk = a.mask + b * S;
    const int64_t chunk = (S + kGT - 1) / kGT;
    const int64_t lo = (int64_t)threadIdx.x * chunk, hi = lo + chunk < S ? lo + chunk : S;
    int64_t cnt = 0, bytes = 0, kc[3] = {0, 0, 0}, units = 0;
    double ks = 0.0;
    for (int64_t i = lo; i < hi; ++i) {
      if (!mk[i]) continue;
      int l = lb[i];
      l = l > 2 ? 0 : l;
      cnt++;
      bytes += rb[l];
      kc[l]++;
      units += (lb[i] <= 2) ? a.p.bits[l] : 0;
      ks += (double)sc[i];
    }
    int64_t tot_cnt, tot_bytes, t0, t1, t2, t3;
    int64_t row = block_scan_excl(cnt, s_red, &tot_cnt);
    int64_t off = off_base + block_scan_excl(bytes, s_red, &tot_bytes);
    block_scan_excl(kc[0], s_red, &t0);
    block_scan_excl(kc[1], s_red, &t1);
    block_scan_excl(kc[2], s_red, &t2);
    block_scan_excl(units, s_red, &t3);
    for (int64_t i = lo; i < hi; ++i) {
      if (!mk[i]) continue;
      int l = lb[i];
      l = l > 2 ? 0 : l;
      if (row < cap) {
        a.kept_index[b * cap + row] = (int32_t)i;
        if (a.row_offset) a.row_offset[b * cap + row] = off;
      }
      row++;
      off += rb[l];
    }
    ks = wave_sum(ks);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = 0;
    __syncthreads();
    __shared__ double s_ks;
    if (threadIdx.x == 0) s_ks = 0.0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) atomicAdd(&s_ks, ks);
    __syncthreads();
    if (threadIdx.x == 0) {
      rtkv_batch_stats* bs = reinterpret_cast<rtkv_batch_stats*>(a.stats + 1) + b;
      bs->kept = tot_cnt;
      bs->kept_class[0] = t0;
      bs->kept_class[1] = t1;
      bs->kept_class[2] = t2;
      bs->cost_units = t3;
      bs->packed_bytes = tot_bytes;
      bs->fallback = fallback;
      bs->kept_score_sum = s_ks;
    }
    off_base += tot_bytes;
    if (tot_cnt > max_kept) max_kept = tot_cnt;
    __syncthreads();
  }
  for (int64_t b = 0; b < B; ++b) {
    const int64_t kept = reinterpret_cast<const rtkv_batch_stats*>(a.stats + 1)[b].kept;
    for (int64_t r = kept + threadIdx.x; r < max_kept && r < cap; r += kGT) a.kept_index[b * cap + r] = -1;
  }
  if (threadIdx.x == 0) {
    a.stats->max_kept = max_kept;
    a.stats->total_packed_bytes = off_base;
    g.L.glob->max_kept = max_kept;
  }
}

// ------------------------------------------------------------------------------------ launcher
size_t select_workspace_bytes(int64_t B, int64_t S) {
  const size_t nb = (size_t)sel_nb(S);
  const size_t pipe = 256 + ((B * sizeof(SelState) + 255) / 256) * 256 + sel_hist_words(B) * 4 + B * nb * sizeof(SelPartial) + 256;
  const size_t fast = select_fast_workspace_bytes(S);  // select_fast.hip shares the region
  return pipe > fast ? pipe : fast;
}

static SelLayout carve_select(void* ws, int64_t B, int64_t S) {
  SelLayout L;
  char* p = static_cast<char*>(ws);
  L.glob = reinterpret_cast<SelGlobal*>(p);
  p += 256;
  L.state = reinterpret_cast<SelState*>(p);
  p += ((B * sizeof(SelState) + 255) / 256) * 256;
  L.hist = reinterpret_cast<uint32_t*>(p);
  p += sel_hist_words(B) * 4;
  L.part = reinterpret_cast<SelPartial*>(p);
  L.nb = sel_nb(S);
  return L;
}

// Bytes at the start of the select workspace that must be zero before K2a (glob + state), and the
// histogram region (zeroed too); both are zeroed by K1 (rtkv_compress_layer) or by hipMemsetAsync.
size_t select_zero_bytes(int64_t B) { return 256 + ((B * sizeof(SelState) + 255) / 256) * 256 + sel_hist_words(B) * 4; }

int launch_select(const FinalizeArgs& f, void* sel_ws, bool zeroed, hipStream_t st) {
  RTKV_REQUIRE(f.scores && f.labels && f.stats, "select: null scores/labels/stats");
  RTKV_REQUIRE(f.B >= 1 && f.S >= 1 && f.B <= 65535, "select: bad shape");
  RTKV_REQUIRE(!f.mode_scores || f.A, "select: null aggregation input");
  RTKV_REQUIRE(f.S < ((int64_t)1 << 31), "select: S must be < 2^31");
  RTKV_REQUIRE(!f.mode_select || f.mask, "select: selection needs a mask buffer");
  if (select_fast_eligible(f)) return launch_select_fast(f, sel_ws, zeroed, st);
  SelArgs g;
  g.f = f;
  // The emergency fallback (selective_propagation.py:205-211) runs only when no token fits the
  // budget.  If U = floor(8·S·ratio) covers the widest class, every non-empty class keeps at least
  // one token, so the fallback group need not be histogrammed at all (the common case).
  {
    const double u8 = 8.0 * ((double)f.S * f.p.propagation_ratio);
    int wmax = 0;
    for (int k = 0; k < 3; ++k) wmax = f.p.bits[k] > wmax ? f.p.bits[k] : wmax;
    const bool possible = f.mode_select == 1 && !(f.p.flags & RTKV_NO_FALLBACK) && !(u8 >= (double)wmax);
    g.f.fb_group = (possible || !f.mode_labels) ? 1 : 0;  // caller classes: keep the general bookkeeping
  }
  g.L = carve_select(sel_ws, f.B, f.S);
  if (!zeroed) {
    RTKV_HIP_CHECK(hipMemsetAsync(sel_ws, 0, select_zero_bytes(f.B), st));
    RTKV_HIP_CHECK(hipMemsetAsync(f.stats, 0, rtkv_stats_bytes(f.B), st));
  }
  const dim3 grid((unsigned)g.L.nb, (unsigned)f.B);
  hipLaunchKernelGGL(sel_scores_kernel, grid, dim3(kNT), 0, st, g);
  RTKV_HIP_CHECK(hipGetLastError());
  if (!f.mode_select) {
    // statistics without selection: one small pass for Σ(s-mean)² and the header
    hipLaunchKernelGGL(sel_count_kernel, grid, dim3(kNT), 0, st, g);
    RTKV_HIP_CHECK(hipGetLastError());
    return RTKV_OK;
  }
  hipLaunchKernelGGL(sel_refine_kernel, grid, dim3(kNT), 0, st, g);
  hipLaunchKernelGGL(sel_count_kernel, grid, dim3(kNT), 0, st, g);
  hipLaunchKernelGGL(sel_compact_kernel, grid, dim3(kNT), 0, st, g);
  RTKV_HIP_CHECK(hipGetLastError());
  if (!f.mode_labels && f.mode_select == 1) {  // caller-given classes may interleave in score order
    RTKV_REQUIRE(f.S <= kGenMaxS, "select: caller classes interleave in score order; the exact general "
                                  "path supports S <= 16384");
    int n = 1;
    while (n < f.S) n <<= 1;
    static bool attr = false;
    if (!attr) {
      RTKV_HIP_CHECK(hipFuncSetAttribute((const void*)sel_general_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)(kGenMaxS * 8)));
      attr = true;
    }
    hipLaunchKernelGGL(sel_general_kernel, dim3(1), dim3(kGT), (size_t)n * 8, st, g);
    RTKV_HIP_CHECK(hipGetLastError());
  }
  return RTKV_OK;
}

}  // namespace rtkv
