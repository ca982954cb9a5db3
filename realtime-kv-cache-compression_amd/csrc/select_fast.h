// select_fast.h — K2 for one batch row (B = 1, S <= 65536: every reference configuration, and the
// replicated global selection of the sequence-sharded prefill up to the north star's S = 64k) in ONE launch instead of select.hip's four, with every per-token pass spread over
// the whole grid.  Same outputs, bit for bit (scores, classes, mask, kept_index, row_offset,
// row_label, counts; the double statistics to 1e-12 relative).
//
// Reference (per batch row), as in select.hip:
//   scores      token_importance.py:134-176   s = α·N·w_l + β·log(i+1)/log(S) + γ·min(1, P/S)
//   min-max     token_importance.py:49-85     (global min/max of A: K1 per-block partials)
//   classes     dynamic_quantization.py:21-60
//   selection   selective_propagation.py:68-161  greedy in closed form: top n_g of each class
//   fallback    selective_propagation.py:205-211  topk(max(1, int(0.1·S))) if nothing selected
//   compaction  selective_propagation.py:214-232  kept rows in ascending original index
//
// G = ceil(S/1024) workgroups of 1024 threads, one token per thread, three phases:
// 1 scores  Scores and classes; per-workgroup class counts and score sums; a 4096-bin histogram per
//           class over a FIXED linear binning of the score range (any monotone map of the score
//           works: the histogram only has to tell which bin holds each class's threshold), and every
//           token's (key, index) appended to a 64-entry slot list of its bin (slot = the histogram
//           atomic's return value, one atomic per bin and wave).
// 2 select  EVERY workgroup (the same inputs, the same deterministic result, so no selection word
//           travels between workgroups; workgroup G−1 publishes the statistics and the early host
//           mirror): once every workgroup's counts and score-sum/range words are published, the quotas
//           n_g from the class counts (the greedy in closed form) and the statistics — a layer that keeps
//           whole classes only is selected here, without waiting for any workgroup's drain; otherwise,
//           once every ready word is in too, per partially kept class the bin where the
//           count from the top reaches n_g (one packed scan for all classes), and the exact threshold
//           from that bin's slot list (≤ 64 entries, one wave): key T and the tie CUTOFF, the index of
//           the n_g-th token in (key desc, index asc) order.  A bin with more than 64 tokens (heavy
//           ties) takes the exact rescan path: all S keys in registers, ≤ 3 LDS-histogram rounds, the
//           cutoff from a block scan of per-thread tie counts.
// 3 compact Every workgroup, its token still in registers: keep decisions, all local (mode, T, cutoff
//           per group); per-class ranks by wave ballots; the workgroup's kept counts per class
//           published, its predecessors' summed (decoupled look-back: every count is published before
//           any is awaited, and all G <= 64 workgroups are resident at once); mask, kept_index,
//           row_label, row_offset; its kept-token statistics are added atomically.
//
// Hand-offs between workgroups are TAGGED 8-byte words (bit 63 set on a zeroed word: the region is
// cleared before every launch), written with sc1 stores and polled with sc1 loads, so a consumer sees
// data and flag in one round trip and producers need no drain between them (MI355X_MICROARCH.md
// hand-off rows: each separate flag or drain costs a memory round trip, ≈1–2 µs).  The one drain
// left is phase 1's: a workgroup's slot-list entries are complete (s_waitcnt vmcnt(0)) before its
// tagged ready word, which phase 2 polls only when a class is partly kept.
#pragma once
#include <type_traits>

#include "common.h"

#ifdef RTKV_SELECT_PROBE  // diagnostic build (tools/k2_probe.hip): phase timestamps (s_memrealtime, 100 MHz)
__device__ unsigned long long g_k2_probe[16];   // the selecting workgroup's phases
__device__ unsigned long long g_k2_clock[16];
__device__ unsigned long long g_k2_wg[64][10];  // per workgroup phase timestamps (G <= 64)
__device__ int g_k2_rep;  // the probe's second pass over phase 2 (warm instruction cache) records at k + 8
#define K2_PROBE(k) do { if (threadIdx.x == 0 && blockIdx.x == (unsigned)((g.f.S + kST - 1) / kST - 1)) { g_k2_probe[(k) + 8 * g_k2_rep] = __builtin_amdgcn_s_memrealtime(); g_k2_clock[(k) + 8 * g_k2_rep] = __builtin_amdgcn_s_memtime(); } } while (0)
#define K2_WG(k) do { if (threadIdx.x == 0) g_k2_wg[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
__device__ int g_k2_twice;  // set by the probe: run phase 2 twice (the first pass cold)
#else
#define K2_PROBE(k) do { } while (0)
#define K2_WG(k) do { } while (0)
#endif

namespace rtkv {

namespace {

constexpr int kST = 1024;          // threads per workgroup
constexpr int kSW = kST / kWave;   // waves
constexpr int kBinBits = 12;
constexpr int kNBin = 1 << kBinBits;
constexpr int kGrp = 4;            // classes LOW, MEDIUM, HIGH + "all tokens" (fallback)
constexpr int kCap = 64;           // slot list entries per bin (one per lane of a wave)
constexpr int kMaxS = 64 * kST;    // 64 tokens per thread in the rescan path (S = 65536: 64 workgroups)
constexpr int kMaxG = kMaxS / kST; // workgroups (<= 64: one wave's lanes poll them all)
constexpr uint64_t kTag = 1ull << 63;
enum { M_NONE = 0, M_ALL = 1, M_PART = 2 };

struct FastHead {                  // zeroed before the launch (K1 or a memset): tagged hand-off words
  uint64_t part[kMaxG];            // phase 1, per workgroup: kTag | class counts (3 x 11 bits), from registers
  uint64_t ready[kMaxG];           // phase 1, per workgroup: kTag once its slot entries, partials, scores and
                                   // classes are complete (drained)
  uint64_t agg[kMaxG];             // phase 3, per workgroup: kTag | kept tokens per class (3 x 11 bits)
  uint64_t pst[kMaxG][4];          // phase 1, per workgroup, from registers: kTag | low / high half of the
                                   // score sum's bits, kTag | score key min, kTag | score key max
};
struct FastPartial {               // phase 1, per workgroup (complete before its counts word)
  double ssum;
  uint32_t kmn, kmx;               // score key range
  double m2;                       // quantization-only kernel: Σ (s - workgroup mean)^2
};
struct FastLayout {
  FastHead* head;                  // zeroed
  uint32_t* hist;                  // [kGrp][kNBin] (zeroed)
  FastPartial* part;               // [G]
  uint64_t* slots;                 // [kGrp][kNBin][kCap] of (key << 32 | index)
};

struct FastArgs {
  FinalizeArgs f;
  FastLayout L;
  float bin_lo[kGrp];              // bin(s) = clamp(floor((s - lo) * inv), 0, kNBin - 1): monotone in s
  float bin_inv[kGrp];
  int hist_fb;                     // histogram the fallback group too (fallback possible)
  rtkv_early_stats* early;         // host-mapped stats mirror (nullable), published by the selecting workgroup
  uint64_t early_seq;
  uint32_t spin_limit;             // polls before a hand-off wait gives up (poll_tagged)
  int withhold;                    // RTKV_TEST_WITHHOLD_SELECTION: workgroup G-1 never publishes its ready
                                   // word (phase 2 times out everywhere when a group is partly kept, the
                                   // only case that reads the histograms); RTKV_TEST_WITHHOLD_LOOKBACK:
                                   // workgroup 0 never publishes its phase-3 counts (the look-back times out
                                   // AFTER the early statistics are out)
};

__device__ __forceinline__ float key_score(uint32_t k) {
  const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __builtin_bit_cast(float, u);
}

// Monotone non-decreasing in the order-preserving key of s (NaNs: sign-bit ones below every
// number, the others above, as in score_key).
__device__ __forceinline__ int bin_of(float s, float lo, float inv) {
  const float x = floorf((s - lo) * inv);
  if (x != x) return (__builtin_bit_cast(uint32_t, s) >> 31) ? 0 : kNBin - 1;
  return x <= 0.f ? 0 : (x >= (float)(kNBin - 1) ? kNBin - 1 : (int)x);
}

// Hide a value's provenance from the optimiser at a phase boundary, so that per-token values derived
// from it (the 2-bit groups) are recomputed in each phase instead of being kept live across phases.
template <typename T> __device__ __forceinline__ void opaque(T& v) { asm volatile("" : "+v"(v)); }

__device__ __forceinline__ uint32_t fld(uint64_t v, int g) { return (uint32_t)(v >> (16 * g)) & 0xffffu; }

// Exclusive block scan of a uint32 (block total < 2^32); *total = the block total.  `sh` is a [kSW]
// LDS array private to this call site.
// Inclusive wave scan on DPP lane moves (row_shr within rows of 16, then row_bcast:15 / :31 across
// rows): register-to-register, no LDS round trips as __shfl's ds_bpermute takes.
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v) {
  int x = (int)v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 into rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 into rows 2, 3
  return (uint32_t)x;
}

// Exclusive block scans of four uint32 counters (block totals < 2^32: a group's count reaches S = 65536,
// so 16-bit fields packed two to a word would carry into each other) as four DPP wave scans sharing one
// barrier: the threshold bins of every partially kept group in one pass.  `sh` is a [kGrp][kSW] LDS
// array private to the call site.
__device__ __forceinline__ void block_excl_scan32x4(const uint32_t (&v)[kGrp], uint32_t (&ex)[kGrp],
                                                    uint32_t (*sh)[kSW]) {
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  uint32_t inc[kGrp];
#pragma unroll
  for (int q = 0; q < kGrp; ++q) inc[q] = wave_scan_dpp(v[q]);
  if (lane == kWave - 1) {
#pragma unroll
    for (int q = 0; q < kGrp; ++q) sh[q][wid] = inc[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kGrp; ++q) {
    uint32_t w = sh[q][lane & (kSW - 1)];
#pragma unroll
    for (int o = 1; o < kSW; o <<= 1) {
      const uint32_t n = __shfl_up(w, o, kWave);
      if ((lane & (kSW - 1)) >= o) w += n;
    }
    const uint32_t base = wid > 0 ? __shfl(w, wid - 1, kWave) : 0u;
    ex[q] = base + inc[q] - v[q];
  }
}

// Ranks in thread order of NF one-bit flags per thread, and their workgroup totals, from wave
// ballots (the popcount below the lane plus the counts of the preceding waves): one barrier, no
// shuffles.  `sh` is an [NF][kSW] LDS array private to the call site.
template <int NF>
__device__ __forceinline__ void block_flag_ranks(const bool (&f)[NF], uint32_t (&rank)[NF], uint32_t (&total)[NF],
                                                 uint32_t (*sh)[kSW]) {
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const uint64_t lt = (1ull << lane) - 1ull;
  uint64_t b[NF];
#pragma unroll
  for (int q = 0; q < NF; ++q) {
    b[q] = __ballot(f[q]);
    if (lane == 0) sh[q][wid] = (uint32_t)__popcll(b[q]);
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NF; ++q) {
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kSW; ++w) {
      const uint32_t v = sh[q][w];
      tot += v;
      before += w < wid ? v : 0u;
    }
    rank[q] = before + (uint32_t)__popcll(b[q] & lt);
    total[q] = tot;
  }
}

__device__ __forceinline__ int64_t row_bytes(const FinalizeArgs& a, int lab) {
  return (a.F * field_width(a.kv_dtype < 0 ? RTKV_F32 : a.kv_dtype, a.p.bits[lab]) + 7) / 8;
}

__device__ __forceinline__ float bin_lo_of(const FastArgs& g, int q) {
  return q == 3 ? g.bin_lo[3] : (q == 2 ? g.bin_lo[2] : (q == 1 ? g.bin_lo[1] : g.bin_lo[0]));
}
__device__ __forceinline__ float bin_inv_of(const FastArgs& g, int q) {
  return q == 3 ? g.bin_inv[3] : (q == 2 ? g.bin_inv[2] : (q == 1 ? g.bin_inv[1] : g.bin_inv[0]));
}

__device__ __forceinline__ int class_of(float s, const rtkv_layer_params& p) {
  return (s >= p.theta_h) ? 2 : ((s >= p.theta_m && s < p.theta_h) ? 1 : 0);  // dynamic_quantization.py:41-45
}


// 16-bit packed fields <-> 11-bit packed fields (per-workgroup counts are <= 1024)
__device__ __forceinline__ uint64_t to11(uint64_t v16, int n) {
  uint64_t r = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < n) r |= (uint64_t)fld(v16, q) << (11 * q);
  return r;
}
// 11-bit per-workgroup class counts -> 21-bit fields: a sum over the <= 64 workgroups of a row (up to
// S = 65536 tokens in one class) never carries into the next field
__device__ __forceinline__ uint64_t from11w(uint64_t v11) {
  return (v11 & 0x7ffull) | (((v11 >> 11) & 0x7ffull) << 21) | (((v11 >> 22) & 0x7ffull) << 42);
}
__device__ __forceinline__ uint32_t fldw(uint64_t v, int g) { return (uint32_t)(v >> (21 * g)) & 0x1fffffu; }

// A histogram increment whose return value is the token's slot, aggregated over the wave: lanes with
// the same bin id v (< 2^14) share one atomic by the lowest of them, and each takes base + its rank
// among those peers (the slot order within a bin is arbitrary anyway: slot lists are ranked by
// (key, index)).  Attention-like importance piles thousands of tokens into a few bins, where one
// returning atomic per token serialises on the address (~11 ns each).
// Split in two so that independent work can run while the atomic is in flight: hist_issue sends it,
// hist_slot_of (the first use of its return value) waits for it.
struct HistTicket {
  uint32_t base;  // the leader's atomic return (pending until hist_slot_of)
  int leader, below;
};
__device__ __forceinline__ HistTicket hist_issue(uint32_t* addr, uint32_t v, bool part) {
  uint64_t peers = __ballot(part);
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const uint64_t bk = __ballot((v >> k) & 1u);
    peers &= ((v >> k) & 1u) ? bk : ~bk;
  }
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t below = peers & ((1ull << lane) - 1ull);
  HistTicket h;
  h.leader = peers ? __ffsll((unsigned long long)peers) - 1 : 0;
  h.below = __popcll(below);
  h.base = 0u;
  if (part && below == 0ull) h.base = atomicAdd(addr, (uint32_t)__popcll(peers));
  return h;
}
__device__ __forceinline__ uint32_t hist_slot_of(const HistTicket& h) {
  return (uint32_t)__shfl((int)h.base, h.leader, kWave) + (uint32_t)h.below;
}

// A 16-byte coherent load (global_load_dwordx4 ... sc1, as ld_sc1 for one word).  The compiler does not
// track inline-asm loads: the caller waits (s_waitcnt vmcnt(0)) before the first use.
__device__ __forceinline__ rtkv_u32x4 ld16_sc1(const uint32_t* p) {
  rtkv_u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// Poll tagged words: lanes l < n of the calling wave wait for words[l * stride] to carry kTag and
// return it (0 for the other lanes).  Bounded: after `limit` polls (≈1 µs each: a coherent load round
// trip plus s_sleep) a lane gives up with an untagged 0 and RTKV_FLAG_SPIN_TIMEOUT is raised in the
// layer statistics, so a hand-off that never comes ends the kernel instead of hanging the GPU.
__device__ __forceinline__ uint64_t poll_tagged(const uint64_t* words, int stride, int n, uint32_t limit,
                                                rtkv_layer_stats* stats) {
  const int lane = threadIdx.x & (kWave - 1);
  uint64_t w = 0;
  if (lane < n) {
    w = ld_sc1(words + (size_t)lane * stride);
    for (uint32_t it = 0; !(w & kTag); ++it) {
      if (it >= limit) {
        atomicOr(&stats->error_flags, (int)RTKV_FLAG_SPIN_TIMEOUT);
        w = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      w = ld_sc1(words + (size_t)lane * stride);
    }
  }
  return w;
}

// ------------------------------------------------------------------------------------ rescan path
// Exact threshold of every group in `heavy` (a threshold bin with more than kCap tokens: heavy
// ties) from all S keys: candidates = the group's tokens in its threshold bin, then ≤ 3 rounds of
// key-range LDS histograms (span −12 bits per round).  need[q]: tokens to take from the candidates on
// entry, tokens at the threshold key on exit.  Thread t owns tokens [t·TPT, (t+1)·TPT) (TPT = S/1024
// rounded up to 16, 32 or 64).  The scores are reloaded (from L2) in chunks of 8 for every pass, so nothing
// per token stays live: the rare heavy-tie path pays the reloads instead of the whole kernel paying TPT
// registers of keys (held in registers, the keys spilled 15 VGPRs at TPT = 16 and 110 at TPT = 32 once the
// scans went to 32 bits; streamed, the kernel takes 99-100 VGPRs at every TPT and spills none).
template <int TPT>
__device__ __forceinline__ void rescan_thresholds(const FastArgs& g, uint32_t* hist_lds, int heavy, bool fallback,
                                                  const int (&bstar)[kGrp], int (&need)[kGrp], uint32_t (&thr)[kGrp],
                                                  uint32_t (&cut)[kGrp]) {
  constexpr int kCh = 8;  // tokens per load batch
  using Mask = typename std::conditional<(TPT > 32), uint64_t, uint32_t>::type;
  const FinalizeArgs& a = g.f;
  __shared__ uint32_t s_scan[4][kGrp][kSW];
  __shared__ uint32_t s_key[2 * kGrp][kSW];
  __shared__ uint32_t s_pick[2][kGrp][2];
  __shared__ uint32_t s_cs[kGrp][kSW];
  __shared__ uint32_t s_cut[kGrp];
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const int S = (int)a.S;
  const int i0 = t * TPT;
  const int nv = S - i0 < 0 ? 0 : (S - i0 > TPT ? TPT : S - i0);
  // a token's group, and whether it is a candidate of group q (q heavy, the token in q's threshold bin)
  auto group_of = [&](float s) { return fallback ? 3 : class_of(s, a.p); };
  auto cand_q = [&](float s, int e, int k, int q) {
    return (k < nv) & (e == q) & (((heavy >> q) & 1) != 0) & (bin_of(s, g.bin_lo[q], g.bin_inv[q]) == bstar[q]);
  };
  uint32_t kmn[kGrp], kmx[kGrp];
#pragma unroll
  for (int q = 0; q < kGrp; ++q) { kmn[q] = 0xffffffffu; kmx[q] = 0u; }
#pragma unroll 1
  for (int k0 = 0; k0 < TPT; k0 += kCh) {
    float sv[kCh];
#pragma unroll
    for (int j = 0; j < kCh; ++j) sv[j] = ld_sc1(a.scores + (i0 + k0 + j < S ? i0 + k0 + j : S - 1));
#pragma unroll
    for (int j = 0; j < kCh; ++j) {
      const float s = sv[j];
      const int e = group_of(s);
      const uint32_t kk = score_key(s);
#pragma unroll
      for (int q = 0; q < kGrp; ++q) {
        const bool cq = cand_q(s, e, k0 + j, q);
        kmn[q] = cq ? min(kmn[q], kk) : kmn[q];
        kmx[q] = cq ? max(kmx[q], kk) : kmx[q];
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int q = 0; q < kGrp; ++q) {
      kmn[q] = min(kmn[q], (uint32_t)__shfl_xor((int)kmn[q], o, kWave));
      kmx[q] = max(kmx[q], (uint32_t)__shfl_xor((int)kmx[q], o, kWave));
    }
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < kGrp; ++q) { s_key[q][wid] = kmn[q]; s_key[kGrp + q][wid] = kmx[q]; }
  }
  __syncthreads();
  uint32_t lo[kGrp], hi[kGrp];
  {
    const int src = lane & (kSW - 1);
#pragma unroll
    for (int q = 0; q < kGrp; ++q) { kmn[q] = s_key[q][src]; kmx[q] = s_key[kGrp + q][src]; }
#pragma unroll
    for (int o = kSW / 2; o > 0; o >>= 1)
#pragma unroll
      for (int q = 0; q < kGrp; ++q) {
        kmn[q] = min(kmn[q], (uint32_t)__shfl_xor((int)kmn[q], o, kWave));
        kmx[q] = max(kmx[q], (uint32_t)__shfl_xor((int)kmx[q], o, kWave));
      }
#pragma unroll
    for (int q = 0; q < kGrp; ++q) { lo[q] = kmn[q]; hi[q] = kmx[q]; }
  }
#pragma unroll 1
  for (int round = 0; round < 4; ++round) {
    int act = 0, sh[kGrp];
#pragma unroll
    for (int q = 0; q < kGrp; ++q) {
      if (((heavy >> q) & 1) && lo[q] != hi[q]) act |= 1 << q;
      const int bl = 32 - __clz((int)(hi[q] - lo[q]));
      sh[q] = bl > kBinBits ? bl - kBinBits : 0;
    }
    if (!act) break;
    for (int w = t; w < kGrp * kNBin / 4; w += kST) reinterpret_cast<uint4*>(hist_lds)[w] = make_uint4(0u, 0u, 0u, 0u);
    if (t < kGrp) { s_pick[round & 1][t][0] = 0u; s_pick[round & 1][t][1] = 0u; }
    __syncthreads();
    // each candidate token into its group's key-range histogram (per-group compares combined by masks: no
    // per-token indexing)
#pragma unroll 1
    for (int k0 = 0; k0 < TPT; k0 += kCh) {
      float sv[kCh];
#pragma unroll
      for (int j = 0; j < kCh; ++j) sv[j] = ld_sc1(a.scores + (i0 + k0 + j < S ? i0 + k0 + j : S - 1));
#pragma unroll
      for (int j = 0; j < kCh; ++j) {
        const int e = group_of(sv[j]);
        const uint32_t kk = score_key(sv[j]);
        bool in = false;
        uint32_t off = 0u;
#pragma unroll
        for (int q = 0; q < kGrp; ++q) {
          const bool iq = cand_q(sv[j], e, k0 + j, q) & (((act >> q) & 1) != 0) & (kk >= lo[q]) & (kk <= hi[q]);
          in |= iq;
          off = iq ? (uint32_t)(q * kNBin) + ((kk - lo[q]) >> sh[q]) : off;
        }
        if (in) atomicAdd(&hist_lds[off], 1u);
      }
    }
    __syncthreads();
    uint32_t c[kGrp][4];
    uint32_t pk[kGrp], ex[kGrp];
#pragma unroll
    for (int q = 0; q < kGrp; ++q) {
      const uint4 h4 = (act >> q) & 1 ? reinterpret_cast<const uint4*>(hist_lds + q * kNBin)[kNBin / 4 - 1 - t]
                                      : make_uint4(0u, 0u, 0u, 0u);
      c[q][0] = h4.w; c[q][1] = h4.z; c[q][2] = h4.y; c[q][3] = h4.x;
      pk[q] = c[q][0] + c[q][1] + c[q][2] + c[q][3];
    }
    block_excl_scan32x4(pk, ex, s_scan[round]);
#pragma unroll
    for (int q = 0; q < kGrp; ++q) {
      if (!((act >> q) & 1)) continue;
      int run = (int)ex[q];
      if (run < need[q] && need[q] <= run + (int)pk[q]) {
        bool found = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (!found && run + (int)c[q][j] >= need[q]) {
            s_pick[round & 1][q][0] = (uint32_t)(kNBin - 1 - 4 * t - j);
            s_pick[round & 1][q][1] = (uint32_t)run;
            found = true;
          }
          run += c[q][j];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kGrp; ++q) {
      if (!((act >> q) & 1)) continue;
      const uint64_t nlo = (uint64_t)lo[q] + ((uint64_t)s_pick[round & 1][q][0] << sh[q]);
      const uint64_t nhi = nlo + ((1ull << sh[q]) - 1ull);
      need[q] -= (int)s_pick[round & 1][q][1];
      lo[q] = (uint32_t)nlo;
      hi[q] = nhi < (uint64_t)hi[q] ? (uint32_t)nhi : hi[q];
    }
  }
  // the ties to take at the exact threshold key lo[q] are the first need[q] of the group's tokens at
  // that key in token order (thread t holds tokens i0..i0+TPT-1, so a block scan of per-thread tie
  // counts is in token order): the cutoff is the index of the last one taken
  // (the scores are reloaded, 4 at a time, so that no per-token key stays live past the rounds)
  Mask atm[kGrp] = {0, 0, 0, 0};
  opaque(heavy);
#pragma unroll 1
  for (int k0 = 0; k0 < TPT; k0 += 4) {
    float s4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) s4[j] = ld_sc1(a.scores + (i0 + k0 + j < S ? i0 + k0 + j : S - 1));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t kk = score_key(s4[j]);
      const int e = group_of(s4[j]);
#pragma unroll
      for (int q = 0; q < kGrp; ++q)
        atm[q] |= (Mask)((k0 + j < nv) & (e == q) & (((heavy >> q) & 1) != 0) & (kk == lo[q])) << (k0 + j);
    }
  }
  uint32_t pc[kGrp], exc[kGrp];
#pragma unroll
  for (int q = 0; q < kGrp; ++q) pc[q] = (uint32_t)__popcll((uint64_t)atm[q]);
  block_excl_scan32x4(pc, exc, s_cs);
#pragma unroll
  for (int q = 0; q < kGrp; ++q) {
    const int base = (int)exc[q];
    if (((heavy >> q) & 1) && base < need[q] && need[q] <= base + (int)pc[q]) {
      Mask m = atm[q];
      for (int j = base + 1; j < need[q]; ++j) m &= m - 1;  // drop the ties taken before the last one
      s_cut[q] = (uint32_t)(i0 + __ffsll((unsigned long long)m) - 1);
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kGrp; ++q)
    if ((heavy >> q) & 1) { thr[q] = lo[q]; cut[q] = s_cut[q]; }
}

// ------------------------------------------------------------------------------------ phase 2
// Workgroup G−1, after its own phase 1: quotas, threshold bins, exact thresholds; publishes the
// selection words and the statistics.  s_selw receives the selection words (thread 0 writes them;
// the caller's barrier publishes them to the workgroup).
// The layer statistics phase 2 knows (class counts, quotas = the final kept counts unless the fallback
// runs, score sum and range, the f16 16-bit flag) into the device block and, with an early buffer, the
// host mirror — published by the selecting workgroup as soon as the quotas and the partials are in,
// before its threshold search: the drop-in host allocates the exact outputs while the selection runs.
// Called by ONE lane; with an early buffer it fills `line` (16 words in LDS) for host_line_store, which the
// whole wave then issues.
__device__ __forceinline__ void publish_stats(const FastArgs& g, bool fallback, double ssum, uint32_t kr0, uint32_t kr1,
                                           const int64_t (&ccount)[3], const int64_t (&quota)[3], uint64_t* line) {
  const FinalizeArgs& a = g.f;
  rtkv_layer_stats* hs = a.stats;
  rtkv_batch_stats* bs = reinterpret_cast<rtkv_batch_stats*>(hs + 1);
  for (int q = 0; q < 3; ++q) bs->class_count[q] = ccount[q];
  bs->fallback = fallback ? 1 : 0;
  hs->score_sum = ssum;
  hs->score_min = key_score(kr0);
  hs->score_max = key_score(kr1);
  int flags = 0;
  if (a.kv_dtype == RTKV_F16)
    for (int q = 0; q < 3; ++q)
      if (ccount[q] > 0 && a.p.bits[q] >= 16) flags |= RTKV_FLAG_F16_QMAX_OVERFLOW;
  if (flags) atomicOr(&hs->error_flags, flags);  // a spin timeout may have been flagged already
  hs->B = 1;
  if (!fallback) {  // the kept counts are the quotas: final here (phase 3 adds only the score sums)
    int64_t n = 0, units = 0, bytes = 0;
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
  if (g.early && line) {  // host-mapped mirror for the caller's early return (rtkv_compress_layer_early)
    const bool complete = !fallback && g.withhold != 1;  // withheld: the host takes the synchronised statistics
    for (int k = 0; k < 16; ++k) line[k] = 0ull;
    line[0] = line[15] = g.early_seq;
    if (complete) {
      line[1] = (uint64_t)bs->kept;
      line[2] = (uint64_t)bs->packed_bytes;
      line[3] = __builtin_bit_cast(uint64_t, ssum);
      line[4] = (uint64_t)__builtin_bit_cast(uint32_t, hs->score_min) |
                ((uint64_t)__builtin_bit_cast(uint32_t, hs->score_max) << 32);
      line[5] = (uint64_t)(uint32_t)(flags | ld_sc1(&hs->error_flags)) | (1ull << 32);
      for (int q = 0; q < 3; ++q) {
        line[6 + q] = (uint64_t)ccount[q];
        line[9 + q] = (uint64_t)quota[q];
      }
      line[12] = (uint64_t)bs->cost_units;
    }
  }
}

// The greedy in closed form (selective_propagation.py:93-131) from a row's class counts N3: per group q
// (LOW, MEDIUM, HIGH, then the fallback's "all tokens") q_mode[q] (M_NONE / M_ALL / M_PART) and
// q_mode[kGrp + q] the tokens to keep (the fallback's k = max(1, int(0.1·S))), quota / ccount the int64
// kept and class counts; returns whether a group is partly kept (a threshold search is needed).
__device__ __forceinline__ bool quotas_closed_form(const FinalizeArgs& a, int S, const uint32_t (&N3)[3], int* q_mode,
                                                   int64_t* quota, int64_t* ccount) {
  // In 32-bit integers: N <= S <= 2^16 and bits <= 16, so every product and quotient that can decide n
  // fits; the budget U = floor(8·S·ratio) (int64 in the reference) is compared as a double, exact below
  // 2^53 (beyond, every class fits whole).
  const double u8 = 8.0 * ((double)S * a.p.propagation_ratio);
  const double Ud = u8 >= 9.0e18 ? 9.0e18 : floor(u8);
  int used = 0, kept = 0;
  bool partly = false;
  for (int k = 2; k >= 0; --k) {
    const int N = (int)N3[k], bb = a.p.bits[k];
    int n;
    if (a.mode_select == 2) n = N;
    else if (!(u8 >= 0.0)) n = 0;  // U = -1 (selective_propagation.py: nothing fits)
    else if (bb <= 0) n = N;
    else {
      const double x = Ud - (double)used;  // U - used >= 0
      n = x >= (double)bb * (double)N ? N : (int)((uint32_t)x / (uint32_t)bb);
    }
    used += n * (bb > 0 ? bb : 0);
    kept += n;
    q_mode[kGrp + k] = n;
    quota[k] = n;
    ccount[k] = N;
    const int md = (n == 0) ? M_NONE : (n == N ? M_ALL : M_PART);
    q_mode[k] = md;
    partly |= md == M_PART;
  }
  int64_t kf = (int64_t)((double)S * 0.1);
  if (kf < 1) kf = 1;
  const bool fb = a.mode_select == 1 && !(a.p.flags & RTKV_NO_FALLBACK) && kept == 0;
  q_mode[kGrp + 3] = (int)kf;
  const int md3 = !fb ? M_NONE : (kf >= S ? M_ALL : M_PART);
  q_mode[3] = md3;
  return partly || md3 == M_PART;
}

// Phase 2's shared state (LDS), written by select_quotas and read by select_thresholds and phase 3.
struct SelShared {
  double ssum;          // the row's score sum
  uint32_t kr[2];       // the row's score key range
  int q[2 * kGrp];      // per group: mode (M_NONE / M_ALL / M_PART), then the tokens to keep
  int64_t cc[3], quota[3];
  int partly;           // a group is partly kept: the threshold search (and phase 1's slot lists) run
};

// Phase 2a, EVERY workgroup: wave 0 waits for every workgroup's class counts and takes the quotas (the
// greedy in closed form), wave 1 for their score sums and ranges — tagged words each workgroup publishes
// from registers right after its scores, so nothing here waits for a drain.  Workgroup G−1 then publishes
// the statistics and the early host mirror.  When no class is partly kept (most layers at ratio >= 0.6
// keep whole classes) the selection is complete here: phase 1's slot lists are never written and no
// ready word is awaited.
template <int TPT>
__device__ __forceinline__ void select_quotas(const FastArgs& g, SelShared& sh, bool publish) {
  const FinalizeArgs& a = g.f;
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const int S = (int)a.S;
  const int G = (S + kST - 1) / kST;
  (void)t;
  K2_PROBE(0);
  if (wid == 0) {
    // ---- every workgroup's class counts, the quotas (selective_propagation.py:93-131), lane l reading
    // workgroup l (G <= 64)
    const uint64_t w = poll_tagged(g.L.head->part, 1, G, g.spin_limit, a.stats);
    uint64_t cnt = lane < G ? from11w(w & ~kTag) : 0ull;
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, kWave);
    if (lane == 0) {
      const uint32_t N3[3] = {(uint32_t)fldw(cnt, 0), (uint32_t)fldw(cnt, 1), (uint32_t)fldw(cnt, 2)};
      sh.partly = quotas_closed_form(a, S, N3, sh.q, sh.quota, sh.cc) ? 1 : 0;
    }
  } else if (wid == 1) {
    // ---- every workgroup's score sum and key range (four tagged words, polled together)
    double p_ss = 0.0;
    uint32_t p_kmn = 0xffffffffu, p_kmx = 0u;
    if (lane < G) {
      const uint64_t* pw = g.L.head->pst[lane];
      uint64_t w0, w1, w2, w3;
      for (uint32_t it = 0;; ++it) {
        w0 = ld_sc1(pw);
        w1 = ld_sc1(pw + 1);
        w2 = ld_sc1(pw + 2);
        w3 = ld_sc1(pw + 3);
        if (w0 & w1 & w2 & w3 & kTag) break;
        if (it >= g.spin_limit) {
          atomicOr(&a.stats->error_flags, (int)RTKV_FLAG_SPIN_TIMEOUT);
          w0 = w1 = w2 = 0ull;
          w3 = 0ull;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      p_ss = __builtin_bit_cast(double, (w0 & 0xffffffffull) | ((w1 & 0xffffffffull) << 32));
      if (w2 & kTag) p_kmn = (uint32_t)w2;
      p_kmx = (uint32_t)w3;
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {  // lanes >= G hold the neutral values
      p_ss += __shfl_xor(p_ss, o, kWave);
      p_kmn = min(p_kmn, (uint32_t)__shfl_xor((int)p_kmn, o, kWave));
      p_kmx = max(p_kmx, (uint32_t)__shfl_xor((int)p_kmx, o, kWave));
    }
    if (lane == 0) { sh.ssum = p_ss; sh.kr[0] = p_kmn; sh.kr[1] = p_kmx; }
  }
  __syncthreads();
  K2_PROBE(1);
  // statistics known here; phase 3 adds the kept-token sums (stats zeroed before).  Published by the LAST wave
  // (its later vmcnt waits include the host store; wave 0 runs the thresholds and the look-back): lane 0
  // writes the device block and the line's words, the wave stores the host line in one instruction
  if (publish && wid == kSW - 1) {
    __shared__ uint64_t s_line[16];
    if (lane == 0) {
      const int64_t ccount[3] = {sh.cc[0], sh.cc[1], sh.cc[2]};
      const int64_t quota[3] = {sh.quota[0], sh.quota[1], sh.quota[2]};
      publish_stats(g, sh.q[3] != M_NONE, sh.ssum, sh.kr[0], sh.kr[1], ccount, quota, s_line);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");  // (the same wave: its LDS writes are read in order)
    if (g.early) host_line_store(reinterpret_cast<uint64_t*>(g.early), s_line);
  }
}

// Phase 2b, EVERY workgroup, after select_quotas (and, when a class is partly kept, after this workgroup's
// slot lists are drained and its ready word is out): per partly kept group the bin where the count from
// the top reaches its quota (one packed scan), and the exact threshold from that bin's slot list (or the
// rescan rounds); then the selection words into s_selw (thread 0; the caller's barrier publishes them).
template <int TPT>
__device__ __forceinline__ void select_thresholds(const FastArgs& g, uint32_t* hist_lds, uint64_t* s_selw,
                                                  const SelShared& sh) {
  const FinalizeArgs& a = g.f;
  __shared__ uint32_t s_scan32[kGrp][kSW];
  __shared__ uint32_t s_pick[kGrp][3];
  __shared__ uint32_t s_thr[kGrp];
  __shared__ uint32_t s_cutw[kGrp];
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const int S = (int)a.S;
  const int G = (S + kST - 1) / kST;
  const int* s_q = sh.q;
  int mode[kGrp], need[kGrp];
#pragma unroll
  for (int q = 0; q < kGrp; ++q) { mode[q] = s_q[q]; need[q] = s_q[kGrp + q]; }
  const bool fallback = mode[3] != M_NONE;
  int part = 0;
#pragma unroll
  for (int q = 0; q < kGrp; ++q) part |= (mode[q] == M_PART) << q;
  uint32_t thr[kGrp] = {0u, 0u, 0u, 0u}, cut[kGrp] = {0u, 0u, 0u, 0u};
  K2_PROBE(5);
  if (part) {
    // ---- every workgroup's histogram atomics and slot entries complete (its ready word)
    if (wid == 0) (void)poll_tagged(g.L.head->ready, 1, G, g.spin_limit, a.stats);
    __syncthreads();
    // ---- every histogram load the thresholds may need (thread t owns descending bins 4t..4t+3), in one
    // round trip
    const int ngrp = g.hist_fb ? 4 : 3;
    uint32_t c[kGrp][4];
    {
      rtkv_u32x4 h[kGrp];
#pragma unroll
      for (int q = 0; q < kGrp; ++q) {
        h[q] = rtkv_u32x4{0u, 0u, 0u, 0u};
        if (q < ngrp) h[q] = ld16_sc1(g.L.hist + q * kNBin + (kNBin - 4 - 4 * t));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int q = 0; q < kGrp; ++q) { c[q][0] = h[q].w; c[q][1] = h[q].z; c[q][2] = h[q].y; c[q][3] = h[q].x; }
    }
    K2_PROBE(4);
    // ---- the bin holding each partial group's threshold: every partial group's bin counts in one
    // scan (four 32-bit DPP scans, one barrier)
    if (t < kGrp) { s_pick[t][0] = 0u; s_pick[t][1] = 0u; s_pick[t][2] = 0u; }
    uint32_t pk[kGrp], ex[kGrp];
#pragma unroll
    for (int q = 0; q < kGrp; ++q) pk[q] = ((part >> q) & 1) ? c[q][0] + c[q][1] + c[q][2] + c[q][3] : 0u;
    block_excl_scan32x4(pk, ex, s_scan32);
    K2_PROBE(6);
#pragma unroll
    for (int q = 0; q < kGrp; ++q) {
      if (!((part >> q) & 1)) continue;
      const uint32_t sum = pk[q];
      int run = (int)ex[q];
      if (run < need[q] && need[q] <= run + (int)sum) {
        bool found = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (!found && run + (int)c[q][j] >= need[q]) {
            s_pick[q][0] = (uint32_t)(kNBin - 1 - 4 * t - j);
            s_pick[q][1] = (uint32_t)run;          // tokens of the group in higher bins
            s_pick[q][2] = c[q][j];                // tokens in the bin
            found = true;
          }
          run += c[q][j];
        }
      }
    }
    K2_PROBE(7);
    __syncthreads();
    int bstar[kGrp] = {0, 0, 0, 0};
    int heavy = 0;
#pragma unroll
    for (int q = 0; q < kGrp; ++q) {
      if (!((part >> q) & 1)) continue;
      bstar[q] = (int)s_pick[q][0];
      need[q] -= (int)s_pick[q][1];
      if ((int)s_pick[q][2] > kCap) heavy |= 1 << q;
    }
    K2_PROBE(2);
    // ---- light bins: wave q ranks its group's slot list (≤ 64 entries, one per lane)
    if (wid < kGrp && ((part >> wid) & 1) && !((heavy >> wid) & 1)) {
      const int q = wid;
      const int n = (int)s_pick[q][2];
      const uint64_t* sl = g.L.slots + ((size_t)q * kNBin + (size_t)bstar[q]) * kCap;
      const uint64_t e = lane < n ? ld_sc1(sl + lane) : 0ull;
      const uint32_t k = (uint32_t)(e >> 32), idx = (uint32_t)e;
      // rank = entries ahead of this one in (key desc, index asc) order
      int rank = 0;
      for (int j = 0; j < n; ++j) {
        const uint64_t o = __shfl(e, j, kWave);
        const uint32_t ok = (uint32_t)(o >> 32), oi = (uint32_t)o;
        rank += (ok > k) | ((ok == k) & (oi < idx));
      }
      const int r = need[q];  // 1 <= r <= n
      const uint64_t hit = __ballot(lane < n && rank == r - 1);
      const int src = hit ? (__ffsll((unsigned long long)hit) - 1) : 0;
      const uint32_t T = (uint32_t)__shfl((int)k, src, kWave);
      // the r-th token in (key desc, index asc) order is the last one kept: the ties at T with an
      // index up to its index are kept
      const uint32_t cut = (uint32_t)__shfl((int)idx, src, kWave);
      if (lane == 0) { s_thr[q] = T; s_cutw[q] = cut; }
    }
    if (heavy) rescan_thresholds<TPT>(g, hist_lds, heavy, fallback, bstar, need, thr, cut);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kGrp; ++q) {
      if (!((part >> q) & 1) || ((heavy >> q) & 1)) continue;
      thr[q] = s_thr[q];
      cut[q] = s_cutw[q];
    }
  }
  K2_PROBE(3);
  if (t != 0) return;
  // ---- the selection words (this workgroup's phase 3 reads them from LDS)
  const double ssum = sh.ssum;
  const double mean = ssum / (double)S;
  const uint64_t mb = __builtin_bit_cast(uint64_t, mean);
  for (int q = 0; q < kGrp; ++q) {
    const uint64_t w = kTag | ((uint64_t)(fallback ? 1 : 0) << 50) | ((uint64_t)mode[q] << 48) |
                       ((uint64_t)(cut[q] & 0xffff) << 32) | thr[q];
    s_selw[q] = w;
  }
  const uint64_t m_lo = kTag | (mb & 0xffffffffu), m_hi = kTag | (mb >> 32);
  s_selw[4] = m_lo;
  s_selw[5] = m_hi;
}

// ------------------------------------------------------------------------------------ phase 3
// Every workgroup: keep decisions for its token (s, l) still in registers, ranked across the row.
// selw: the selection words in LDS.  A token is kept iff its group takes all of its tokens, or takes
// part and its key is above the threshold T, or at T with an index up to the group's cutoff (phase 2
// resolved the ties, which go in token order): a local decision, so the only exchange is the kept
// count per class for the ranks across workgroups (decoupled look-back).
__device__ __forceinline__ void compact_phase(const FastArgs& g, float s, int l, int i, bool valid,
                                              const uint64_t* selw) {
  const FinalizeArgs& a = g.f;
  __shared__ uint32_t s_f3[3][kSW];
  __shared__ double s_d[2][kSW];
  __shared__ uint64_t s_base;
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const int blk = blockIdx.x;
  const bool fallback = ((selw[0] >> 50) & 1u) != 0;
  const double mean = __builtin_bit_cast(double, (selw[4] & 0xffffffffull) | ((selw[5] & 0xffffffffull) << 32));
  const uint32_t key = score_key(s);
  const int e = valid ? (fallback ? 3 : l) : 4;
  bool kept = false;
#pragma unroll
  for (int q = 0; q < kGrp; ++q) {
    const uint64_t w = selw[q];
    const int mode = (int)((w >> 48) & 3u);
    const uint32_t thr = (uint32_t)w, cut = (uint32_t)((w >> 32) & 0xffffu);
    kept |= (e == q) & ((mode == M_ALL) | ((mode == M_PART) & ((key > thr) | ((key == thr) & ((uint32_t)i <= cut)))));
  }
  // ---- kept-row ranks per class in index order; the workgroup's counts (the aggregate, published
  // before any wait) and the predecessors' (look-back)
  bool f3[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) f3[c] = kept & (l == c);
  uint32_t r3[3], t3[3];
  block_flag_ranks<3>(f3, r3, t3, s_f3);
  const uint64_t kept_tot = (uint64_t)t3[0] | ((uint64_t)t3[1] << 16) | ((uint64_t)t3[2] << 32);
  // statistics partials (Σ kept scores, Σ (s - mean)^2) per wave, while wave 0 waits on the look-back
  {
    const double d = (double)s - mean;
    const double ks = wave_sum(kept ? (double)s : 0.0), m2 = wave_sum(valid ? d * d : 0.0);
    if (lane == 0) { s_d[0][wid] = ks; s_d[1][wid] = m2; }
  }
  if (wid == 0) {
    if (lane == 0 && !(g.withhold == 2 && blk == 0)) st_sc1(&g.L.head->agg[blk], kTag | to11(kept_tot, 3));
    K2_WG(6);
    const uint64_t w0 = poll_tagged(&g.L.head->agg[0], 1, blk, g.spin_limit, a.stats);
    const uint64_t ps = wave_sum(lane < blk ? from11w(w0 & ~kTag) : 0ull);
    if (lane == 0) s_base = ps;
  }
  __syncthreads();
  K2_WG(7);
  const uint64_t kept_before = s_base;
  K2_WG(9);
  int64_t rb[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) rb[q] = row_bytes(a, q);
  if (a.shard_ranges) {
    // rtkv_shard_ranges in this launch (sequence shards): rank j's first output row / packed byte = the kept
    // rows before token j·S_local (r3: this workgroup's kept tokens of each class before this thread, kept or
    // not), and the row's end after the last workgroup's tokens
    const int64_t Sl = a.shard_S_local;
    const int G = ((int)a.S + kST - 1) / kST;
    // (a thread can be both a rank's first token and the row's end writer: thread 0 of the last workgroup)
    for (int end = 0; end < 2; ++end) {
      if (end ? !(blk == G - 1 && t == 0) : !(valid && (int64_t)i % Sl == 0)) continue;
      int64_t nr = 0, nb = 0;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int64_t k = (int64_t)fldw(kept_before, q) + (end ? t3[q] : r3[q]);
        nr += k;
        nb += k * rb[q];
      }
      const int64_t j = end ? (int64_t)a.shard_nranks : (int64_t)i / Sl;
      a.shard_ranges[2 * j] = nr;
      a.shard_ranges[2 * j + 1] = a.row_offset ? nb : 0;
    }
  }
  if (valid) {
    a.mask[i] = kept ? 1 : 0;
    if (kept) {
      const int64_t k0 = (int64_t)r3[0] + fldw(kept_before, 0), k1 = (int64_t)r3[1] + fldw(kept_before, 1),
                    k2 = (int64_t)r3[2] + fldw(kept_before, 2);
      const int64_t row = k0 + k1 + k2;
      if (row < a.row_capacity) {
        a.kept_index[row] = i;
        if (a.row_label) a.row_label[row] = (uint8_t)l;
        if (a.row_offset) a.row_offset[row] = k0 * rb[0] + k1 * rb[1] + k2 * rb[2];
      }
    }
  }
  // ---- statistics: Σ kept scores, Σ (s - mean)^2 and the kept-token counts, added per workgroup (the
  // wave partials were complete at the look-back barrier)
  if (wid == 1) {
    double x = s_d[0][lane & (kSW - 1)], y = s_d[1][lane & (kSW - 1)];
#pragma unroll
    for (int o = kSW / 2; o > 0; o >>= 1) { x += __shfl_xor(x, o, kWave); y += __shfl_xor(y, o, kWave); }
    if (lane == 0) {
      rtkv_layer_stats* hs = a.stats;
      rtkv_batch_stats* bs = reinterpret_cast<rtkv_batch_stats*>(hs + 1);
      unsigned long long n = 0, units = 0, bytes = 0;
      for (int q = 0; q < 3; ++q) {
        const unsigned long long nq = fld(kept_tot, q);
        if (nq && fallback) atomicAdd((unsigned long long*)&bs->kept_class[q], nq);
        n += nq;
        units += nq * (unsigned long long)a.p.bits[q];
        bytes += nq * (unsigned long long)rb[q];
      }
      if (n) {
        if (fallback) {  // otherwise phase 2 wrote the final counts (the quotas)
          atomicAdd((unsigned long long*)&bs->kept, n);
          atomicAdd((unsigned long long*)&bs->cost_units, units);
          atomicAdd((unsigned long long*)&bs->packed_bytes, bytes);
          atomicAdd((unsigned long long*)&hs->max_kept, n);
          atomicAdd((unsigned long long*)&hs->total_packed_bytes, bytes);
        }
        atomicAdd(&bs->kept_score_sum, x);
      }
      atomicAdd(&hs->score_m2, y);
    }
  }
}

// Host: the launch arguments of the one-launch K2 over the selection workspace `ws` (layout
// [FastHead][hist][partials][slots]).
inline FastArgs make_fast_args(const FinalizeArgs& f, void* ws) {
  FastArgs g;
  g.f = f;
  g.early = f.early;
  g.early_seq = f.early_seq;
  g.withhold = (f.p.flags & RTKV_TEST_WITHHOLD_SELECTION) ? 1 : ((f.p.flags & RTKV_TEST_WITHHOLD_LOOKBACK) ? 2 : 0);
  static const uint32_t spin_limit = [] {  // RTKV_SPIN_LIMIT: polls per hand-off wait (default ≈ 2 s)
    const char* e = getenv("RTKV_SPIN_LIMIT");
    return e ? (uint32_t)strtoul(e, nullptr, 10) : (1u << 21);
  }();
  g.spin_limit = spin_limit;
  char* p = static_cast<char*>(ws);
  g.L.head = reinterpret_cast<FastHead*>(p);
  p += sizeof(FastHead);
  g.L.hist = reinterpret_cast<uint32_t*>(p);
  p += (size_t)kGrp * kNBin * 4;
  g.L.part = reinterpret_cast<FastPartial*>(p);
  p += kMaxG * sizeof(FastPartial) + 256;
  g.L.slots = reinterpret_cast<uint64_t*>((reinterpret_cast<uintptr_t>(p) + 255) & ~(uintptr_t)255);
  // Fixed score binning.  s = t1 + t2 + t3 with t1 = α·w·N (N in [0, 1]), t2 = β·pos (pos in
  // [0, 1]), t3 = γ·ctx: any range works for correctness (bins are clamped, the map stays
  // monotone); this one spreads the scores over the bins.
  const double aw = (double)f.p.alpha * (double)f.p.layer_weight, be = f.p.beta, t3 = (double)f.p.gamma * f.ctx;
  double smin = (aw < 0 ? aw : 0.0) + (be < 0 ? be : 0.0) + t3, smax = (aw > 0 ? aw : 0.0) + (be > 0 ? be : 0.0) + t3;
  const double pad = 1e-3 * (smax - smin) + 1e-6;
  smin -= pad;
  smax += pad;
  const double th = f.p.theta_h, tm = f.p.theta_m;
  const double lo[kGrp] = {smin, tm > smin ? tm : smin, th > smin ? th : smin, smin};
  const double hi[kGrp] = {tm < smax ? tm : smax, th < smax ? th : smax, smax, smax};
  for (int q = 0; q < kGrp; ++q) {
    g.bin_lo[q] = (float)lo[q];
    g.bin_inv[q] = hi[q] > lo[q] ? (float)(kNBin / (hi[q] - lo[q])) : 0.f;
  }
  {
    const double u8 = 8.0 * ((double)f.S * f.p.propagation_ratio);
    int wmax = 0;
    for (int k = 0; k < 3; ++k) wmax = f.p.bits[k] > wmax ? f.p.bits[k] : wmax;
    g.hist_fb = (f.mode_select == 1 && !(f.p.flags & RTKV_NO_FALLBACK) && !(u8 >= (double)wmax)) ? 1 : 0;
  }
  return g;
}

// ------------------------------------------------------------------------------------ kernel
// Global min/max of A (token_importance.py:71-83): K1's per-block partials, or the row.  Every
// workgroup of the selection computes it (min/max are exact: the same values everywhere).
__device__ __forceinline__ void amin_amax(const FinalizeArgs& a, float& mn, float& mx) {
  __shared__ float s_mm[2][kSW];
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  mn = INFINITY;
  mx = -INFINITY;
  if (a.A_part) {
    for (int k = t; k < a.A_nparts; k += kST) { mn = fminf(mn, a.A_part[2 * k]); mx = fmaxf(mx, a.A_part[2 * k + 1]); }
  } else if ((a.S & 3) == 0 && ((uintptr_t)a.A & 15) == 0) {
    // the whole row (a gathered A of a sequence-sharded layer, no K1 partials): 16-byte loads, 4 in flight
    const float4* A4 = reinterpret_cast<const float4*>(a.A);
    const int n4 = (int)(a.S >> 2);
#pragma unroll 4
    for (int k = t; k < n4; k += kST) {
      const float4 v = A4[k];
      mn = fminf(mn, fminf(fminf(v.x, v.y), fminf(v.z, v.w)));
      mx = fmaxf(mx, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    }
  } else {
    for (int k = t; k < (int)a.S; k += kST) { mn = fminf(mn, a.A[k]); mx = fmaxf(mx, a.A[k]); }
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  if (lane == 0) { s_mm[0][wid] = mn; s_mm[1][wid] = mx; }
  __syncthreads();
  mn = s_mm[0][lane & (kSW - 1)];
  mx = s_mm[1][lane & (kSW - 1)];
#pragma unroll
  for (int o = kSW / 2; o > 0; o >>= 1) { mn = fminf(mn, __shfl_xor(mn, o, kWave)); mx = fmaxf(mx, __shfl_xor(mx, o, kWave)); }
}

// The importance score of token i (token_importance.py:134-176).  Every op is an fp32 op rounded to
// the dtype (PyTorch CPU).  The barriers keep it so for f16: without them LLVM narrows
// fptrunc(fdiv(fpext h, fpext h)) to an f16 division (not correctly rounded on gfx950) and
// fptrunc(fmul(fpext h, f32)) to v_fma_mix (one rounding instead of two).  The fused kernel's
// quantization waves recompute it with this same code: bit-identical to the score phase 1 stores.
template <int DT, bool HAS_T2>
__device__ __forceinline__ float token_score(const FinalizeArgs& a, int i, float Ai, float T2i, float mn, float den,
                                             float eps) {
  float qn = Dt<DT>::rnd(Ai - mn) / den;
  opaque(qn);
  const float N = (den > eps) ? Dt<DT>::rnd(qn) : 0.f;
  float p1 = N * a.p.alpha;
  opaque(p1);
  float p2 = Dt<DT>::rnd(p1) * a.p.layer_weight;
  opaque(p2);
  const float t1 = Dt<DT>::rnd(p2);
  const float t2 = HAS_T2 ? T2i : a.p.beta * ((a.S > 1) ? torch_logf((uint32_t)(i + 1)) / a.logS : 0.f);
  float s = t1 + t2;
  s = s + a.p.gamma * a.ctx;
  return s;
}

// The selection, in workgroup blk < G of the launch (G = ceil(S / 1024)): phases 1-3 above.
template <int TPT, bool HAS_T2, int DT>
__device__ __forceinline__ void k2_body(const FastArgs& g, uint32_t* hist_lds) {
  const FinalizeArgs& a = g.f;
  __shared__ double s_sum[kSW];
  __shared__ uint32_t s_c[5][kSW];
  __shared__ uint64_t s_selw[8];
  __shared__ SelShared sh;
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const int S = (int)a.S;
  const int G = (S + kST - 1) / kST;
  const int blk = blockIdx.x;
  K2_WG(0);
  // this thread's token's A (and β·pos term) in flight together with the min/max partials: the loads
  // do not depend on the row-wide min/max, and issued here they cost no round trip of their own
  const int i = blk * kST + t;
  const bool valid = i < S;
  const float Ai = valid ? a.A[i] : 0.f;
  const float T2i = (HAS_T2 && valid) ? a.T2[i] : 0.f;
  float mn, mx;
  amin_amax(a, mn, mx);
  K2_WG(1);
  const float den = Dt<DT>::rnd(mx - mn), eps = Dt<DT>::rnd(1e-8f);
  // ---- phase 1: this thread's token: score, class
  float s = 0.f;
  int l = 0;
  if (valid) {
    s = token_score<DT, HAS_T2>(a, i, Ai, T2i, mn, den, eps);
    l = class_of(s, a.p);
    st_sc1(a.scores + i, s);
    a.labels[i] = (uint8_t)l;
  }
  // ---- the class counts, published straight from registers (the quotas need nothing else)
  const uint64_t b0 = __ballot(valid && l == 0), b1 = __ballot(valid && l == 1), b2 = __ballot(valid && l == 2);
  if (lane == 0) { s_c[0][wid] = __popcll(b0); s_c[1][wid] = __popcll(b1); s_c[2][wid] = __popcll(b2); }
  __syncthreads();
  if (wid == 0) {
    const int src = lane & (kSW - 1);
    uint32_t c0 = s_c[0][src], c1 = s_c[1][src], c2 = s_c[2][src];
#pragma unroll
    for (int o = kSW / 2; o > 0; o >>= 1) {
      c0 += __shfl_xor(c0, o, kWave);
      c1 += __shfl_xor(c1, o, kWave);
      c2 += __shfl_xor(c2, o, kWave);
    }
    if (lane == 0) st_sc1(&g.L.head->part[blk], kTag | (uint64_t)c0 | ((uint64_t)c1 << 11) | ((uint64_t)c2 << 22));
  }
  K2_WG(2);
  // ---- histogram bin of the token: the (returning) atomics go out now, the workgroup partials below
  // are reduced while they are in flight, and the slots are taken after
  const bool hist = a.mode_select == 1;  // wave-uniform: every lane takes part in the peer matching
  const int hb = l * kNBin + bin_of(s, bin_lo_of(g, l), bin_inv_of(g, l));
  const int hb3 = 3 * kNBin + bin_of(s, g.bin_lo[3], g.bin_inv[3]);
  HistTicket tk0{0u, 0, 0}, tk3{0u, 0, 0};
  if (hist) {
    tk0 = hist_issue(&g.L.hist[hb], (uint32_t)hb, valid);
    if (g.hist_fb) tk3 = hist_issue(&g.L.hist[hb3], (uint32_t)hb3, valid);
  }
  // ---- workgroup partials: score sum, score key range
  const double sw = wave_sum(valid ? (double)s : 0.0);
  uint32_t kmn = valid ? score_key(s) : 0xffffffffu, kmx = valid ? score_key(s) : 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    kmn = min(kmn, (uint32_t)__shfl_xor((int)kmn, o, kWave));
    kmx = max(kmx, (uint32_t)__shfl_xor((int)kmx, o, kWave));
  }
  if (lane == 0) { s_c[3][wid] = kmn; s_c[4][wid] = kmx; s_sum[wid] = sw; }
  __syncthreads();
  if (wid == 0) {
    const int src = lane & (kSW - 1);
    uint32_t m0 = s_c[3][src], m1 = s_c[4][src];
    double ss = s_sum[src];
#pragma unroll
    for (int o = kSW / 2; o > 0; o >>= 1) {
      m0 = min(m0, (uint32_t)__shfl_xor((int)m0, o, kWave));
      m1 = max(m1, (uint32_t)__shfl_xor((int)m1, o, kWave));
      ss += __shfl_xor(ss, o, kWave);
    }
    if (lane == 0) {  // tagged words: phase 2 takes them without waiting for this workgroup's drain
      const uint64_t sb = __builtin_bit_cast(uint64_t, ss);
      uint64_t* w = g.L.head->pst[blk];
      st_sc1(w + 0, (uint64_t)(kTag | (sb & 0xffffffffull)));
      st_sc1(w + 1, (uint64_t)(kTag | (sb >> 32)));
      st_sc1(w + 2, (uint64_t)(kTag | (uint64_t)m0));
      st_sc1(w + 3, (uint64_t)(kTag | (uint64_t)m1));
    }
  }
  K2_WG(3);
  if (hist) {  // the slot of the token in its bin's list (stored now; awaited only if a class is partly kept)
    const uint64_t entry = ((uint64_t)score_key(s) << 32) | (uint32_t)i;
    const uint32_t slot = hist_slot_of(tk0);
    if (valid && slot < kCap) st_sc1(g.L.slots + (size_t)hb * kCap + slot, entry);
    if (g.hist_fb) {
      const uint32_t slot3 = hist_slot_of(tk3);
      if (valid && slot3 < kCap) st_sc1(g.L.slots + (size_t)hb3 * kCap + slot3, entry);
    }
  }
  K2_WG(4);
  // ---- phase 2a: the quotas and the statistics (every workgroup's counts and partials)
  select_quotas<TPT>(g, sh, blk == G - 1);
  if (sh.partly) {  // (workgroup-uniform) the threshold search reads every workgroup's histogram and slots
    // ---- this workgroup's histogram atomics and slot entries are complete
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // (RTKV_TEST_WITHHOLD_SELECTION: the last workgroup never reports ready, so every workgroup's wait in
    // phase 2b runs into its poll bound)
    if (t == 0 && !(g.withhold == 1 && blk == G - 1)) st_sc1(&g.L.head->ready[blk], kTag);
  }
  // ---- phase 2b in EVERY workgroup (the same inputs, the same deterministic result): no selection hand-off
  // between workgroups
  select_thresholds<TPT>(g, hist_lds, s_selw, sh);
  __syncthreads();
  K2_WG(5);
  compact_phase(g, s, l, i, valid, s_selw);
  K2_WG(8);
}

// ------------------------------------------------------------------------------------ quantization only
// RTKV_NO_SELECTION (BASELINE config 2: the quantizer alone, dynamic_quantization.py:128-196, every token
// kept): no thresholds, no ranking.  Kept row = token index, so the only exchange between workgroups is
// the exclusive prefix of packed row bytes, which follows from the predecessors' class counts — published
// straight from registers right after the scores (one tagged word per workgroup, one look-back round
// trip).  The last workgroup also gathers every workgroup's partials (score sum, range and Σ(s - mean_j)^2,
// combined exactly in double: M2 = Σ M2_j + n_j·(mean_j − mean)^2) for the layer statistics and the
// early host mirror.  Chain: min/max partials → scores → counts word → look-back → stores (about three
// round trips, against the selection kernel's seven).
template <bool HAS_T2, int DT>
__global__ __launch_bounds__(kST) void fsel_quant_kernel(FastArgs g) {
  const FinalizeArgs& a = g.f;
  __shared__ uint32_t s_f3[3][kSW];
  __shared__ double s_d[kSW];
  __shared__ uint32_t s_k[2][kSW];
  __shared__ uint64_t s_base;
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const int S = (int)a.S;
  const int G = (S + kST - 1) / kST;
  const int blk = blockIdx.x;
  const int i = blk * kST + t;
  const bool valid = i < S;
  const float Ai = valid ? a.A[i] : 0.f;
  const float T2i = (HAS_T2 && valid) ? a.T2[i] : 0.f;
  float mn, mx;
  amin_amax(a, mn, mx);
  const float den = Dt<DT>::rnd(mx - mn), eps = Dt<DT>::rnd(1e-8f);
  float s = 0.f;
  int l = 0;
  if (valid) {
    s = token_score<DT, HAS_T2>(a, i, Ai, T2i, mn, den, eps);
    l = class_of(s, a.p);
  }
  // ---- per-class ranks in token order and the workgroup's class counts, published at once
  bool f3[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) f3[c] = valid & (l == c);
  uint32_t r3[3], t3[3];
  block_flag_ranks<3>(f3, r3, t3, s_f3);
  if (t == 0) st_sc1(&g.L.head->part[blk], kTag | (uint64_t)t3[0] | ((uint64_t)t3[1] << 11) | ((uint64_t)t3[2] << 22));
  // ---- the predecessors' counts (wave 0) while the others store the per-token outputs
  if (wid == 0) {
    const uint64_t w = poll_tagged(g.L.head->part, 1, blk, g.spin_limit, a.stats);
    const uint64_t ps = wave_sum(lane < blk ? from11w(w & ~kTag) : 0ull);
    if (lane == 0) s_base = ps;
  }
  if (valid) {
    a.scores[i] = s;
    a.labels[i] = (uint8_t)l;
    a.mask[i] = 1;
    if (i < a.row_capacity) {
      a.kept_index[i] = i;
      if (a.row_label) a.row_label[i] = (uint8_t)l;
    }
  }
  // ---- workgroup partials: score sum and key range, then Σ (s - workgroup mean)^2
  const int nb = min(kST, S - blk * kST);
  {
    const double sw = wave_sum(valid ? (double)s : 0.0);
    uint32_t kmn = valid ? score_key(s) : 0xffffffffu, kmx = valid ? score_key(s) : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      kmn = min(kmn, (uint32_t)__shfl_xor((int)kmn, o, kWave));
      kmx = max(kmx, (uint32_t)__shfl_xor((int)kmx, o, kWave));
    }
    if (lane == 0) { s_d[wid] = sw; s_k[0][wid] = kmn; s_k[1][wid] = kmx; }
  }
  __syncthreads();
  double bsum = s_d[lane & (kSW - 1)];
  uint32_t bmn = s_k[0][lane & (kSW - 1)], bmx = s_k[1][lane & (kSW - 1)];
#pragma unroll
  for (int o = kSW / 2; o > 0; o >>= 1) {
    bsum += __shfl_xor(bsum, o, kWave);
    bmn = min(bmn, (uint32_t)__shfl_xor((int)bmn, o, kWave));
    bmx = max(bmx, (uint32_t)__shfl_xor((int)bmx, o, kWave));
  }
  const double bmean = bsum / (double)nb;
  const double dl = (double)s - bmean;
  const double m2w = wave_sum(valid ? dl * dl : 0.0);
  int64_t rb[3];  // (s_base: wave 0's look-back, published by the barrier above)
#pragma unroll
  for (int q = 0; q < 3; ++q) rb[q] = row_bytes(a, q);
  __syncthreads();
  if (lane == 0) s_d[wid] = m2w;
  if (valid && a.row_offset && i < a.row_capacity)
    a.row_offset[i] = ((int64_t)r3[0] + fldw(s_base, 0)) * rb[0] + ((int64_t)r3[1] + fldw(s_base, 1)) * rb[1] +
                      ((int64_t)r3[2] + fldw(s_base, 2)) * rb[2];
  if (a.shard_ranges) {  // rtkv_shard_ranges in this launch: every token is kept, so rank j's first row is j·S_local
    const int64_t Sl = a.shard_S_local;
    for (int end = 0; end < 2; ++end) {  // (thread 0 of the last workgroup may write both entries)
      if (end ? !(blk == G - 1 && t == 0) : !(valid && (int64_t)i % Sl == 0)) continue;
      int64_t nb = 0;
#pragma unroll
      for (int q = 0; q < 3; ++q) nb += ((int64_t)fldw(s_base, q) + (end ? t3[q] : r3[q])) * rb[q];
      const int64_t j = end ? (int64_t)a.shard_nranks : (int64_t)i / Sl;
      a.shard_ranges[2 * j] = end ? (int64_t)S : (int64_t)i;
      a.shard_ranges[2 * j + 1] = a.row_offset ? nb : 0;
    }
  }
  __syncthreads();
  if (wid == 0) {
    double m2 = s_d[lane & (kSW - 1)];
#pragma unroll
    for (int o = kSW / 2; o > 0; o >>= 1) m2 += __shfl_xor(m2, o, kWave);
    if (lane == 0) {
      FastPartial* pp = g.L.part + blk;
      st_sc1(&pp->ssum, bsum);
      st_sc1(&pp->m2, m2);
      st_sc1(&pp->kmn, bmn);
      st_sc1(&pp->kmx, bmx);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st_sc1(&g.L.head->ready[blk], kTag);
    }
  }
  if (blk != G - 1 || wid != 0) return;
  // ---- the last workgroup: every workgroup's counts and partials → the layer statistics
  const uint64_t wc = poll_tagged(g.L.head->part, 1, G, g.spin_limit, a.stats);
  const uint64_t cnt = wave_sum(lane < G ? from11w(wc & ~kTag) : 0ull);
  (void)poll_tagged(g.L.head->ready, 1, G, g.spin_limit, a.stats);
  double ps = 0.0, pm2 = 0.0;
  uint32_t pmn = 0xffffffffu, pmx = 0u;
  int nj = 0;
  if (lane < G) {
    const FastPartial* pp = g.L.part + lane;
    ps = ld_sc1(&pp->ssum);
    pm2 = ld_sc1(&pp->m2);
    pmn = ld_sc1(&pp->kmn);
    pmx = ld_sc1(&pp->kmx);
    nj = min(kST, S - lane * kST);
  }
  double ssum = ps;
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    ssum += __shfl_xor(ssum, o, kWave);
    pmn = min(pmn, (uint32_t)__shfl_xor((int)pmn, o, kWave));
    pmx = max(pmx, (uint32_t)__shfl_xor((int)pmx, o, kWave));
  }
  const double mean = ssum / (double)S;
  const double dj = nj ? ps / (double)nj - mean : 0.0;
  const double M2 = wave_sum(lane < G ? pm2 + (double)nj * dj * dj : 0.0);
  __shared__ uint64_t s_line[16];
  if (lane == 0) {
    rtkv_layer_stats* hs = a.stats;
    rtkv_batch_stats* bs = reinterpret_cast<rtkv_batch_stats*>(hs + 1);
    const int64_t ccount[3] = {(int64_t)fldw(cnt, 0), (int64_t)fldw(cnt, 1), (int64_t)fldw(cnt, 2)};
    publish_stats(g, false, ssum, pmn, pmx, ccount, ccount, s_line);
    hs->score_m2 = M2;
    bs->kept_score_sum = ssum;
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  if (g.early) host_line_store(reinterpret_cast<uint64_t*>(g.early), s_line);
}

template <int TPT, bool HAS_T2, int DT>
__global__ __launch_bounds__(kST) void fsel_kernel(FastArgs g) {
  extern __shared__ uint32_t hist_lds[];   // [kGrp][kNBin] (the rescan path's rounds)
  k2_body<TPT, HAS_T2, DT>(g, hist_lds);
}

}  // namespace

}  // namespace rtkv
