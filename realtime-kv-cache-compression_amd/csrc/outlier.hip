// outlier.hip — extension "rtkv-gq/1": per-channel outlier detection and per-head group-wise 2/4/8-bit
// pack of a compressed layer's kept K/V rows, its unpack, and decode attention over it.
//
// NO REFERENCE COUNTERPART.  The reference quantizes each token with ONE (scale, zero_point) over all H·D
// channels (src/compression/dynamic_quantization.py:181-194); BASELINE.json's north_star asks for
// "per-channel outlier detection and 2/4/8-bit group-wise K/V pack … wavefront shuffle/ballot for outlier
// voting".  This mode is opt-in (rtkv.GroupQuantConfig; default off, so every reference golden is
// untouched) and its parity is UNPINNED: oracle/rtkv_oracle.c (rtkvo_gq_*) defines it and the kernels
// below are checked against that definition byte for byte (tests/test_gpu_gq.py).
//
// The scheme (D = 128: one group per head):
//   1 vote    every vote_stride-th kept row votes, per head, for its n_vote channels of largest |x| (a
//             wave per (sampled row, tensor), a head on each 16-lane DPP row: n_vote rounds of a row maximum
//             over keys unique within the head, four row_ror max steps each; votes to LDS counters, one
//             global atomic per nonzero channel and workgroup at the end).
//   2 select  per (tensor, head) the n_outlier channels with the most votes (at least min_votes): the
//             layer's outlier channels, fixed for every row (KVQuant-style dense-and-sparse split with a
//             per-layer channel list instead of per-row coordinates) — in the vote grid's last workgroup.
//   3 pack    per (kept row, tensor, head): the reference's per-token formulas (dynamic_quantization.py
//             :62-126, each op rounded to the dtype) over the head's non-outlier channels, codes of the
//             row's class width (2/4/8 bits) for every channel (outliers: code 0) in the per-token
//             layout's row slots (the same row_offset table), {scale, zero_point} per head in the
//             dtype, the outlier channels' raw values beside them.  A head's 16 chunks of 8 channels sit
//             on 16 consecutive lanes (a DPP row): one transposed row reduction per 8 chunks leaves each
//             lane one head's statistics, whose parameters it computes once and broadcasts (row_newbcast).
// Bytes per kept row and tensor: F·w/8 codes + 2·H·e meta + H·n_outlier·e raw values.
#include <cstring>

#include "quant_impl.h"

namespace rtkv {

namespace {

constexpr int kGqD = 128;       // head_dim (one group per head)
constexpr int kGqMaxOut = 16;   // outlier slots per head (4-bit slot ids)

struct GqArgs {
  rtkv_kv_desc kv;
  const int32_t* kept_index;    // [cap] token of each kept row (B = 1)
  const uint8_t* labels;        // [S] class of each token
  const rtkv_layer_stats* stats;
  int bits[3];
  int n_out, n_vote, vote_stride, min_votes_pm;
  int64_t row_cap;              // rows the meta/raw buffers (and the grids) cover
  uint32_t* votes;              // [2][F]
  int16_t* idx;                 // [2][H][n_out]
  const int64_t* row_offset;    // [cap]
  uint8_t* codes[2];
  int64_t codes_capacity;
  void* meta;                   // [rows][2][H][2] dtype
  void* raw;                    // [rows][2][H][n_out] dtype
  int which;                    // unpack: tensor
  void* out;                    // unpack: [rows][F] dtype
};

__device__ __forceinline__ int gq_rows(const GqArgs& a) {
  const rtkv_batch_stats* bs = reinterpret_cast<const rtkv_batch_stats*>(a.stats + 1);
  const int64_t n = bs[0].kept;
  return (int)(n < 0 ? 0 : (n < a.row_cap ? n : a.row_cap));
}

// ---- DPP inside a 16-lane row (a head's 16 chunks of one pack chunk index): lane j ↔ j^8 (row_ror:8),
// j ↔ j^7 (row_half_mirror), j ↔ j^2 / j^1 (quad_perm), and lane n broadcast to its row (row_newbcast:n)
constexpr int kDppRor8 = 0x128, kDppHalfMirror = 0x141, kDppXor2 = 0x4E, kDppXor1 = 0xB1, kDppRowBcast = 0x150;
template <int CTL> __device__ __forceinline__ uint32_t dppu(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTL, 0xf, 0xf, false);
}
template <int CTL> __device__ __forceinline__ float dppf(float v) { return __uint_as_float(dppu<CTL>(__float_as_uint(v))); }
// lane 2c of the row to every lane of it (c compile-time after unrolling)
__device__ __forceinline__ uint32_t row_bcast2(uint32_t v, int c) {
  switch (c) {
    case 0: return dppu<kDppRowBcast + 0>(v);
    case 1: return dppu<kDppRowBcast + 2>(v);
    case 2: return dppu<kDppRowBcast + 4>(v);
    case 3: return dppu<kDppRowBcast + 6>(v);
    case 4: return dppu<kDppRowBcast + 8>(v);
    case 5: return dppu<kDppRowBcast + 10>(v);
    case 6: return dppu<kDppRowBcast + 12>(v);
    default: return dppu<kDppRowBcast + 14>(v);
  }
}

// ------------------------------------------------------------------------------------ 2 select
// Per (tensor, head) the n_outlier channels with the most votes (ties: lower channel), at least min_votes each;
// one wave, lane l holding channels 2l, 2l+1.  Run by the vote grid's last workgroup (below), which reads the
// votes with agent-scope loads (the other workgroups' flush atomics are performed at L2).
__device__ __forceinline__ void gq_select_head(const GqArgs& a, int t, int h, int lane, uint32_t v0, uint32_t v1) {
  const int rows = gq_rows(a);
  const int64_t nsamp = (rows + a.vote_stride - 1) / a.vote_stride;
  int64_t mv = (nsamp * a.min_votes_pm + 999) / 1000;
  const uint32_t min_votes = (uint32_t)(mv < 1 ? 1 : mv);
  const int c0 = 2 * lane, c1 = c0 + 1;
  // unique 32-bit keys votes·2^7 + (127 − channel) (votes < 2^25: the host bounds the sampled rows), so the
  // wave maximum is one DPP row reduction plus the four rows' maxima — no 64-bit shuffle butterfly
  uint32_t k0 = v0 >= min_votes ? (v0 << 7) | (127u - (uint32_t)c0) : 0u;
  uint32_t k1 = v1 >= min_votes ? (v1 << 7) | (127u - (uint32_t)c1) : 0u;
  for (int s = 0; s < a.n_out; ++s) {
    uint32_t m = k0 > k1 ? k0 : k1;
    m = max(m, dppu<0x128>(m));  // row_ror:8
    m = max(m, dppu<0x124>(m));  // row_ror:4
    m = max(m, dppu<0x122>(m));  // row_ror:2
    m = max(m, dppu<0x121>(m));  // row_ror:1
    const uint32_t best = max(max((uint32_t)__builtin_amdgcn_readlane((int)m, 0), (uint32_t)__builtin_amdgcn_readlane((int)m, 16)),
                              max((uint32_t)__builtin_amdgcn_readlane((int)m, 32), (uint32_t)__builtin_amdgcn_readlane((int)m, 48)));
    const int c = best ? (int)(127u - (best & 127u)) : -1;
    if (c == c0) k0 = 0u;
    if (c == c1) k1 = 0u;
    if (lane == 0) a.idx[((int64_t)t * a.kv.H + h) * a.n_out + s] = (int16_t)c;
  }
}

// ------------------------------------------------------------------------------------ 1 vote
// A wave per (sampled kept row, tensor), lane l owning 8-element chunks k·64 + l like the pack, so chunk k
// holds heads 4k..4k+3 on the four 16-lane DPP rows, and the row is read with 16-byte coalesced loads.  Per
// head and round: the lane's best untaken element (largest |x| bits + 1, lowest element on ties), the row's
// maximum by four row_ror steps, the lowest lane of the row holding it by a ballot — the oracle's order
// (larger |x|, then lower channel) — and that lane's vote into the workgroup's LDS counters.  The rounds run
// over 8 chunks at a time (a round of every chunk, then the next round), so eight independent DPP / ballot
// chains interleave instead of one chunk's rounds running back to back.  1024-thread workgroups, one per
// CU: the LDS counters are flushed to the layer's counters (one atomic per nonzero channel) once per 16
// waves.
template <int DT, int NCH>
__global__ __launch_bounds__(1024) void gq_vote_rows_kernel(GqArgs a) {
  using S_ = typename Dt<DT>::S;
  constexpr int F = NCH * 512;
  constexpr int kWaves = 16;
  __shared__ uint32_t s_votes[2 * F];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 2 * F; i += blockDim.x) s_votes[i] = 0u;
  __syncthreads();
  const int rows = gq_rows(a);
  const int vs = a.vote_stride;
  const int nsamp = (rows + vs - 1) / vs;
  const int gw = blockIdx.x * kWaves + (threadIdx.x >> 6), nw = gridDim.x * kWaves;
  for (int task = gw; task < 2 * nsamp; task += nw) {
    const int t = task & 1, j = task >> 1;
    const int tok = __builtin_amdgcn_readfirstlane(a.kept_index[j * vs]);
    if ((unsigned)tok >= (unsigned)a.kv.S) continue;
    const S_* src = static_cast<const S_*>(t ? a.kv.v_dev : a.kv.k_dev) + (int64_t)tok * a.kv.stride_s + lane * 8;
    uint32_t* sv = s_votes + t * F + lane * 8;
    // Composite keys, unique within a head: K·2^7 + (15 − lane % 16)·8 + (7 − e), K from |x| (larger |x|, then
    // lower channel: the oracle's order).  Round m's row maximum M_m is then the winner itself, and a lane's
    // candidate for round m + 1 is its largest key below M_m — the smallest (M_m − 1 − key) over its
    // elements, keys at or above M_m wrapping out of range: no taken flags, no arg-max bookkeeping, no ballot
    // (1.5 VALU per element and round instead of 5).  16-bit dtypes: K = |x| bits + 1 (exact, shifted by 16).
    // fp32: K = (|x| bits >> 7) + 1, exact up to buckets of 2^7 ulps; the top-n_vote SET (all that a vote
    // is) can differ from the exact one only when the bucket of the n-th winner also holds the best
    // remaining key, which one more round detects; such a chunk is redone with exact keys (votes are a set,
    // so the order inside it never matters).
    constexpr bool kTrunc = DT == RTKV_F32;
    const uint32_t lp = (15u - (uint32_t)(lane & 15)) << 3;
#pragma unroll
    for (int k0 = 0; k0 < NCH; k0 += 8) {
      constexpr int kG = NCH < 8 ? NCH : 8;
      uint32_t key[kG][8];
#pragma unroll
      for (int i = 0; i < kG; ++i) {
        if (k0 + i < NCH) {
          const Chunk<DT> c = load_chunk_nt<DT>(src + (k0 + i) * 512);
          if constexpr (kTrunc) {
            float x[8];
            chunk_to_f32<DT>(c, x);
#pragma unroll
            for (int e = 0; e < 8; ++e)
              key[i][e] = ((((__float_as_uint(x[e]) & 0x7fffffffu) >> 7) + 1u) << 7) | lp | (7u - (uint32_t)e);
          } else {
            const uint32_t w4[4] = {c.a.x, c.a.y, c.a.z, c.a.w};
#pragma unroll
            for (int e = 0; e < 8; ++e)
              key[i][e] = ((((w4[e >> 1] >> (16 * (e & 1))) & 0x7fffu) + 1u) << 16) | lp | (7u - (uint32_t)e);
          }
        }
      }
      uint32_t bound[kG], won[kG];  // bound: the previous round's winner (exclusive)
#pragma unroll
      for (int i = 0; i < kG; ++i) { bound[i] = ~0u; won[i] = 0u; }
      auto round = [&](int i, bool vote) {  // one round of chunk i: returns the row maximum
        const uint32_t b1 = bound[i] - 1u;
        uint32_t md = ~0u;
#pragma unroll
        for (int e = 0; e < 8; ++e) md = min(md, b1 - key[i][e]);
        const uint32_t c = md <= b1 ? b1 - md : 0u;
        uint32_t M = c;
        M = max(M, dppu<0x128>(M));  // row_ror:8
        M = max(M, dppu<0x124>(M));  // row_ror:4
        M = max(M, dppu<0x122>(M));  // row_ror:2
        M = max(M, dppu<0x121>(M));  // row_ror:1
        if (vote) {
          won[i] |= (c == M && M != 0u) ? 1u << (7u - (M & 7u)) : 0u;
          bound[i] = M != 0u ? M : 1u;  // (no key left in the row: later rounds find none either)
        }
        return M;
      };
      for (int m = 0; m < a.n_vote; ++m) {
#pragma unroll
        for (int i = 0; i < kG; ++i)
          if (k0 + i < NCH) round(i, true);
      }
#pragma unroll
      for (int i = 0; i < kG; ++i) {
        if (k0 + i >= NCH) continue;
        if constexpr (kTrunc) {
          const uint32_t Mn = round(i, false);  // the best key left after the n_vote winners
          const bool amb = Mn != 0u && bound[i] != 1u && (Mn >> 7) == (bound[i] >> 7);
          if (__builtin_amdgcn_ballot_w64(amb)) {  // (rare) redo the chunk with exact |x| keys
            float x[8];
            chunk_to_f32<DT>(load_chunk_nt<DT>(src + (k0 + i) * 512), x);
            uint32_t kx[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) kx[e] = (__float_as_uint(x[e]) & 0x7fffffffu) + 1u;
            won[i] = 0u;
            for (int m = 0; m < a.n_vote; ++m) {
              uint32_t lb = 0u;
              int le = 0;
#pragma unroll
              for (int e = 0; e < 8; ++e)
                if (kx[e] > lb) { lb = kx[e]; le = e; }
              uint32_t M = lb;
              M = max(M, dppu<0x128>(M));
              M = max(M, dppu<0x124>(M));
              M = max(M, dppu<0x122>(M));
              M = max(M, dppu<0x121>(M));
              const uint64_t b = __ballot(lb == M && M != 0u);
              const uint32_t rowbits = (uint32_t)(b >> (lane & 48)) & 0xffffu;
              if ((int)(lane & 15) == __ffs(rowbits) - 1) {  // the row's winner: its element taken
                won[i] |= 1u << le;
#pragma unroll
                for (int e = 0; e < 8; ++e) kx[e] = e == le ? 0u : kx[e];
              }
            }
          }
        }
        for (uint32_t w = won[i]; w; w &= w - 1) atomicAdd(sv + (k0 + i) * 512 + (__ffs(w) - 1), 1u);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * F; i += blockDim.x)
    if (s_votes[i]) atomicAdd(a.votes + i, s_votes[i]);
  // the last workgroup to finish selects the outlier channels (one launch less than a separate select
  // kernel, whose ~5 us were mostly its launch): this workgroup's flush atomics drained (vmcnt: a memory
  // round trip — an agent-scope __threadfence here writes back and invalidates the XCD's L2 and cost
  // ~100 us over the grid), then the done count; the last one reads the votes with agent-scope loads
  __shared__ uint32_t s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(a.votes + 2 * F, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  // (every pair's votes loaded before the first selection: one memory round trip per wave, not one per pair)
  constexpr int kPairs = (2 * 64 + kWaves - 1) / kWaves;  // (tensor, head) pairs per wave, H <= 64
  uint32_t vv[kPairs][2];
  const int np = 2 * (int)a.kv.H;
#pragma unroll
  for (int j = 0; j < kPairs; ++j) {
    const int p = (threadIdx.x >> 6) + j * kWaves;
    if (p < np) {
      const uint32_t* v = a.votes + (int64_t)(p & 1) * a.kv.H * kGqD + (int64_t)(p >> 1) * kGqD + 2 * lane;
      vv[j][0] = ld_sc1(v);
      vv[j][1] = ld_sc1(v + 1);
    }
  }
#pragma unroll
  for (int j = 0; j < kPairs; ++j) {
    const int p = (threadIdx.x >> 6) + j * kWaves;
    if (p < np) gq_select_head(a, p & 1, p >> 1, lane, vv[j][0], vv[j][1]);
  }
}

// ------------------------------------------------------------------------------------ 3 pack / unpack
// The outlier positions of this lane's chunks of tensor t: bit e of mask[k] set when element e of chunk
// k·64 + lane is an outlier channel, its slot in bits [4e, 4e + 4) of slots[k].
// unused[k] (optional): bit s set when outlier slot s of the chunk's head holds no channel.
// idx: the outlier lists [2][H][n_out] (staged in LDS by gq_stage_idx: a wave's NCH·n_out lookups were a
// chain of dependent global loads at the start of every wave).
template <int NCH>
__device__ __forceinline__ void gq_masks(const GqArgs& a, const int16_t* idx, int t, int lane, uint32_t (&mask)[NCH],
                                         uint32_t (&slots)[NCH], uint32_t* unused = nullptr) {
  const int H = (int)a.kv.H;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = k * 64 + lane, h = c >> 4, sub = c & 15;
    uint32_t m = 0, sl = 0, un = 0;
    if (h < H) {
      for (int s = 0; s < a.n_out; ++s) {
        const int ch = idx[(t * H + h) * a.n_out + s];
        if (ch >= 0 && (ch >> 3) == sub) {
          m |= 1u << (ch & 7);
          sl |= (uint32_t)s << (4 * (ch & 7));
        }
        if (ch < 0) un |= 1u << s;
      }
    }
    mask[k] = m;
    slots[k] = sl;
    if (unused) unused[k] = un;
  }
}

template <int DT> __device__ __forceinline__ uint32_t chunk_bits(const Chunk<DT>& c, int e) {
  if constexpr (DT == RTKV_F32) {
    const float v = e == 0 ? c.a.x : e == 1 ? c.a.y : e == 2 ? c.a.z : e == 3 ? c.a.w
                  : e == 4 ? c.b.x : e == 5 ? c.b.y : e == 6 ? c.b.z : c.b.w;
    return __float_as_uint(v);
  } else {
    const uint32_t w = (e >> 1) == 0 ? c.a.x : (e >> 1) == 1 ? c.a.y : (e >> 1) == 2 ? c.a.z : c.a.w;
    return (e & 1) ? (w >> 16) : (w & 0xffffu);
  }
}
template <int DT> __device__ __forceinline__ void store_bits(void* p, int64_t i, uint32_t b) {
  if constexpr (DT == RTKV_F32) static_cast<uint32_t*>(p)[i] = b;
  else static_cast<uint16_t*>(p)[i] = (uint16_t)b;
}
template <int DT> __device__ __forceinline__ uint32_t load_bits(const void* p, int64_t i) {
  if constexpr (DT == RTKV_F32) return static_cast<const uint32_t*>(p)[i];
  else return static_cast<const uint16_t*>(p)[i];
}
template <int DT> __device__ __forceinline__ float bits_f32(uint32_t b) {
  if constexpr (DT == RTKV_F32) return __uint_as_float(b);
  else return Dt<DT>::load((uint16_t)b);
}

// The outlier lists [2][H][n_out] (H <= 64, n_out <= 16) into LDS by the whole workgroup (a barrier).
__device__ __forceinline__ void gq_stage_idx(const GqArgs& a, int16_t* s_idx) {
  const int n = 2 * (int)a.kv.H * a.n_out;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s_idx[i] = a.idx[i];
  __syncthreads();
}

// element u < 4 of a register array by selects (a runtime index into a private array goes to scratch)
template <typename T> __device__ __forceinline__ T pick4(const T (&v)[4], int u) {
  return u == 0 ? v[0] : (u == 1 ? v[1] : (u == 2 ? v[2] : v[3]));
}

// A head's statistics over its non-outlier channels: min, max (NaN ignored, as fminf/fmaxf and the oracle's
// `<` / `>`), and the smallest nonzero |x| as the key 2|x| − 1 (unsigned; zero → ~0u, NaN above every
// number) for the fast-division gate.
struct GqStat { float mn, mx; uint32_t az; };
__device__ __forceinline__ GqStat gq_comb(const GqStat& a, const GqStat& b) {
  return {fminf(a.mn, b.mn), fmaxf(a.mx, b.mx), a.az < b.az ? a.az : b.az};
}
template <int CTL> __device__ __forceinline__ GqStat gq_dpp(const GqStat& s) {
  return {dppf<CTL>(s.mn), dppf<CTL>(s.mx), dppu<CTL>(s.az)};
}
__device__ __forceinline__ GqStat gq_pick(bool c, const GqStat& a, const GqStat& b) {
  return {c ? a.mn : b.mn, c ? a.mx : b.mx, c ? a.az : b.az};
}
__device__ __forceinline__ float gq_anz(uint32_t az) { return az == ~0u ? INFINITY : __uint_as_float((az + 1u) >> 1); }

// Transposed row reduction of 8 chunks' statistics: s[i] holds this lane's statistics of chunk i; on return
// every lane j of a 16-lane row holds the ROW's statistics of chunk (j >> 1) & 7.  Each butterfly step
// halves the chunks a lane carries (it keeps one half, sends the other to its partner): 4 + 2 + 1 + 1 DPP
// operations per statistic instead of 8 chunks × 4 steps, and the row parameters are then computed once per
// lane instead of once per chunk.  The partners (j^8, j^7, j^2, j^1) span all 16 lanes.
__device__ __forceinline__ GqStat gq_row_transpose(GqStat (&s)[8], int lane) {
  const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2;
#pragma unroll
  for (int i = 0; i < 4; ++i) s[i] = gq_comb(gq_pick(b3, s[i + 4], s[i]), gq_dpp<kDppRor8>(gq_pick(b3, s[i], s[i + 4])));
#pragma unroll
  for (int i = 0; i < 2; ++i)
    s[i] = gq_comb(gq_pick(b2, s[i + 2], s[i]), gq_dpp<kDppHalfMirror>(gq_pick(b2, s[i], s[i + 2])));
  s[0] = gq_comb(gq_pick(b1, s[1], s[0]), gq_dpp<kDppXor2>(gq_pick(b1, s[0], s[1])));
  return gq_comb(s[0], gq_dpp<kDppXor1>(s[0]));
}

// The outlier channels of a chunk set to NaN (all-ones bits: a quiet NaN in every dtype), in place: the row
// statistics then ignore them like any NaN, and their codes come out 0 like a NaN element's (the saturating
// conversion of a NaN).  2 VALU per element (fp32) / per pair (16-bit).
template <int DT> __device__ __forceinline__ void gq_nan_outliers(Chunk<DT>& c, uint32_t mk) {
  auto m1 = [&](int e) { return (uint32_t)((int32_t)(mk << (31 - e)) >> 31); };  // v_bfe_i32
  if constexpr (DT == RTKV_F32) {
    c.a.x = __uint_as_float(__float_as_uint(c.a.x) | m1(0)); c.a.y = __uint_as_float(__float_as_uint(c.a.y) | m1(1));
    c.a.z = __uint_as_float(__float_as_uint(c.a.z) | m1(2)); c.a.w = __uint_as_float(__float_as_uint(c.a.w) | m1(3));
    c.b.x = __uint_as_float(__float_as_uint(c.b.x) | m1(4)); c.b.y = __uint_as_float(__float_as_uint(c.b.y) | m1(5));
    c.b.z = __uint_as_float(__float_as_uint(c.b.z) | m1(6)); c.b.w = __uint_as_float(__float_as_uint(c.b.w) | m1(7));
  } else {
    auto m2 = [&](int j) { return (m1(2 * j) & 0xffffu) | (m1(2 * j + 1) & 0xffff0000u); };  // v_bfi_b32
    c.a.x |= m2(0); c.a.y |= m2(1); c.a.z |= m2(2); c.a.w |= m2(3);
  }
}

// This lane's statistics of one (outlier-free) chunk.
template <int DT> __device__ __forceinline__ GqStat gq_chunk_stat(const Chunk<DT>& c) {
  GqStat s{INFINITY, -INFINITY, ~0u};
  if constexpr (DT == RTKV_F16) {  // packed f16 min/max (NaN ignored, as fminf); no |x| gate for fp16
    const _Float16 pinf = (_Float16)INFINITY;
    h2_t mn2 = {pinf, pinf}, mx2 = {-pinf, -pinf};
    const uint32_t w4[4] = {c.a.x, c.a.y, c.a.z, c.a.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mn2 = __builtin_elementwise_min(mn2, as_h2(w4[j]));
      mx2 = __builtin_elementwise_max(mx2, as_h2(w4[j]));
    }
    s.mn = fminf((float)mn2[0], (float)mn2[1]);
    s.mx = fmaxf((float)mx2[0], (float)mx2[1]);
  } else {
    float x[8];
    chunk_to_f32<DT>(c, x);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s.mn = fminf(s.mn, x[e]);
      s.mx = fmaxf(s.mx, x[e]);
      const uint32_t k = (__float_as_uint(x[e]) << 1) - 1u;
      s.az = k < s.az ? k : s.az;
    }
  }
  return s;
}

// Codes of one chunk (outliers already NaN) at width W: clamp(rint(RN(RN(x / s) + zp)), 0, qmax) as in
// dynamic_quantization.py:120-121, in integers — the saturating v_cvt_u32_f32 maps negative values, −0 and
// NaN to 0 (the float clamp's result for them), then a min with qmax.  FAST: the proven quotient from the
// head's reciprocal (quant_impl.h fast_quotient; without its e == 0 guard, which only keeps the sign of a
// zero quotient that no code sees).  fp16 FAST: K4's native packed-f16 form (f16_chunk_codes).
template <int DT, int W, bool FAST>
__device__ __forceinline__ void gq_chunk_codes(const Chunk<DT>& c, float s, float r, float zp, uint32_t qmaxU,
                                               uint8_t* dst) {
  uint32_t q[8];
  if constexpr (DT == RTKV_F16 && FAST) {
    const _Float16 zph = (_Float16)zp;
    const h2_t zp2 = {zph, zph};
    uint32_t dq[4];
    f16_chunk_codes<false>(c.a, s, r, zp2, zp2, (_Float16)(float)qmaxU, q, dq);
  } else {
    float x[8];
    chunk_to_f32<DT>(c, x);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float qd;
      if constexpr (FAST) {
        const float q0 = x[e] * r;
        qd = __builtin_fmaf(__builtin_fmaf(-q0, s, x[e]), r, q0);
      } else {
        qd = x[e] / s;
      }
      const float t = __builtin_rintf(Dt<DT>::rnd(Dt<DT>::rnd(qd) + zp));
      uint32_t u;
      asm("v_cvt_u32_f32 %0, %1" : "=v"(u) : "v"(t));
      q[e] = u < qmaxU ? u : qmaxU;
    }
  }
  pack_store<W>(dst, q, true);
}

// A wave per (kept row, tensor), lane l owning 8-element chunks k·64 + l (16-byte coalesced loads); chunk k
// holds heads 4k..4k+3 on the wave's four 16-lane rows.  Per row: the outlier channels' raw values stored and
// set to NaN; per chunk the lane's statistics; per 8 chunks one transposed row reduction, so lane j of a row
// holds the statistics of chunk 8g + ((j >> 1) & 7) and computes that head's (scale, zero-point, reciprocal)
// once (row_params: the reference's formulas, dynamic_quantization.py:79-93); the parameters go back to every
// lane of the row by row_newbcast; the codes of the row's width (compile-time per row) with the fast quotient
// when every head of the row admits it (wave-uniform), else the IEEE division.
template <int DT, int NCH>
__global__ __launch_bounds__(256, NCH <= 8 ? 4 : 2) void gq_pack_kernel(GqArgs a) {
  using S_ = typename Dt<DT>::S;
  constexpr int NG = (NCH + 7) / 8;  // groups of 8 chunks (one transposed reduction each)
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  const int t = gw & 1;  // this wave's tensor (0 = K, 1 = V): its outlier masks are built once
  const int H = (int)a.kv.H;
  const int rows = gq_rows(a);
  const int cj = (lane >> 1) & 7;  // the chunk (within a group) whose head parameters this lane computes
  // this wave's outlier maps (mask, slots, unused per chunk) in LDS, read per chunk: 3·NCH fewer live VGPRs
  // (the kernel holds a whole fp32 row in registers, 64 VGPRs, at 4 waves per SIMD)
  __shared__ uint32_t s_maps[4][3][NCH][64];
  __shared__ int16_t s_idx[2 * 64 * kGqMaxOut];
  gq_stage_idx(a, s_idx);
  {
    const int wv = threadIdx.x >> 6;
    uint32_t mask[NCH], slots[NCH], unused[NCH];
    gq_masks<NCH>(a, s_idx, t, lane, mask, slots, unused);
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      s_maps[wv][0][k][lane] = mask[k];
      s_maps[wv][1][k][lane] = slots[k];
      s_maps[wv][2][k][lane] = unused[k];
    }
  }
  const uint32_t (*maps)[NCH][64] = s_maps[threadIdx.x >> 6];  // (wave-private: no barrier needed)
  const S_* base = static_cast<const S_*>(t ? a.kv.v_dev : a.kv.k_dev);
  // kT rows per batch: their tokens, then their classes and packed offsets, all in flight together (two
  // round trips per batch instead of two per row), then the rows one by one
  constexpr int kT = 4;
  const int step = nw >> 1;
  for (int r0 = gw >> 1; r0 < rows; r0 += step * kT) {
  int tokv[kT], labv[kT];
  int64_t roffv[kT];
#pragma unroll
  for (int u = 0; u < kT; ++u) {
    const int r = r0 + u * step;
    tokv[u] = r < rows ? a.kept_index[r] : -1;
    roffv[u] = r < rows ? a.row_offset[r] : -1;
  }
#pragma unroll
  for (int u = 0; u < kT; ++u) {  // (wave-uniform values: scalar registers)
    tokv[u] = __builtin_amdgcn_readfirstlane(tokv[u]);
    roffv[u] = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(roffv[u] >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)roffv[u]));
  }
#pragma unroll
  for (int u = 0; u < kT; ++u)
    labv[u] = __builtin_amdgcn_readfirstlane((unsigned)tokv[u] < (unsigned)a.kv.S ? (int)a.labels[tokv[u]] : 0);
  // (a one-row-ahead prefetch of fp16 rows — 126 instead of 94 VGPRs, 4 instead of 5 waves per SIMD —
  // measured 82 against 74 us at cfg3: the occupancy already hides the row loads)
#pragma unroll 1
  for (int u = 0; u < kT; ++u) {
    const int r = r0 + u * step;
    const int tok = pick4(tokv, u);
    if (r >= rows || (unsigned)tok >= (unsigned)a.kv.S) continue;
    const int lab = pick4(labv, u);
    const int bits = a.bits[lab > 2 ? 0 : lab];
    const int64_t roff = pick4(roffv, u);
    if (roff < 0 || roff + (int64_t)H * kGqD * bits / 8 > a.codes_capacity) continue;
    Chunk<DT> rawc[NCH];
    const S_* src_lane = base + (int64_t)tok * a.kv.stride_s + lane * 8;
#pragma unroll
    for (int k = 0; k < NCH; ++k) rawc[k] = load_chunk_nt<DT>(src_lane + k * 512);
    // this row and tensor's first head (32-bit indices: rows·2·H·max(2, n_out) < 2^31); the opaque copy of
    // lane >> 4 keeps the per-chunk head offsets from being hoisted out of the row loop as 64-bit values
    // (register spills)
    const int mrow0 = (r * 2 + t) * H;
    int hrow = lane >> 4;
    asm volatile("" : "+v"(hrow));
    // the outlier channels' raw values, bit for bit; then NaN in their place
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      __builtin_amdgcn_sched_barrier(0);  // one chunk's temporaries live at a time
      const uint32_t mk = maps[0][k][lane];
      if (mk) {
        const uint32_t sk = maps[1][k][lane];
        const int mrow = mrow0 + 4 * k + hrow;
        for (uint32_t m = mk; m; m &= m - 1) {
          const int e = __ffs(m) - 1;
          store_bits<DT>(a.raw, mrow * a.n_out + (int)((sk >> (4 * e)) & 15u), chunk_bits<DT>(rawc[k], e));
        }
      }
      gq_nan_outliers<DT>(rawc[k], mk);
    }
    // head parameters: lane j of a row owns chunk 8g + cj of each group g
    float sc[NG], zp[NG], rc[NG];
    bool fast = true;
    const float qmax = (float)((1u << bits) - 1u);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      GqStat st[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        __builtin_amdgcn_sched_barrier(0);
        st[i] = 8 * g + i < NCH ? gq_chunk_stat<DT>(rawc[8 * g + i]) : GqStat{INFINITY, -INFINITY, ~0u};
      }
      const GqStat hs = gq_row_transpose(st, lane);
      const RowParams rp = row_params<DT>(hs.mn, hs.mx, bits, gq_anz(hs.az));
      sc[g] = rp.scale;
      zp[g] = rp.zp;
      rc[g] = rp.rcp;
      fast = fast && rp.fast && !(hs.mn != hs.mn) && !(hs.mx != hs.mx);
      const int k = 8 * g + cj;
      if (k < NCH) {
        const int mrow = mrow0 + 4 * k + hrow;
        if (!(lane & 1)) {  // {scale, zero_point} of the head, in the dtype, one store
          if constexpr (DT == RTKV_F32)
            *reinterpret_cast<float2*>(static_cast<float*>(a.meta) + mrow * 2) = make_float2(rp.scale, rp.zp);
          else
            *reinterpret_cast<uint32_t*>(static_cast<S_*>(a.meta) + mrow * 2) =
                (uint32_t)Dt<DT>::store(rp.scale) | ((uint32_t)Dt<DT>::store(rp.zp) << 16);
        } else {  // unused outlier slots of the head hold zero
          for (uint32_t m = maps[2][k][lane]; m; m &= m - 1) store_bits<DT>(a.raw, mrow * a.n_out + (__ffs(m) - 1), 0u);
        }
      }
    }
    // the quotient x / scale: the proven fast form where every head of the row admits it (fast_div_ok),
    // else the IEEE division — the same value either way
    const bool all_fast = __builtin_amdgcn_ballot_w64(!fast) == 0ull;
    uint8_t* dst_lane = a.codes[t] + roff;  // (+ lane·W + k·64·W: 32-bit lane offsets, constant chunk offsets)
    const uint32_t qmaxU = (uint32_t)qmax;
    (void)qmaxU;
    auto emit = [&](auto wtag, auto ftag) {
      constexpr int W = decltype(wtag)::value;
      constexpr bool FAST = decltype(ftag)::value;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        __builtin_amdgcn_sched_barrier(0);  // one chunk's temporaries live at a time
        const int g = k / 8, c = k % 8;
        const float s = __uint_as_float(row_bcast2(__float_as_uint(sc[g]), c));
        const float z = __uint_as_float(row_bcast2(__float_as_uint(zp[g]), c));
        const float rr = FAST ? __uint_as_float(row_bcast2(__float_as_uint(rc[g]), c)) : 0.f;
        gq_chunk_codes<DT, W, FAST>(rawc[k], s, rr, z, (uint32_t)((1u << W) - 1u), dst_lane + (uint32_t)(lane * W) + k * 64 * W);
      }
    };
    auto by_fast = [&](auto wtag) {
      if (all_fast) emit(wtag, std::true_type{});
      else emit(wtag, std::false_type{});
    };
    switch (bits) {
      case 2: by_fast(std::integral_constant<int, 2>{}); break;
      case 4: by_fast(std::integral_constant<int, 4>{}); break;
      default: by_fast(std::integral_constant<int, 8>{}); break;
    }
  }
  }
}

// Reconstruct tensor `which`'s dequantized kept rows from the gq format (bit-identical to rtkvo_gq_pack's deq).
template <int DT, int NCH>
__global__ __launch_bounds__(256) void gq_unpack_kernel(GqArgs a) {
  using S_ = typename Dt<DT>::S;
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  const int t = a.which, H = (int)a.kv.H;
  const int64_t F = (int64_t)H * kGqD;
  const int rows = gq_rows(a);
  __shared__ int16_t s_idx[2 * 64 * kGqMaxOut];
  gq_stage_idx(a, s_idx);
  uint32_t mask[NCH], slots[NCH];
  gq_masks<NCH>(a, s_idx, t, lane, mask, slots);
  for (int r = gw; r < rows; r += nw) {
    const int tok = a.kept_index[r];
    if ((unsigned)tok >= (unsigned)a.kv.S) continue;
    const int lab = a.labels[tok];
    const int bits = a.bits[lab > 2 ? 0 : lab];
    const int64_t roff = a.row_offset[r];
    if (roff < 0 || roff + F * bits / 8 > a.codes_capacity) continue;
    const uint8_t* src_row = a.codes[t] + roff;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = k * 64 + lane, h = c >> 4;
      const uint8_t* src = src_row + (int64_t)c * bits;
      uint64_t word = 0;
      if (bits == 2) word = *reinterpret_cast<const uint16_t*>(src);
      else if (bits == 4) word = *reinterpret_cast<const uint32_t*>(src);
      else word = *reinterpret_cast<const uint64_t*>(src);
      const int64_t mrow = ((int64_t)r * 2 + t) * H + h;
      RowParams rp;
      rp.scale = bits_f32<DT>(load_bits<DT>(a.meta, mrow * 2));
      rp.zp = bits_f32<DT>(load_bits<DT>(a.meta, mrow * 2 + 1));
      float d[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float q = (float)(uint32_t)((word >> (e * bits)) & ((1u << bits) - 1u));
        d[e] = dequant<DT>(q, rp);
      }
      Chunk<DT> oc = f32_to_chunk<DT>(d);
      S_* orow = static_cast<S_*>(a.out) + (int64_t)r * F + (int64_t)c * 8;
      *reinterpret_cast<Chunk<DT>*>(orow) = oc;
      for (uint32_t m = mask[k]; m; m &= m - 1) {  // outlier channels: their raw values, bit for bit
        const int e = __ffs(m) - 1;
        const int s = (int)((slots[k] >> (4 * e)) & 15u);
        store_bits<DT>(orow, e, load_bits<DT>(a.raw, mrow * a.n_out + s));
      }
    }
  }
}

// ------------------------------------------------------------------------------------ 4 decode attention
// out[hq] = softmax_j(q[hq]·K'[j, hq/G]·scale)·V'[j, hq/G] over the kept rows, K'/V' decoded from the gq
// format on the fly (the values rtkvo_gq_pack's deq holds).  Flash-decoding split: workgroup (split, kv
// head), a wave walks rows split·4 + wave, step nsplit·4, lane l holding channels 2l, 2l+1 of the head for
// all G query heads; per-wave (m, l, acc) partials, merged by gq_decode_merge_kernel.
constexpr int kGqMaxG = 8;

struct GqDecArgs {
  GqArgs g;
  const void* q;      // [Hq][D] dtype
  int Hq, G;
  float scale;
  float* part;        // [Hq][nwaves][2 + D]
  float* out;         // [Hq][D]
};

template <int DT, int W>
__device__ __forceinline__ void gq_dec_codes(const uint8_t* hrow, int lane, float& q0, float& q1) {
  uint32_t v;
  if constexpr (W == 2) v = (hrow[lane >> 1] >> (4 * (lane & 1))) & 0xfu;
  else if constexpr (W == 4) v = hrow[lane];
  else v = *reinterpret_cast<const uint16_t*>(hrow + 2 * lane);
  q0 = (float)(v & ((1u << W) - 1u));
  q1 = (float)(v >> W);
}

template <int DT>
__global__ __launch_bounds__(256) void gq_decode_kernel(GqDecArgs d) {
  using S_ = typename Dt<DT>::S;
  const GqArgs& a = d.g;
  const int lane = threadIdx.x & 63;
  const int hk = blockIdx.y, H = (int)a.kv.H, G = d.G;
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), nwv = gridDim.x * 4;
  const int rows = gq_rows(a);
  const int c0 = 2 * lane;
  float qv[kGqMaxG][2];
#pragma unroll
  for (int g = 0; g < kGqMaxG; ++g) {
    qv[g][0] = qv[g][1] = 0.f;
    if (g < G) {
      const S_* qp = static_cast<const S_*>(d.q) + (int64_t)(hk * G + g) * kGqD + c0;
      qv[g][0] = Dt<DT>::load(qp[0]);
      qv[g][1] = Dt<DT>::load(qp[1]);
    }
  }
  // outlier slots of this lane's two channels, per tensor (-1: none)
  int sl[2][2] = {{-1, -1}, {-1, -1}};
  for (int t = 0; t < 2; ++t)
    for (int s = 0; s < a.n_out; ++s) {
      const int ch = a.idx[((int64_t)t * H + hk) * a.n_out + s];
      if (ch == c0) sl[t][0] = s;
      if (ch == c0 + 1) sl[t][1] = s;
    }
  float m[kGqMaxG], l[kGqMaxG], acc[kGqMaxG][2];
#pragma unroll
  for (int g = 0; g < kGqMaxG; ++g) { m[g] = -INFINITY; l[g] = 0.f; acc[g][0] = acc[g][1] = 0.f; }
  for (int r = wv; r < rows; r += nwv) {
    const int tok = a.kept_index[r];
    if ((unsigned)tok >= (unsigned)a.kv.S) continue;
    const int lab = a.labels[tok];
    const int bits = a.bits[lab > 2 ? 0 : lab];
    const int64_t roff = a.row_offset[r] + (int64_t)hk * kGqD * bits / 8;
    if (a.row_offset[r] < 0 || roff + kGqD * bits / 8 > a.codes_capacity) continue;
    float kd[2], vd[2];
    for (int t = 0; t < 2; ++t) {
      const uint8_t* hrow = a.codes[t] + roff;
      float q0, q1;
      if (bits == 2) gq_dec_codes<DT, 2>(hrow, lane, q0, q1);
      else if (bits == 4) gq_dec_codes<DT, 4>(hrow, lane, q0, q1);
      else gq_dec_codes<DT, 8>(hrow, lane, q0, q1);
      const int64_t mrow = ((int64_t)r * 2 + t) * H + hk;
      RowParams rp;
      rp.scale = bits_f32<DT>(load_bits<DT>(a.meta, mrow * 2));
      rp.zp = bits_f32<DT>(load_bits<DT>(a.meta, mrow * 2 + 1));
      float x0 = dequant<DT>(q0, rp), x1 = dequant<DT>(q1, rp);
      if (sl[t][0] >= 0) x0 = bits_f32<DT>(load_bits<DT>(a.raw, mrow * a.n_out + sl[t][0]));
      if (sl[t][1] >= 0) x1 = bits_f32<DT>(load_bits<DT>(a.raw, mrow * a.n_out + sl[t][1]));
      (t ? vd : kd)[0] = x0;
      (t ? vd : kd)[1] = x1;
    }
#pragma unroll
    for (int g = 0; g < kGqMaxG; ++g) {
      if (g >= G) break;
      float s = qv[g][0] * kd[0] + qv[g][1] * kd[1];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
      s *= d.scale;
      const float mn = fmaxf(m[g], s);
      const float corr = __expf(m[g] - mn), p = __expf(s - mn);
      l[g] = l[g] * corr + p;
      acc[g][0] = acc[g][0] * corr + p * vd[0];
      acc[g][1] = acc[g][1] * corr + p * vd[1];
      m[g] = mn;
    }
  }
#pragma unroll
  for (int g = 0; g < kGqMaxG; ++g) {
    if (g >= G) break;
    float* p = d.part + ((int64_t)(hk * G + g) * nwv + wv) * (2 + kGqD);
    if (lane == 0) { p[0] = m[g]; p[1] = l[g]; }
    p[2 + c0] = acc[g][0];
    p[2 + c0 + 1] = acc[g][1];
  }
}

__global__ __launch_bounds__(kGqD) void gq_decode_merge_kernel(GqDecArgs d, int nwv) {
  const int hq = blockIdx.x, c = threadIdx.x;
  const float* p = d.part + (int64_t)hq * nwv * (2 + kGqD);
  float M = -INFINITY;
  for (int w = 0; w < nwv; ++w) M = fmaxf(M, p[(int64_t)w * (2 + kGqD)]);
  float L = 0.f, O = 0.f;
  for (int w = 0; w < nwv; ++w) {
    const float* q = p + (int64_t)w * (2 + kGqD);
    if (q[0] == -INFINITY) continue;
    const float f = __expf(q[0] - M);
    L += q[1] * f;
    O += q[2 + c] * f;
  }
  d.out[(int64_t)hq * kGqD + c] = L > 0.f ? O / L : 0.f;
}

constexpr int kGqDecSplit = 64;  // workgroups per kv head (4 waves each)

}  // namespace

// ------------------------------------------------------------------------------------ host
static int gq_check(const rtkv_kv_desc* kv, const int32_t* kept_index, const uint8_t* labels,
                    const rtkv_layer_stats* stats, const rtkv_gq_params* g) {
  RTKV_REQUIRE(kv && kept_index && labels && stats && g, "gq: null argument");
  RTKV_REQUIRE(kv->B == 1, "gq: one batch row (B = 1)");
  RTKV_REQUIRE(kv->D == kGqD, "gq: head_dim 128 (one group per head)");
  RTKV_REQUIRE(kv->stride_h == kv->D, "gq: heads contiguous within a row ([B, S, H*D] layout)");
  RTKV_REQUIRE(kv->H >= 4 && kv->H % 4 == 0 && kv->H <= 64, "gq: H a multiple of 4 up to 64");
  RTKV_REQUIRE(g->n_outlier >= 0 && g->n_outlier <= kGqMaxOut, "gq: n_outlier in [0, 16]");
  RTKV_REQUIRE(g->n_vote >= 1 && g->n_vote <= kGqD && g->vote_stride >= 1 && g->min_votes_pm >= 0,
               "gq: n_vote in [1, 128], vote_stride >= 1, min_votes_pm >= 0");
  const int esz = kv->dtype == RTKV_F32 ? 4 : 2;
  RTKV_REQUIRE(((uintptr_t)kv->k_dev % 16) == 0 && ((uintptr_t)kv->v_dev % 16) == 0 && (kv->stride_s * esz) % 16 == 0,
               "gq: 16-byte aligned rows");
  return RTKV_OK;
}

static GqArgs gq_args(const rtkv_kv_desc* kv, const int32_t* kept_index, const uint8_t* labels,
                      const rtkv_layer_stats* stats, const rtkv_gq_params* g) {
  GqArgs a;
  std::memset(&a, 0, sizeof(a));
  a.kv = *kv;
  a.kept_index = kept_index;
  a.labels = labels;
  a.stats = stats;
  a.n_out = g->n_outlier;
  a.n_vote = g->n_vote;
  a.vote_stride = g->vote_stride;
  a.min_votes_pm = g->min_votes_pm;
  return a;
}

template <int DT> static int launch_gq_pack(const GqArgs& a, unsigned blocks, hipStream_t st) {
  const int nch = (int)(a.kv.H * kGqD / 512);
#define RTKV_GQ(N)                                                                      \
  if (nch == N) {                                                                       \
    hipLaunchKernelGGL((gq_pack_kernel<DT, N>), dim3(blocks), dim3(256), 0, st, a);     \
    RTKV_HIP_CHECK(hipGetLastError());                                                  \
    return RTKV_OK;                                                                     \
  }
  RTKV_GQ(1) RTKV_GQ(2) RTKV_GQ(3) RTKV_GQ(4) RTKV_GQ(5) RTKV_GQ(6) RTKV_GQ(7) RTKV_GQ(8) RTKV_GQ(10) RTKV_GQ(12)
  RTKV_GQ(16)
#undef RTKV_GQ
  set_error("gq: H must be 4..32, 40, 48 or 64");
  return RTKV_ERR_UNSUPPORTED;
}
template <int DT> static int launch_gq_vote(const GqArgs& a, unsigned blocks, hipStream_t st) {
  const int nch = (int)(a.kv.H * kGqD / 512);
#define RTKV_GQ(N)                                                                      \
  if (nch == N) {                                                                       \
    hipLaunchKernelGGL((gq_vote_rows_kernel<DT, N>), dim3(blocks), dim3(1024), 0, st, a); \
    RTKV_HIP_CHECK(hipGetLastError());                                                  \
    return RTKV_OK;                                                                     \
  }
  RTKV_GQ(1) RTKV_GQ(2) RTKV_GQ(3) RTKV_GQ(4) RTKV_GQ(5) RTKV_GQ(6) RTKV_GQ(7) RTKV_GQ(8) RTKV_GQ(10) RTKV_GQ(12)
  RTKV_GQ(16)
#undef RTKV_GQ
  set_error("gq: H must be 4..32, 40, 48 or 64");
  return RTKV_ERR_UNSUPPORTED;
}
template <int DT> static int launch_gq_unpack(const GqArgs& a, unsigned blocks, hipStream_t st) {
  const int nch = (int)(a.kv.H * kGqD / 512);
#define RTKV_GQ(N)                                                                      \
  if (nch == N) {                                                                       \
    hipLaunchKernelGGL((gq_unpack_kernel<DT, N>), dim3(blocks), dim3(256), 0, st, a);   \
    RTKV_HIP_CHECK(hipGetLastError());                                                  \
    return RTKV_OK;                                                                     \
  }
  RTKV_GQ(1) RTKV_GQ(2) RTKV_GQ(3) RTKV_GQ(4) RTKV_GQ(5) RTKV_GQ(6) RTKV_GQ(7) RTKV_GQ(8) RTKV_GQ(10) RTKV_GQ(12)
  RTKV_GQ(16)
#undef RTKV_GQ
  set_error("gq: H must be 4..32, 40, 48 or 64");
  return RTKV_ERR_UNSUPPORTED;
}

}  // namespace rtkv

using namespace rtkv;

extern "C" {

size_t rtkv_gq_workspace_size(int64_t H, int64_t D) { return (size_t)(2 * H * D) * sizeof(uint32_t) + 64; }  // + done count

int rtkv_gq_outlier_channels(const rtkv_kv_desc* kv, const int32_t* kept_index_dev, const uint8_t* labels_dev,
                             const rtkv_layer_stats* stats_dev, const rtkv_gq_params* g, int64_t row_capacity,
                             int16_t* outlier_idx_dev, void* workspace_dev, size_t workspace_bytes, void* stream) {
  int rc = gq_check(kv, kept_index_dev, labels_dev, stats_dev, g);
  if (rc) return rc;
  RTKV_REQUIRE(outlier_idx_dev || g->n_outlier == 0, "gq: null outlier index buffer");
  RTKV_REQUIRE(workspace_dev && workspace_bytes >= rtkv_gq_workspace_size(kv->H, kv->D), "gq: workspace too small");
  RTKV_REQUIRE(row_capacity >= 1 && row_capacity < ((int64_t)1 << 25), "gq: row_capacity in [1, 2^25)");
  if (g->n_outlier == 0) return RTKV_OK;
  hipStream_t st = (hipStream_t)stream;
  GqArgs a = gq_args(kv, kept_index_dev, labels_dev, stats_dev, g);
  a.row_cap = row_capacity;
  a.votes = static_cast<uint32_t*>(workspace_dev);
  a.idx = outlier_idx_dev;
  RTKV_HIP_CHECK(hipMemsetAsync(a.votes, 0, rtkv_gq_workspace_size(kv->H, kv->D), st));
  // (sampled row, tensor) tasks over 1024-thread workgroups, at most one per CU (each flushes its LDS
  // counters once: with 4-wave workgroups, ~900 of them at cfg3, the flush atomics were most of the kernel)
  const int64_t nsamp = (row_capacity + g->vote_stride - 1) / g->vote_stride;
  int64_t blocks = (2 * nsamp + 15) / 16;
  blocks = blocks < 1 ? 1 : (blocks > 256 ? 256 : blocks);
  int rc2 = RTKV_OK;
  switch (kv->dtype) {
    case RTKV_F16: rc2 = launch_gq_vote<RTKV_F16>(a, (unsigned)blocks, st); break;
    case RTKV_BF16: rc2 = launch_gq_vote<RTKV_BF16>(a, (unsigned)blocks, st); break;
    default: rc2 = launch_gq_vote<RTKV_F32>(a, (unsigned)blocks, st); break;
  }
  if (rc2) return rc2;
  return RTKV_OK;
}

int rtkv_gq_pack(const rtkv_kv_desc* kv, const int32_t* kept_index_dev, const uint8_t* labels_dev,
                 const rtkv_layer_stats* stats_dev, const int32_t bits[3], const rtkv_gq_params* g,
                 const int16_t* outlier_idx_dev, const int64_t* row_offset_dev, uint8_t* codes_k_dev,
                 uint8_t* codes_v_dev, int64_t codes_capacity, void* meta_dev, void* raw_dev, int64_t row_capacity,
                 void* stream) {
  int rc = gq_check(kv, kept_index_dev, labels_dev, stats_dev, g);
  if (rc) return rc;
  RTKV_REQUIRE(bits && row_offset_dev && codes_k_dev && codes_v_dev && meta_dev, "gq: null output");
  RTKV_REQUIRE(g->n_outlier == 0 || (outlier_idx_dev && raw_dev), "gq: null outlier index or raw-value buffer");
  for (int c = 0; c < 3; ++c) RTKV_REQUIRE(bits[c] == 2 || bits[c] == 4 || bits[c] == 8, "gq: class widths 2, 4 or 8 bits");
  RTKV_REQUIRE(row_capacity >= 1, "gq: row_capacity >= 1");
  RTKV_REQUIRE(row_capacity * 2 * kv->H * (g->n_outlier > 2 ? g->n_outlier : 2) < ((int64_t)1 << 31),
               "gq: meta / raw-value indices beyond 2^31 elements");
  GqArgs a = gq_args(kv, kept_index_dev, labels_dev, stats_dev, g);
  for (int c = 0; c < 3; ++c) a.bits[c] = bits[c];
  a.row_cap = row_capacity;
  a.idx = const_cast<int16_t*>(outlier_idx_dev);
  a.row_offset = row_offset_dev;
  a.codes[0] = codes_k_dev;
  a.codes[1] = codes_v_dev;
  a.codes_capacity = codes_capacity;
  a.meta = meta_dev;
  a.raw = raw_dev;
  const int64_t tasks = 2 * row_capacity;  // (row, tensor); a wave keeps one tensor's outlier masks
  int64_t blocks = (tasks + 15) / 16;      // ~4 rows per wave
  blocks = blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks);
  hipStream_t st = (hipStream_t)stream;
  switch (kv->dtype) {
    case RTKV_F16: return launch_gq_pack<RTKV_F16>(a, (unsigned)blocks, st);
    case RTKV_BF16: return launch_gq_pack<RTKV_BF16>(a, (unsigned)blocks, st);
    default: return launch_gq_pack<RTKV_F32>(a, (unsigned)blocks, st);
  }
}

int rtkv_gq_unpack(const rtkv_kv_desc* kv, const int32_t* kept_index_dev, const uint8_t* labels_dev,
                   const rtkv_layer_stats* stats_dev, const int32_t bits[3], const rtkv_gq_params* g,
                   const int16_t* outlier_idx_dev, const int64_t* row_offset_dev, const uint8_t* codes_dev,
                   int64_t codes_capacity, const void* meta_dev, const void* raw_dev, int64_t row_capacity, int which,
                   void* out_dev, void* stream) {
  int rc = gq_check(kv, kept_index_dev, labels_dev, stats_dev, g);
  if (rc) return rc;
  RTKV_REQUIRE(bits && row_offset_dev && codes_dev && meta_dev && out_dev, "gq: null argument");
  RTKV_REQUIRE(g->n_outlier == 0 || (outlier_idx_dev && raw_dev), "gq: null outlier index or raw-value buffer");
  RTKV_REQUIRE(which == 0 || which == 1, "gq: which is 0 (K) or 1 (V)");
  RTKV_REQUIRE(((uintptr_t)out_dev % 16) == 0, "gq: 16-byte aligned output");
  for (int c = 0; c < 3; ++c) RTKV_REQUIRE(bits[c] == 2 || bits[c] == 4 || bits[c] == 8, "gq: class widths 2, 4 or 8 bits");
  GqArgs a = gq_args(kv, kept_index_dev, labels_dev, stats_dev, g);
  for (int c = 0; c < 3; ++c) a.bits[c] = bits[c];
  a.row_cap = row_capacity;
  a.idx = const_cast<int16_t*>(outlier_idx_dev);
  a.row_offset = row_offset_dev;
  a.codes[0] = a.codes[1] = const_cast<uint8_t*>(codes_dev);
  a.codes_capacity = codes_capacity;
  a.meta = const_cast<void*>(meta_dev);
  a.raw = const_cast<void*>(raw_dev);
  a.which = which;
  a.out = out_dev;
  int64_t blocks = (row_capacity + 7) / 8;
  blocks = blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks);
  hipStream_t st = (hipStream_t)stream;
  switch (kv->dtype) {
    case RTKV_F16: return launch_gq_unpack<RTKV_F16>(a, (unsigned)blocks, st);
    case RTKV_BF16: return launch_gq_unpack<RTKV_BF16>(a, (unsigned)blocks, st);
    default: return launch_gq_unpack<RTKV_F32>(a, (unsigned)blocks, st);
  }
}

size_t rtkv_gq_decode_workspace_size(int64_t Hq, int64_t Hkv) {
  (void)Hkv;
  return (size_t)Hq * kGqDecSplit * 4 * (2 + kGqD) * sizeof(float);
}

int rtkv_gq_decode_attention(const rtkv_kv_desc* kv, const int32_t* kept_index_dev, const uint8_t* labels_dev,
                             const rtkv_layer_stats* stats_dev, const int32_t bits[3], const rtkv_gq_params* g,
                             const int16_t* outlier_idx_dev, const int64_t* row_offset_dev, const uint8_t* codes_k_dev,
                             const uint8_t* codes_v_dev, int64_t codes_capacity, const void* meta_dev,
                             const void* raw_dev, int64_t row_capacity, const void* q_dev, int64_t Hq, float scale,
                             float* out_dev, void* workspace_dev, size_t workspace_bytes, void* stream) {
  int rc = gq_check(kv, kept_index_dev, labels_dev, stats_dev, g);
  if (rc) return rc;
  RTKV_REQUIRE(bits && row_offset_dev && codes_k_dev && codes_v_dev && meta_dev && q_dev && out_dev, "gq: null argument");
  RTKV_REQUIRE(g->n_outlier == 0 || (outlier_idx_dev && raw_dev), "gq: null outlier index or raw-value buffer");
  RTKV_REQUIRE(Hq >= kv->H && Hq % kv->H == 0 && Hq / kv->H <= kGqMaxG, "gq decode: Hq a multiple of Hkv, G <= 8");
  RTKV_REQUIRE(workspace_dev && workspace_bytes >= rtkv_gq_decode_workspace_size(Hq, kv->H), "gq decode: workspace too small");
  for (int c = 0; c < 3; ++c) RTKV_REQUIRE(bits[c] == 2 || bits[c] == 4 || bits[c] == 8, "gq: class widths 2, 4 or 8 bits");
  GqDecArgs d;
  std::memset(&d, 0, sizeof(d));
  d.g = gq_args(kv, kept_index_dev, labels_dev, stats_dev, g);
  for (int c = 0; c < 3; ++c) d.g.bits[c] = bits[c];
  d.g.row_cap = row_capacity;
  d.g.idx = const_cast<int16_t*>(outlier_idx_dev);
  d.g.row_offset = row_offset_dev;
  d.g.codes[0] = const_cast<uint8_t*>(codes_k_dev);
  d.g.codes[1] = const_cast<uint8_t*>(codes_v_dev);
  d.g.codes_capacity = codes_capacity;
  d.g.meta = const_cast<void*>(meta_dev);
  d.g.raw = const_cast<void*>(raw_dev);
  d.q = q_dev;
  d.Hq = (int)Hq;
  d.G = (int)(Hq / kv->H);
  d.scale = scale;
  d.part = static_cast<float*>(workspace_dev);
  d.out = out_dev;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)kGqDecSplit, (unsigned)kv->H);
  switch (kv->dtype) {
    case RTKV_F16: hipLaunchKernelGGL((gq_decode_kernel<RTKV_F16>), grid, dim3(256), 0, st, d); break;
    case RTKV_BF16: hipLaunchKernelGGL((gq_decode_kernel<RTKV_BF16>), grid, dim3(256), 0, st, d); break;
    default: hipLaunchKernelGGL((gq_decode_kernel<RTKV_F32>), grid, dim3(256), 0, st, d); break;
  }
  RTKV_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(gq_decode_merge_kernel, dim3((unsigned)Hq), dim3(kGqD), 0, st, d, kGqDecSplit * 4);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

}  // extern "C"
