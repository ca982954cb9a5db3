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
//             wave per (sampled row, tensor), a head on each 16-lane DPP row: n_vote rounds of a row
//             arg-max — lane-local best, four row_ror max steps, the lowest lane by ballot — each vote an
//             LDS atomic; one global atomic per channel and workgroup at the end).
//   2 select  per (tensor, head) the n_outlier channels with the most votes (at least min_votes): the
//             layer's outlier channels, fixed for every row (KVQuant-style dense-and-sparse split with a
//             per-layer channel list instead of per-row coordinates).
//   3 pack    per (kept row, tensor, head): the reference's per-token formulas (dynamic_quantization.py
//             :62-126, each op rounded to the dtype) over the head's non-outlier channels, codes of the
//             row's class width (2/4/8 bits) for every channel (outliers: code 0) in the per-token
//             layout's row slots (the same row_offset table), {scale, zero_point} per head in the
//             dtype, the outlier channels' raw values beside them.  A head's 16 chunks of 8 channels sit
//             on 16 consecutive lanes, so its min/max is a 4-step xor butterfly inside a DPP row.
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

// wave-wide maximum of a 64-bit key (two 32-bit butterfly shuffles per step)
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o, kWave);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o, kWave);
    const uint64_t w = ((uint64_t)hi << 32) | lo;
    v = w > v ? w : v;
  }
  return v;
}

// two consecutive elements (2l, 2l+1) of a row as fp32
template <int DT> __device__ __forceinline__ void load2(const typename Dt<DT>::S* p, float& x0, float& x1) {
  if constexpr (DT == RTKV_F32) {
    const float2 v = *reinterpret_cast<const float2*>(p);
    x0 = v.x;
    x1 = v.y;
  } else {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
    x0 = Dt<DT>::load((uint16_t)(w & 0xffffu));
    x1 = Dt<DT>::load((uint16_t)(w >> 16));
  }
}

// ------------------------------------------------------------------------------------ 1 vote
// A wave per (sampled kept row, tensor), lane l owning 8-element chunks
// k·64 + l like the pack, so chunk k holds heads 4k..4k+3 on the four 16-lane DPP rows, and the row is read
// with 16-byte coalesced loads.  Per head and round: the lane's best untaken element (largest |x| bits + 1,
// lowest element on ties), the row's maximum by four row_ror steps, the lowest lane of the row holding it
// by a ballot — the oracle's order (larger |x|, then lower channel) — and that lane's vote into the
// workgroup's LDS counters, flushed to the layer's counters once per workgroup.
template <int DT, int NCH>
__global__ __launch_bounds__(256, 2) void gq_vote_rows_kernel(GqArgs a) {
  using S_ = typename Dt<DT>::S;
  constexpr int F = NCH * 512;
  __shared__ uint32_t s_votes[2 * F];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 2 * F; i += blockDim.x) s_votes[i] = 0u;
  __syncthreads();
  const int rows = gq_rows(a);
  const int vs = a.vote_stride;
  const int nsamp = (rows + vs - 1) / vs;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  for (int task = gw; task < 2 * nsamp; task += nw) {
    const int t = task & 1, j = task >> 1;
    const int tok = __builtin_amdgcn_readfirstlane(a.kept_index[j * vs]);
    if ((unsigned)tok >= (unsigned)a.kv.S) continue;
    const S_* src = static_cast<const S_*>(t ? a.kv.v_dev : a.kv.k_dev) + (int64_t)tok * a.kv.stride_s;
    Chunk<DT> rawc[NCH];
#pragma unroll
    for (int k = 0; k < NCH; ++k) rawc[k] = load_chunk_nt<DT>(src + (k * 64 + lane) * 8);
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      float x[8];
      chunk_to_f32<DT>(rawc[k], x);
      uint32_t key[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) key[e] = (__float_as_uint(x[e]) & 0x7fffffffu) + 1u;
      for (int m = 0; m < a.n_vote; ++m) {
        uint32_t lb = 0u;
        int le = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (key[e] > lb) { lb = key[e]; le = e; }
        uint32_t M = lb;
        M = max(M, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)M, 0x128, 0xf, 0xf, false));  // row_ror:8
        M = max(M, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)M, 0x124, 0xf, 0xf, false));  // row_ror:4
        M = max(M, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)M, 0x122, 0xf, 0xf, false));  // row_ror:2
        M = max(M, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)M, 0x121, 0xf, 0xf, false));  // row_ror:1
        const uint64_t b = __ballot(lb == M);
        const uint32_t rowbits = (uint32_t)(b >> (lane & 48)) & 0xffffu;
        if ((int)(lane & 15) == __ffs(rowbits) - 1) {  // the row's winner: one vote, its element taken
          atomicAdd(&s_votes[t * F + (k * 64 + lane) * 8 + le], 1u);
#pragma unroll
          for (int e = 0; e < 8; ++e) key[e] = e == le ? 0u : key[e];
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * F; i += blockDim.x)
    if (s_votes[i]) atomicAdd(a.votes + i, s_votes[i]);
}

// ------------------------------------------------------------------------------------ 2 select
__global__ __launch_bounds__(64) void gq_select_kernel(GqArgs a) {
  const int lane = threadIdx.x;
  const int h = blockIdx.x, t = blockIdx.y;
  const int rows = gq_rows(a);
  const int64_t nsamp = (rows + a.vote_stride - 1) / a.vote_stride;
  int64_t mv = (nsamp * a.min_votes_pm + 999) / 1000;
  const uint32_t min_votes = (uint32_t)(mv < 1 ? 1 : mv);
  const int c0 = 2 * lane, c1 = c0 + 1;
  const uint32_t* v = a.votes + (int64_t)t * a.kv.H * kGqD + (int64_t)h * kGqD;
  const uint32_t v0 = v[c0], v1 = v[c1];
  uint64_t k0 = v0 >= min_votes ? ((uint64_t)v0 << 32) | (0xffffffffu - (uint32_t)c0) : 0ull;
  uint64_t k1 = v1 >= min_votes ? ((uint64_t)v1 << 32) | (0xffffffffu - (uint32_t)c1) : 0ull;
  for (int s = 0; s < a.n_out; ++s) {
    const uint64_t best = wave_max_u64(k0 > k1 ? k0 : k1);
    const int c = best ? (int)(0xffffffffu - (uint32_t)best) : -1;
    if (c == c0) k0 = 0ull;
    if (c == c1) k1 = 0ull;
    if (lane == 0) a.idx[((int64_t)t * a.kv.H + h) * a.n_out + s] = (int16_t)c;
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

// min / max / min-nonzero-|x| combined with the lane N places round in the same row of 16 (DPP row_ror:N)
template <int N> __device__ __forceinline__ void row16_minmax(float& mn, float& mx, float& anz) {
  constexpr int kCtl = 0x120 + N;  // row_ror:N
  mn = fminf(mn, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(mn), kCtl, 0xf, 0xf, false)));
  mx = fmaxf(mx, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(mx), kCtl, 0xf, 0xf, false)));
  anz = fminf(anz, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(anz), kCtl, 0xf, 0xf, false)));
}

// element u < 4 of a register array by selects (a runtime index into a private array goes to scratch)
template <typename T> __device__ __forceinline__ T pick4(const T (&v)[4], int u) {
  return u == 0 ? v[0] : (u == 1 ? v[1] : (u == 2 ? v[2] : v[3]));
}

template <int DT, int NCH>
__global__ __launch_bounds__(256, NCH <= 8 ? 4 : 2) void gq_pack_kernel(GqArgs a) {
  using S_ = typename Dt<DT>::S;
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  const int t = gw & 1;  // this wave's tensor (0 = K, 1 = V): its outlier masks are built once
  const int H = (int)a.kv.H;
  const int rows = gq_rows(a);
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
#pragma unroll 1
  for (int u = 0; u < kT; ++u) {
    const int r = r0 + u * step;
    const int tok = pick4(tokv, u);
    if (r >= rows || (unsigned)tok >= (unsigned)a.kv.S) continue;
    const int lab = pick4(labv, u);
    const int bits = a.bits[lab > 2 ? 0 : lab];
    const int64_t roff = pick4(roffv, u);
    if (roff < 0 || roff + (int64_t)H * kGqD * bits / 8 > a.codes_capacity) continue;
    const S_* src = base + (int64_t)tok * a.kv.stride_s;
    Chunk<DT> rawc[NCH];
#pragma unroll
    for (int k = 0; k < NCH; ++k) rawc[k] = load_chunk_nt<DT>(src + (k * 64 + lane) * 8);
    uint8_t* dst_row = a.codes[t] + roff;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = k * 64 + lane, h = c >> 4;
      const uint32_t mk = maps[0][k][lane], sk = maps[1][k][lane], uk = maps[2][k][lane];
      float x[8];
      chunk_to_f32<DT>(rawc[k], x);
      float mn = INFINITY, mx = -INFINITY, anz = INFINITY;  // anz: min |x| over the nonzero elements
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (!((mk >> e) & 1u)) {
          mn = fminf(mn, x[e]);
          mx = fmaxf(mx, x[e]);
          if constexpr (DT != RTKV_F16) {  // (fp16's fast quotient needs no lower bound)
            const float ax = __builtin_fabsf(x[e]);
            anz = ax != 0.f ? fminf(anz, ax) : anz;
          }
        }
      // the head's 16 lanes are a DPP row: rotations by 8, 4, 2, 1 within it leave every lane the row's value
      row16_minmax<8>(mn, mx, anz);
      row16_minmax<4>(mn, mx, anz);
      row16_minmax<2>(mn, mx, anz);
      row16_minmax<1>(mn, mx, anz);
      const RowParams rp = row_params<DT>(mn, mx, bits, anz);
      const int64_t mrow = ((int64_t)r * 2 + t) * H + h;
      if ((lane & 15) == 0) {
        static_cast<S_*>(a.meta)[mrow * 2] = Dt<DT>::store(rp.scale);
        static_cast<S_*>(a.meta)[mrow * 2 + 1] = Dt<DT>::store(rp.zp);
        for (uint32_t m = uk; m; m &= m - 1)  // unused outlier slots of the head hold zero
          store_bits<DT>(a.raw, mrow * a.n_out + (__ffs(m) - 1), 0u);
      }
      // the quotient x / scale: the proven fast form where the head's range admits it (fast_div_ok), else
      // the IEEE division — the same value either way (quant_impl.h fast_quotient)
      // (wave-uniform choice: the four heads of the chunk all admit it, as almost every head does)
      const bool fast = __all(rp.fast && !(mn != mn) && !(mx != mx));
      uint32_t q[8];
      if (fast) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool out = ((mk >> e) & 1u) || x[e] != x[e];
          q[e] = out ? 0u : (uint32_t)code_from_quotient<DT>(fast_quotient(x[e], rp.scale, rp.rcp), rp);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool out = ((mk >> e) & 1u) || x[e] != x[e];
          q[e] = out ? 0u : (uint32_t)code_from_quotient<DT>(x[e] / rp.scale, rp);
        }
      }
      uint8_t* dst = dst_row + (int64_t)c * bits;
      switch (bits) {
        case 2: pack_store<2>(dst, q, true); break;
        case 4: pack_store<4>(dst, q, true); break;
        default: pack_store<8>(dst, q, true); break;
      }
      for (uint32_t m = mk; m; m &= m - 1) {  // the outlier channels' raw values
        const int e = __ffs(m) - 1;
        const int s = (int)((sk >> (4 * e)) & 15u);
        store_bits<DT>(a.raw, mrow * a.n_out + s, chunk_bits<DT>(rawc[k], e));
      }
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
    hipLaunchKernelGGL((gq_vote_rows_kernel<DT, N>), dim3(blocks), dim3(256), 0, st, a); \
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

size_t rtkv_gq_workspace_size(int64_t H, int64_t D) { return (size_t)(2 * H * D) * sizeof(uint32_t); }

int rtkv_gq_outlier_channels(const rtkv_kv_desc* kv, const int32_t* kept_index_dev, const uint8_t* labels_dev,
                             const rtkv_layer_stats* stats_dev, const rtkv_gq_params* g, int64_t row_capacity,
                             int16_t* outlier_idx_dev, void* workspace_dev, size_t workspace_bytes, void* stream) {
  int rc = gq_check(kv, kept_index_dev, labels_dev, stats_dev, g);
  if (rc) return rc;
  RTKV_REQUIRE(outlier_idx_dev || g->n_outlier == 0, "gq: null outlier index buffer");
  RTKV_REQUIRE(workspace_dev && workspace_bytes >= rtkv_gq_workspace_size(kv->H, kv->D), "gq: workspace too small");
  RTKV_REQUIRE(row_capacity >= 1, "gq: row_capacity >= 1");
  if (g->n_outlier == 0) return RTKV_OK;
  hipStream_t st = (hipStream_t)stream;
  GqArgs a = gq_args(kv, kept_index_dev, labels_dev, stats_dev, g);
  a.row_cap = row_capacity;
  a.votes = static_cast<uint32_t*>(workspace_dev);
  a.idx = outlier_idx_dev;
  RTKV_HIP_CHECK(hipMemsetAsync(a.votes, 0, rtkv_gq_workspace_size(kv->H, kv->D), st));
  // (sampled row, tensor) tasks over workgroups of 4 waves, ~2 tasks per wave: a wave is a latency chain
  // (one row in flight, then its rounds), so the grid supplies the parallelism (each workgroup flushes
  // its LDS counters once)
  const int64_t nsamp = (row_capacity + g->vote_stride - 1) / g->vote_stride;
  int64_t blocks = (2 * nsamp + 7) / 8;
  blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
  int rc2 = RTKV_OK;
  switch (kv->dtype) {
    case RTKV_F16: rc2 = launch_gq_vote<RTKV_F16>(a, (unsigned)blocks, st); break;
    case RTKV_BF16: rc2 = launch_gq_vote<RTKV_BF16>(a, (unsigned)blocks, st); break;
    default: rc2 = launch_gq_vote<RTKV_F32>(a, (unsigned)blocks, st); break;
  }
  if (rc2) return rc2;
  hipLaunchKernelGGL(gq_select_kernel, dim3((unsigned)kv->H, 2u), dim3(64), 0, st, a);
  RTKV_HIP_CHECK(hipGetLastError());
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
