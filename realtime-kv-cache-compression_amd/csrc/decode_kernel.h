// decode_kernel.h — attention of one new token over a layer's PACKED mixed-precision KV.
//
// Reference: after compression the reference attends over the dequantized floats K', V'
// (modified_llama.py:140-142, 165-166: softmax(q·K'ᵀ/√d)·V' on the kept rows).  Here the keys and
// values are decoded from the packed codes on the fly — every element exactly the dequantized value
// K4 writes (dequant<DT>: (code − zp)·scale, each op rounded to the dtype,
// dynamic_quantization.py:124) — so a decode step reads F·w/8 bytes per kept row and tensor instead
// of F·e: 2/4/8-bit rows move 1/8 .. 1/2 of the fp16 bytes.  Attention arithmetic is fp32.
//
// Work decomposition (flash-decoding): one workgroup of 4 waves per (split s, head group hg, batch
// row b, query-head group gs).  Split s owns a contiguous range of kept rows; wave v takes rows
// r0 + v + 4t.  The row's F = Hkv·D elements are 8-element chunks; head group hg covers chunks
// [hg·64·NCH, (hg+1)·64·NCH) (NCH = 1 or 2) and lane l owns chunks c = (hg·NCH + k)·64 + l, i.e. w
// contiguous code bytes per chunk, so one wave instruction reads 64·w consecutive bytes of the row.
// Per-row metadata (kept index → class → width, byte offset, scale/zero-points) is loaded for 64
// rows at a time, one row per lane, and broadcast with readlane; the rows of one field width are
// then taken together (ballot), so each code load has the width's exact size and 2–8 rows of codes
// stay in flight per wave.  GQ query heads of a kv head (GQA) share every decoded chunk.  The D/8
// lanes of one head reduce q·k with DPP adds; every lane keeps the online-softmax state (m, l) and
// 8 value accumulators per (query head, chunk).  fp16 rows are dequantized with packed half2
// arithmetic (bit-identical: each op of dequant<F16> is one rounded fp16 op), bf16 rows with
// v_cvt_pk_bf16_f32 roundings and v_dot2_f32_bf16.  The 4 waves merge in LDS; a second kernel
// merges the splits.
#pragma once

#include "common.h"
#include "quant_impl.h"

#include <cstdlib>
#include <cstring>

namespace rtkv {

struct DecodeArgs {
  const uint8_t* codes_k;
  const uint8_t* codes_v;
  int64_t codes_bytes;        // size of each code buffer
  const int64_t* row_offset;  // [B, cap]
  const float* scale_zp;      // [B, cap, 4]
  const int32_t* kept_index;  // [B, cap]
  const uint8_t* labels;      // [B, S]
  const int64_t* rows;        // [B]
  int64_t S, cap;
  int Hkv, D, G;              // G = Hq / Hkv
  int HG;                     // head groups: F / (512·NCH)
  int GS;                     // query-head groups: G / GQ
  int nrest;                  // splits · HG · B
  int w[3];                   // field width of each class
  const void* q;              // [B, Hq, D] (dtype)
  float scale;
  int splits;
  float* part_m;              // [B][G][splits][Hkv]
  float* part_l;
  float* part_acc;            // [B][G][splits][F]
  float* out;                 // [B, Hq, D] fp32
};

// launches decode_split_kernel<RTKV_F16, …> (decode_f16.hip, its own flags)
int launch_decode_split_f16(const DecodeArgs& a, int nch, int gq, int D, dim3 grid, size_t lds, hipStream_t st);

namespace {


constexpr int kDW = 4;  // waves per workgroup
constexpr float kSlack = 8.f;  // lazy rescale: running max may trail the row max by up to 2^8


using H2 = __attribute__((ext_vector_type(2))) _Float16;
using B2 = __attribute__((ext_vector_type(2))) __bf16;

// bf16: two fp32 values rounded to bf16 (v_cvt_pk_bf16_f32, round to nearest even: Dt<BF16>::rnd
// for finite values) and back
__device__ __forceinline__ B2 rnd_bf2(float a, float b) { return B2{(__bf16)a, (__bf16)b}; }
__device__ __forceinline__ float bf_lo(B2 v) { return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, v) << 16); }
__device__ __forceinline__ float bf_hi(B2 v) { return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, v) & 0xffff0000u); }
// dequant<BF16> of a pair of codes: rnd(rnd(c − zp)·scale), each op rounded to bf16
__device__ __forceinline__ B2 dequant_bf2(float c0, float c1, const RowParams& rp) {
  const B2 d = rnd_bf2(c0 - rp.zp, c1 - rp.zp);
  return rnd_bf2(bf_lo(d) * rp.scale, bf_hi(d) * rp.scale);
}

// Slot order of a chunk's 8 elements in registers.  fp16 works on element pairs (p, p + 4) — the
// pairing the packed code layouts give with one shift per pair — so slot 2p holds element p and
// slot 2p + 1 element p + 4; the other dtypes keep element order.
template <int DT> __device__ __forceinline__ constexpr int slot_elem(int sl) {
  if constexpr (DT == RTKV_F16) return (sl & 1) ? (sl >> 1) + 4 : (sl >> 1);
  else return sl;
}

// The W code bytes of one chunk (W = field width in bits = bytes per 8 elements), as loaded.
template <int W> struct ChunkCodes { uint32_t r[W >= 4 ? W / 4 : 1]; };

template <int W>
__device__ __forceinline__ ChunkCodes<W> load_codes(__amdgpu_buffer_rsrc_t rs, int off) {
  ChunkCodes<W> c;
  if constexpr (W == 2) {
    c.r[0] = __builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 0);
  } else if constexpr (W == 4) {
    c.r[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
  } else if constexpr (W == 8) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
    c.r[0] = v[0]; c.r[1] = v[1];
  } else {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    c.r[0] = v[0]; c.r[1] = v[1]; c.r[2] = v[2]; c.r[3] = v[3];
  }
  return c;
}

// the 8 codes of a chunk as floats in element order
template <int W>
__device__ __forceinline__ void unpack8(const ChunkCodes<W>& x, float (&c)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    uint32_t v;
    if constexpr (W == 16) v = (x.r[e >> 1] >> (16 * (e & 1))) & 0xffffu;
    else if constexpr (W == 8) v = (x.r[e >> 2] >> (8 * (e & 3))) & 0xffu;
    else v = (x.r[0] >> (W * e)) & ((1u << W) - 1u);
    c[e] = (float)v;
  }
}

// fp16: the codes of element pairs (p, p + 4) as exact half2 integers.  For W <= 8 each code lands
// in the mantissa of 1024 (0x6400 | c = 1024 + c, exact), and 1024 is subtracted exactly.
template <int W>
__device__ __forceinline__ void codes_h2(const ChunkCodes<W>& x, H2 (&c)[4]) {
  if constexpr (W == 16) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const uint32_t lo = (x.r[p >> 1] >> (16 * (p & 1))) & 0xffffu, hi = (x.r[2 + (p >> 1)] >> (16 * (p & 1))) & 0xffffu;
      c[p] = H2{(_Float16)lo, (_Float16)hi};  // stored codes are fp16 values (K4 rounds them so)
    }
  } else {
    uint32_t u[4];
    if constexpr (W == 8) {
#pragma unroll
      for (int p = 0; p < 4; ++p)  // byte p of r0 → bits 0..7, byte p of r1 → bits 16..23
        u[p] = __builtin_amdgcn_perm(x.r[1], x.r[0], 0x0c000c00u | (uint32_t)p | ((uint32_t)(4 + p) << 16));
    } else {
      // W = 4 / 2: (y >> W·p) & mask | 0x6400 in one v_and_or_b32 per pair (the compiler emits and + or).
      // VOP3 takes no literal and one SGPR: the mask in a VGPR, the 0x6400 pair in an SGPR
      const uint32_t y = W == 4 ? x.r[0] : __builtin_amdgcn_perm(0u, x.r[0], 0x0c010c00u);  // W = 2: byte 1 → bits 16..23
      const uint32_t msk = W == 4 ? 0x000f000fu : 0x00030003u, one = 0x64006400u;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        uint32_t r;
        asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(y >> (W * p)), "v"(msk), "s"(one));
        u[p] = r;
      }
      const H2 k1024 = {(_Float16)1024.f, (_Float16)1024.f};
#pragma unroll
      for (int p = 0; p < 4; ++p) c[p] = __builtin_bit_cast(H2, u[p]) - k1024;
      return;
    }
    const H2 k1024 = {(_Float16)1024.f, (_Float16)1024.f};
#pragma unroll
    for (int p = 0; p < 4; ++p) c[p] = __builtin_bit_cast(H2, u[p] | 0x64006400u) - k1024;
  }
}

template <int CTRL> __device__ __forceinline__ float dpp_add(float v) {
  return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// sum over aligned groups of lph lanes (lph = D/8, a power of two ≤ 64), result in every lane;
// LPH > 0 fixes lph at compile time (no branches), LPH = 0 reads it at run time
template <int LPH>
__device__ __forceinline__ float group_sum(float v, int lph_rt) {
  const int lph = LPH > 0 ? LPH : lph_rt;
  if (lph >= 2) v = dpp_add<0xB1>(v);    // quad_perm [1,0,3,2]
  if (lph >= 4) v = dpp_add<0x4E>(v);    // quad_perm [2,3,0,1]
  if (lph >= 8) v = dpp_add<0x141>(v);   // row_half_mirror: lane i <-> 7-i within 8
  if (lph >= 16) v = dpp_add<0x140>(v);  // row_mirror: lane i <-> 15-i within 16
  if (lph >= 32) v += __shfl_xor(v, 16, kWave);
  if (lph >= 64) v += __shfl_xor(v, 32, kWave);
  return v;
}

__device__ __forceinline__ float lane_f(float v, int t) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), t));
}

// One workgroup per (split s, head group hg, batch row b) × query-head group gs (GQ query heads of
// each kv head), ids arranged so the GS workgroups that read the same rows share id mod 8, i.e.
// one XCD and its L2.
template <int DT, int NCH, int GQ, int LPH>
__global__ __launch_bounds__(64 * kDW) void decode_split_kernel(DecodeArgs a) {
  using S_ = typename Dt<DT>::S;
  constexpr bool kH = DT == RTKV_F16;
  constexpr bool kB = DT == RTKV_BF16;
  constexpr int kU = GQ * NCH;    // (query head, chunk) units per lane
  extern __shared__ float lds[];  // [kDW][64][kU][10]: m, l, acc[8] per unit
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int id = blockIdx.x, hi = id >> 3;
  const int gs = hi % a.GS;
  const int rest = (id & 7) + 8 * (hi / a.GS);
  if (rest >= a.nrest) return;
  const int s = rest % a.splits, t1 = rest / a.splits, hg = t1 % a.HG, b = t1 / a.HG;
  const int F = a.HG * NCH * 512, D = a.D, lph = D / 8;  // lanes per head within one chunk column
  const int c0 = hg * NCH * 64;                            // first chunk of this head group
  const int64_t nrows = a.rows[b] < a.cap ? (a.rows[b] > 0 ? a.rows[b] : 0) : a.cap;
  const int64_t per = (nrows + a.splits - 1) / a.splits;
  const int64_t r0 = (int64_t)s * per, r1 = r0 + per < nrows ? r0 + per : nrows;
  const int Hq = a.Hkv * a.G;
  // q (fp16: half2 pairs in slot order; otherwise fp32), accumulators in slot order, m / l
  H2 qh[GQ][NCH][4];
  B2 qb[GQ][NCH][4];
  float qf[GQ][NCH][8], acc[GQ][NCH][8], m[GQ][NCH], l[GQ][NCH];
#pragma unroll
  for (int j = 0; j < GQ; ++j) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int f0 = (c0 + k * 64 + lane) * 8, hk = f0 / D, d0 = f0 - hk * D;
      const int g = gs * GQ + j;
      const S_* qp = static_cast<const S_*>(a.q) + ((int64_t)b * Hq + (int64_t)hk * a.G + g) * D + d0;
      const Chunk<DT> qc = *reinterpret_cast<const Chunk<DT>*>(qp);
      if constexpr (kH) {
        const uint32_t w4[4] = {qc.a.x, qc.a.y, qc.a.z, qc.a.w};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const uint32_t lo = (w4[p >> 1] >> (16 * (p & 1))) & 0xffffu, hi2 = (w4[2 + (p >> 1)] >> (16 * (p & 1))) & 0xffffu;
          qh[j][k][p] = __builtin_bit_cast(H2, lo | (hi2 << 16));
        }
      } else if constexpr (kB) {
        const uint32_t w4[4] = {qc.a.x, qc.a.y, qc.a.z, qc.a.w};
#pragma unroll
        for (int p = 0; p < 4; ++p) qb[j][k][p] = __builtin_bit_cast(B2, w4[p]);  // elements (2p, 2p+1)
      } else {
        chunk_to_f32<DT>(qc, qf[j][k]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[j][k][e] = 0.f;
      m[j][k] = -INFINITY;
      l[j][k] = 0.f;
    }
  }
  const float qscale = a.scale;  // 1/sqrt(D) · log2(e): scores in the exp2 domain
  // one row of the chunk columns this lane owns: K' → dots → online softmax → V' → accumulators
  auto row = [&](auto wtag, const ChunkCodes<decltype(wtag)::value> (&xk)[NCH],
                 const ChunkCodes<decltype(wtag)::value> (&xv)[NCH], const RowParams& rk, const RowParams& rv,
                 H2 zsk, H2 zsv) {  // fp16: {zp, scale} of K and V as halves (the other dtypes use rk / rv)
    constexpr int W = decltype(wtag)::value;
    float sc[NCH][GQ];
    // K' of each chunk (exactly dequant<DT>: each op rounded to the dtype) and the dots
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      if constexpr (kH) {
        const H2 zp2 = __builtin_shufflevector(zsk, zsk, 0, 0), sc2 = __builtin_shufflevector(zsk, zsk, 1, 1);
        H2 kh[4];
        codes_h2<W>(xk[k], kh);
#pragma unroll
        for (int p = 0; p < 4; ++p) kh[p] = (kh[p] - zp2) * sc2;
#pragma unroll
        for (int j = 0; j < GQ; ++j) {
          float d = 0.f;
#pragma unroll
          for (int p = 0; p < 4; ++p) d = __builtin_amdgcn_fdot2(qh[j][k][p], kh[p], d, false);
          sc[k][j] = d;
        }
      } else if constexpr (kB) {
        float kc[8];
        unpack8<W>(xk[k], kc);
        B2 kb[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) kb[p] = dequant_bf2(kc[2 * p], kc[2 * p + 1], rk);
#pragma unroll
        for (int j = 0; j < GQ; ++j) {
          float d = 0.f;
#pragma unroll
          for (int p = 0; p < 4; ++p) d = __builtin_amdgcn_fdot2_f32_bf16(qb[j][k][p], kb[p], d, false);
          sc[k][j] = d;
        }
      } else {
        float kf[8];
        unpack8<W>(xk[k], kf);
#pragma unroll
        for (int e = 0; e < 8; ++e) kf[e] = dequant<DT>(kf[e], rk);
#pragma unroll
        for (int j = 0; j < GQ; ++j) {
          float d = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) d = __builtin_fmaf(qf[j][k][e], kf[e], d);
          sc[k][j] = d;
        }
      }
    }
    // head sums (independent DPP chains side by side), scores in the exp2 domain
    bool up = false;
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
      for (int j = 0; j < GQ; ++j) {
        sc[k][j] = group_sum<LPH>(sc[k][j], lph) * qscale;
        up |= sc[k][j] > m[j][k] + kSlack;
      }
    // online softmax with a lazily raised reference m: rescale only when a score passes m + kSlack
    // (one wave-uniform branch per row, rare after the first rows); weights stay ≤ 2^kSlack
    if (__ballot(up)) {
#pragma unroll
      for (int k = 0; k < NCH; ++k)
#pragma unroll
        for (int j = 0; j < GQ; ++j) {
          const float mn = sc[k][j] > m[j][k] + kSlack ? sc[k][j] : m[j][k];
          const float cr = __builtin_amdgcn_exp2f(m[j][k] - mn);
          l[j][k] *= cr;
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[j][k][e] *= cr;
          m[j][k] = mn;
        }
    }
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      float pw[GQ];
#pragma unroll
      for (int j = 0; j < GQ; ++j) {
        pw[j] = __builtin_amdgcn_exp2f(sc[k][j] - m[j][k]);
        l[j][k] += pw[j];
      }
      // V' and the accumulators
      if constexpr (kH) {
        const H2 zp2 = __builtin_shufflevector(zsv, zsv, 0, 0), sc2 = __builtin_shufflevector(zsv, zsv, 1, 1);
        H2 vh[4];
        codes_h2<W>(xv[k], vh);
#pragma unroll
        for (int p = 0; p < 4; ++p) vh[p] = (vh[p] - zp2) * sc2;
#pragma unroll
        for (int j = 0; j < GQ; ++j) {
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            acc[j][k][2 * p] = __builtin_fmaf(pw[j], (float)vh[p].x, acc[j][k][2 * p]);
            acc[j][k][2 * p + 1] = __builtin_fmaf(pw[j], (float)vh[p].y, acc[j][k][2 * p + 1]);
          }
        }
      } else if constexpr (kB) {
        float vc[8];
        unpack8<W>(xv[k], vc);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const B2 vb = dequant_bf2(vc[2 * p], vc[2 * p + 1], rv);
          const float v0 = bf_lo(vb), v1 = bf_hi(vb);
#pragma unroll
          for (int j = 0; j < GQ; ++j) {
            acc[j][k][2 * p] = __builtin_fmaf(pw[j], v0, acc[j][k][2 * p]);
            acc[j][k][2 * p + 1] = __builtin_fmaf(pw[j], v1, acc[j][k][2 * p + 1]);
          }
        }
      } else {
        float vf[8];
        unpack8<W>(xv[k], vf);
#pragma unroll
        for (int e = 0; e < 8; ++e) vf[e] = dequant<DT>(vf[e], rv);
#pragma unroll
        for (int j = 0; j < GQ; ++j) {
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[j][k][e] = __builtin_fmaf(pw[j], vf[e], acc[j][k][e]);
        }
      }
    }
  };
  // Rows of this wave: r0 + wave + kDW·t.  Metadata of 64 rows at a time, one row per lane; the
  // rows of each field width are then taken together (ballot), so the code loads have the width's
  // exact size (W bytes per chunk) and PD rows of them are kept in flight.
  // A row's width comes from its byte span: rows are back to back, so row_offset[r + 1] − row_offset[r]
  // = F·W/8 — two independent loads instead of kept_index → labels (two dependent round trips); only
  // the row list's last row (no successor) takes its class.  A span that matches no width (corrupt
  // metadata) leaves the row out.  The next 64 rows' metadata is in flight while this batch's rows are
  // processed.
  const int64_t bcap = (int64_t)b * a.cap;
  auto meta = [&](int64_t jb, int64_t& off, int64_t& offn, float4& sz) {
    const int64_t jr = jb + (int64_t)kDW * lane;
    const bool ok = jr < r1, nx = jr + 1 < nrows;
    const int64_t rj = bcap + (ok ? jr : jb);
    off = a.row_offset[rj];
    offn = (ok && nx) ? a.row_offset[rj + 1] : -1;
    sz = *reinterpret_cast<const float4*>(a.scale_zp + rj * 4);
  };
  int64_t m_off = 0, m_offn = -1;
  float4 m_sz = make_float4(0.f, 0.f, 0.f, 0.f);
  if (r0 + wave < r1) meta(r0 + wave, m_off, m_offn, m_sz);
  for (int64_t jb = r0 + wave; jb < r1; jb += 64 * kDW) {
    const int64_t jr = jb + (int64_t)kDW * lane;
    const bool ok = jr < r1;
    const int64_t off = m_off;
    const float4 sz = m_sz;
    int wl = 0;
    {
      const int64_t span = m_offn - off;  // F·W/8 for a consistent row
      const int fb8 = F / 8;
#pragma unroll
      for (int c = 0; c < 3; ++c)
        if (span == (int64_t)fb8 * a.w[c]) wl = a.w[c];
      const bool lastrow = ok && jr + 1 == nrows;
      if (__ballot(lastrow)) {  // the list's last row: its class (kept index → label)
        const int ki0 = a.kept_index[bcap + (lastrow ? jr : jb)];
        const int ki = ki0 < 0 ? 0 : (ki0 >= a.S ? (int)a.S - 1 : ki0);
        const int lab = a.labels[(int64_t)b * a.S + ki];
        if (lastrow) wl = lab == 2 ? a.w[2] : (lab == 1 ? a.w[1] : a.w[0]);
      }
    }
    if (jb + 64 * kDW < r1) meta(jb + 64 * kDW, m_off, m_offn, m_sz);  // the next batch, in flight meanwhile
    const uint32_t off_lo = (uint32_t)off, off_hi = (uint32_t)(off >> 32);
    // fp16: {zp, scale} of K and V as half pairs (exact: K4 stores fp16-representable values)
    const uint32_t zs_k = kH ? __builtin_bit_cast(uint32_t, H2{(_Float16)sz.y, (_Float16)sz.x}) : 0u;
    const uint32_t zs_v = kH ? __builtin_bit_cast(uint32_t, H2{(_Float16)sz.w, (_Float16)sz.z}) : 0u;
    auto by_width = [&](auto wtag) {
      constexpr int W = decltype(wtag)::value;
      constexpr int PD = W <= 4 ? 8 : (W == 8 ? 4 : 2);  // rows in flight (≤ 32 VGPRs of codes at NCH 2)
      uint64_t mask = __ballot(ok && wl == W);
      const int n = __builtin_popcountll(mask);
      if (n == 0) return;
      int last = 0;
      auto next = [&]() {  // lane index of the next row of this width (the last one again at the end)
        if (mask) {
          last = __builtin_ctzll(mask);
          mask &= mask - 1;
        }
        return last;
      };
      // codes of row t through descriptors bounded to the row's F·W/8 bytes
      auto issue = [&](int t, ChunkCodes<W> (&xk)[NCH], ChunkCodes<W> (&xv)[NCH]) {
        const int64_t o = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)off_hi, t) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane((int)off_lo, t));
        const int64_t nbr = (int64_t)(F / 8) * W;
        const int nb = (o >= 0 && o + nbr <= a.codes_bytes) ? (int)nbr : 0;  // out of range: zero codes
        const auto sk = __builtin_amdgcn_make_buffer_rsrc((void*)(a.codes_k + o), (short)0, nb, 0x00020000);
        const auto sv = __builtin_amdgcn_make_buffer_rsrc((void*)(a.codes_v + o), (short)0, nb, 0x00020000);
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
          const int vo = (c0 + k * 64 + lane) * W;
          xk[k] = load_codes<W>(sk, vo);
          xv[k] = load_codes<W>(sv, vo);
        }
      };
      ChunkCodes<W> bk[PD][NCH], bv[PD][NCH];
      int tl[PD];
#pragma unroll
      for (int i = 0; i < PD; ++i) {
        tl[i] = next();
        issue(tl[i], bk[i], bv[i]);
      }
      auto compute = [&](int i) {
        const int t = tl[i];
        RowParams rk, rv;
        H2 zk = {}, zv = {};
        if constexpr (kH) {  // the halves were packed once per 64-row batch: two readlanes per row
          zk = __builtin_bit_cast(H2, __builtin_amdgcn_readlane((int)zs_k, t));
          zv = __builtin_bit_cast(H2, __builtin_amdgcn_readlane((int)zs_v, t));
        } else {
          rk.scale = lane_f(sz.x, t); rk.zp = lane_f(sz.y, t);
          rv.scale = lane_f(sz.z, t); rv.zp = lane_f(sz.w, t);
        }
        row(wtag, bk[i], bv[i], rk, rv, zk, zv);
      };
      int base = 0;
      for (; base + PD <= n; base += PD) {  // full rounds: straight-line, each slot refilled
#pragma unroll
        for (int i = 0; i < PD; ++i) {
          compute(i);
          tl[i] = next();
          issue(tl[i], bk[i], bv[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < PD; ++i)  // the rest (< PD rows), already loaded
        if (base + i < n) compute(i);
    };
    by_width(std::integral_constant<int, 2>{});
    by_width(std::integral_constant<int, 4>{});
    by_width(std::integral_constant<int, 8>{});
    by_width(std::integral_constant<int, 16>{});
  }
  // ---- merge the kDW waves in LDS, then write this split's partial
  float* mine = lds + ((size_t)wave * 64 + lane) * kU * 10;
#pragma unroll
  for (int j = 0; j < GQ; ++j) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      float* u = mine + (j * NCH + k) * 10;
      u[0] = m[j][k];
      u[1] = l[j][k];
#pragma unroll
      for (int e = 0; e < 8; ++e) u[2 + e] = acc[j][k][e];
    }
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int j = 0; j < GQ; ++j) {
    const int g = gs * GQ + j;
    const int64_t pbase = ((int64_t)b * a.G + g) * a.splits + s;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int un = j * NCH + k;
      float mm = -INFINITY;
      for (int v = 0; v < kDW; ++v) mm = fmaxf(mm, lds[(((size_t)v * 64 + lane) * kU + un) * 10]);
      float ll = 0.f, aa[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int v = 0; v < kDW; ++v) {
        const float* src = lds + (((size_t)v * 64 + lane) * kU + un) * 10;
        const float f = src[0] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(src[0] - mm);
        ll += f * src[1];
#pragma unroll
        for (int e = 0; e < 8; ++e) aa[e] += f * src[2 + e];
      }
      const int f0 = (c0 + k * 64 + lane) * 8, hk = f0 / D;
      if ((lane % lph) == 0) {
        a.part_m[pbase * a.Hkv + hk] = mm;
        a.part_l[pbase * a.Hkv + hk] = ll;
      }
      float* pa = a.part_acc + pbase * F + f0;
#pragma unroll
      for (int sl = 0; sl < 8; ++sl) pa[slot_elem<DT>(sl)] = aa[sl];
    }
  }
}

// the split kernel of one dtype for the lane shape (NCH chunks, GQ query heads) and head_dim
template <int DT>
int launch_decode_split(const DecodeArgs& a, int nch, int gq, int D, dim3 grid, size_t lds, hipStream_t st) {
#define RTKV_D(N, Q)                                                                                  \
  if (nch == N && gq == Q) {                                                                          \
    if (D == 128)                                                                                     \
      hipLaunchKernelGGL((decode_split_kernel<DT, N, Q, 16>), grid, dim3(64 * kDW), lds, st, a);     \
    else                                                                                              \
      hipLaunchKernelGGL((decode_split_kernel<DT, N, Q, 0>), grid, dim3(64 * kDW), lds, st, a);      \
    RTKV_HIP_CHECK(hipGetLastError());                                                                \
    return RTKV_OK;                                                                                   \
  }
  RTKV_D(1, 1) RTKV_D(2, 1) RTKV_D(1, 2) RTKV_D(1, 4)
#undef RTKV_D
  RTKV_REQUIRE(false, "decode: unsupported lane shape");
}

}  // namespace
}  // namespace rtkv
