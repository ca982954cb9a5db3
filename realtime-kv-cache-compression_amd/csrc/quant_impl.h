// quant_impl.h — K4: per-token asymmetric min-max quantization + bit-pack + ordered compaction, plus
// the unpack (consumer) kernel and the whole-tensor quantization helpers.
//
// Reference: DynamicPrecisionQuantizer.get_quantization_params / quantize_tensor /
// apply_mixed_precision_quantization (dynamic_quantization.py:62-196) followed by the gather of
// SelectiveTokenPropagator.apply_token_selection (selective_propagation.py:214-232).  The reference
// fake-quantizes EVERY token with ~12 tiny torch ops and then gathers the kept rows; here each kept
// row is read from HBM once, quantized in registers and written once (dequantized row in the output
// position + packed codes), and dropped rows are never read.
//
// Work decomposition: one wave64 per (kept row, tensor).  Lane l owns 8-element chunks
// c = k*64 + l (k < NCH), so every wave-instruction moves 64 × 16 B = 1 KiB of one row (fp32: two
// such loads).  Row min/max → wave shuffle reduction; the per-element ops are fp32 ops rounded to
// the dtype after each op (bit-identical to PyTorch CPU).  8 codes of w bits pack into exactly w
// bytes, so each lane writes its chunk's codes with one store at byte offset c*w.
#pragma once
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace rtkv {

template <int DT> struct Chunk;  // 8 elements of storage
template <> struct Chunk<RTKV_F32> { float4 a, b; };
template <> struct Chunk<RTKV_F16> { uint4 a; };
template <> struct Chunk<RTKV_BF16> { uint4 a; };

template <int DT> __device__ __forceinline__ void chunk_to_f32(const Chunk<DT>& c, float (&x)[8]) {
  if constexpr (DT == RTKV_F32) {
    x[0] = c.a.x; x[1] = c.a.y; x[2] = c.a.z; x[3] = c.a.w;
    x[4] = c.b.x; x[5] = c.b.y; x[6] = c.b.z; x[7] = c.b.w;
  } else {
    const uint32_t w[4] = {c.a.x, c.a.y, c.a.z, c.a.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x[2 * k] = Dt<DT>::load((uint16_t)(w[k] & 0xffffu));
      x[2 * k + 1] = Dt<DT>::load((uint16_t)(w[k] >> 16));
    }
  }
}
template <int DT> __device__ __forceinline__ Chunk<DT> f32_to_chunk(const float (&x)[8]) {
  Chunk<DT> c;
  if constexpr (DT == RTKV_F32) {
    c.a = make_float4(x[0], x[1], x[2], x[3]);
    c.b = make_float4(x[4], x[5], x[6], x[7]);
  } else {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      w[k] = (uint32_t)Dt<DT>::store(x[2 * k]) | ((uint32_t)Dt<DT>::store(x[2 * k + 1]) << 16);
    c.a = make_uint4(w[0], w[1], w[2], w[3]);
  }
  return c;
}

// Streaming (non-temporal) store of a chunk: the outputs are not re-read by this layer, so they
// bypass cache allocation instead of evicting the next kernel's inputs.
typedef unsigned int nt_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int nt_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void nt_store16(void* dst, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  // (write-through sc1 stores instead: K4 170 -> 186 us, and the K4 -> K1 gap unchanged;
  // profiles/r04l_k4_sc1_ab.json)
  __builtin_nontemporal_store(nt_u32x4{a, b, c, d}, reinterpret_cast<nt_u32x4*>(dst));
}
template <int DT> __device__ __forceinline__ void store_chunk_nt(Chunk<DT>* dst, const Chunk<DT>& c) {
  if constexpr (DT == RTKV_F32) {
    nt_store16(&dst->a, __float_as_uint(c.a.x), __float_as_uint(c.a.y), __float_as_uint(c.a.z), __float_as_uint(c.a.w));
    nt_store16(&dst->b, __float_as_uint(c.b.x), __float_as_uint(c.b.y), __float_as_uint(c.b.z), __float_as_uint(c.b.w));
  } else {
    nt_store16(&dst->a, c.a.x, c.a.y, c.a.z, c.a.w);
  }
}

template <int DT> __device__ __forceinline__ Chunk<DT> load_chunk_nt(const typename Dt<DT>::S* p) {
  Chunk<DT> c;
  if constexpr (DT == RTKV_F32) {
    const uint4 a = load16_nt(p), b = load16_nt(p + 4);
    c.a = make_float4(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z), __uint_as_float(a.w));
    c.b = make_float4(__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z), __uint_as_float(b.w));
  } else {
    c.a = load16_nt(p);
  }
  return c;
}

// Little-endian accumulation of 8 codes of w bits (w <= 17) into 3 × 64-bit words.
__device__ __forceinline__ void pack8(const uint32_t (&q)[8], int w, uint64_t& p0, uint64_t& p1, uint64_t& p2) {
  p0 = p1 = p2 = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int bit = e * w;
    const uint64_t v = q[e];
    const int word = bit >> 6, sh = bit & 63;
    const uint64_t lo = v << sh;
    const uint64_t hi = sh ? (v >> (64 - sh)) : 0ull;
    if (word == 0) { p0 |= lo; p1 |= hi; }
    else if (word == 1) { p1 |= lo; p2 |= hi; }
    else { p2 |= lo; }
  }
}

__device__ __forceinline__ void store_bytes(uint8_t* dst, int nbytes, uint64_t p0, uint64_t p1, uint64_t p2) {
  const uintptr_t addr = (uintptr_t)dst;
  if (nbytes == 16 && (addr & 15) == 0) {
    *reinterpret_cast<uint4*>(dst) = make_uint4((uint32_t)p0, (uint32_t)(p0 >> 32), (uint32_t)p1, (uint32_t)(p1 >> 32));
  } else if (nbytes == 8 && (addr & 7) == 0) {
    *reinterpret_cast<uint2*>(dst) = make_uint2((uint32_t)p0, (uint32_t)(p0 >> 32));
  } else if (nbytes == 4 && (addr & 3) == 0) {
    *reinterpret_cast<uint32_t*>(dst) = (uint32_t)p0;
  } else if (nbytes == 2 && (addr & 1) == 0) {
    *reinterpret_cast<uint16_t*>(dst) = (uint16_t)p0;
  } else {
    for (int k = 0; k < nbytes; ++k) {
      const uint64_t word = k < 8 ? p0 : (k < 16 ? p1 : p2);
      dst[k] = (uint8_t)(word >> ((k & 7) * 8));
    }  // (scalar tail path: non-multiple-of-8 rows and unusual widths only)
  }
}

struct RowParams {
  float scale, zp, qmaxT;
  float rcp;  // 1 / scale (IEEE), used by the fast quotient when `fast`
  bool fast;  // fast_div_ok for this row (row-uniform)
};

// Quotient x / s, bit-identical to the IEEE fp32 division, from the row reciprocal r = RN(1/s):
// q0 = RN(x·r), exact residual e = x − q0·s (one FMA), one Markstein correction RN(q0 + e·r); the
// e == 0 case keeps q0 (then q0 = x/s exactly, and the sign of a zero quotient is preserved).
// Proven by exhaustive enumeration of the admitted (x, s) pairs (rtkv_selfcheck_division, run by
// tests/test_gpu_parity.py):
//   fp16: every finite x and every positive finite s;
//   bf16: 2^-62 <= s <= 2^62, |x| <= 2^62, and x == 0 or |x| >= 2^-48·s (tiny quotients below
//         ~2^-57 are where the correction step can be off; the row gate excludes them).
//   fp32: 2^-100 <= s <= 2^100, |x| <= 2^100·s, and x == 0 or |x| >= max(2^-60, 2^-100·s).  Then
//         1/s, x·r, the residual and the quotient are all normal numbers, so every step commutes
//         with scaling x and s by powers of two, and the pair reduces to its mantissas
//         (X, S) in [1, 2)^2: all 2^46 of them are enumerated (rtkv_selfcheck_division_f32).
// amax = max |x| over the row, amin_nz = min |x| over the nonzero elements (bf16 and fp32).
template <int DT> __device__ __forceinline__ bool fast_div_ok(float s, float amax, float amin_nz) {
  if constexpr (DT == RTKV_F16) return s > 0.f && s < INFINITY;  // false for NaN
  else if constexpr (DT == RTKV_BF16)
    return s >= 0x1p-62f && s <= 0x1p62f && amax <= 0x1p62f && amin_nz >= s * 0x1p-48f;
  else
    return s >= 0x1p-100f && s <= 0x1p100f && amax <= s * 0x1p100f && amin_nz >= 0x1p-60f &&
           amin_nz >= s * 0x1p-100f;
}
__device__ __forceinline__ float fast_quotient(float x, float s, float r) {
  const float q0 = x * r;
  const float e = __builtin_fmaf(-q0, s, x);
  return e == 0.f ? q0 : __builtin_fmaf(e, r, q0);
}

template <int DT>
__device__ __forceinline__ RowParams row_params(float mn, float mx, int bits, float amin_nz = INFINITY) {
  // dynamic_quantization.py:79-93 (each op rounded to the dtype)
  RowParams r;
  const float qmax = (float)((1u << bits) - 1u);
  r.qmaxT = Dt<DT>::rnd(qmax);  // clamp bound as converted by torch.clamp (:121)
  if (mx == mn) {
    r.scale = 1.f;
    r.zp = 0.f;
  } else {
    r.scale = Dt<DT>::rnd(Dt<DT>::rnd(mx - mn) / qmax);
    r.zp = Dt<DT>::rnd(0.f - Dt<DT>::rnd(mn / r.scale));
  }
  r.rcp = 1.f / r.scale;
  r.fast = fast_div_ok<DT>(r.scale, fmaxf(__builtin_fabsf(mn), __builtin_fabsf(mx)), amin_nz);
  return r;
}

// Code from the quotient: dynamic_quantization.py:120-121
template <int DT> __device__ __forceinline__ float code_from_quotient(float qd, const RowParams& rp) {
  const float t = Dt<DT>::rnd(Dt<DT>::rnd(qd) + rp.zp);
  float q = __builtin_rintf(t);  // rint of a dtype value is a dtype value: no rounding needed
  q = q < 0.f ? 0.f : q;
  q = q > rp.qmaxT ? rp.qmaxT : q;
  return q;
}
template <int DT> __device__ __forceinline__ float quant_code(float x, const RowParams& rp) {
  return code_from_quotient<DT>(x / rp.scale, rp);
}
template <int DT> __device__ __forceinline__ float dequant(float q, const RowParams& rp) {
  return Dt<DT>::rnd(Dt<DT>::rnd(q - rp.zp) * rp.scale);  // :124
}

// ------------------------------------------------------------------------------------ fp16 rows
// After the fp32 quotient, every step of an fp16 row is a native f16 op on pairs (v_pk_add_f16,
// v_pk_mul_f16, v_pk_max/min_f16): RN16(a ∘ b) of f16 operands equals RN16(RN32(a ∘ b)), the fp32 op
// rounded to fp16 that torch performs on the CPU — double rounding through a format of p' >= 2p + 2
// bits is innocuous for + − × ÷ (Figueroa 1995; 24 >= 2·11 + 2).  The quotient itself stays the
// proven fp32 fast quotient, rounded once to f16 (RN16(RN32(x / s)) = RN16(x / s) by the same rule).
typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h2_t as_h2(uint32_t w) { return __builtin_bit_cast(h2_t, w); }
__device__ __forceinline__ uint32_t h2_bits(h2_t v) { return __builtin_bit_cast(uint32_t, v); }

// Codes (and, with DEQ, the dequantized f16 pair words) of one 8-element f16 chunk of a row without
// NaN.  DEQ keeps torch.clamp's compare-select (the sign of a zero code reaches the dequantized
// value); codes alone take the packed max/min (equal codes: a zero is code 0 either way).
template <bool DEQ>
__device__ __forceinline__ void f16_chunk_codes(const uint4 raw, float s, float r, h2_t zp2, h2_t s2, _Float16 qmax,
                                                uint32_t (&qi)[8], uint32_t (&dq)[4]) {
  const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
  const h2_t zero2 = {(_Float16)0.f, (_Float16)0.f}, qmax2 = {qmax, qmax};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const h2_t xh = as_h2(w[k]);
    float q[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float x = (float)xh[j];
      const float q0 = x * r;
      const float e = __builtin_fmaf(-q0, s, x);
      // without DEQ the e == 0 guard (which only keeps the sign of a zero quotient) is moot
      float qq = DEQ ? (e == 0.f ? q0 : __builtin_fmaf(e, r, q0)) : __builtin_fmaf(e, r, q0);
      asm volatile("" : "+v"(qq));  // the fp32 quotient, then its f16 rounding (no v_fma_mix)
      q[j] = qq;
    }
    const h2_t qh = {(_Float16)q[0], (_Float16)q[1]};
    const h2_t t = __builtin_elementwise_roundeven(qh + zp2);  // dynamic_quantization.py:120
    h2_t c;
    if constexpr (DEQ) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        _Float16 v = t[j] < (_Float16)0.f ? (_Float16)0.f : t[j];  // :121
        c[j] = v > qmax ? qmax : v;
      }
      dq[k] = h2_bits((c - zp2) * s2);  // :124
    } else {
      c = __builtin_elementwise_min(__builtin_elementwise_max(t, zero2), qmax2);
    }
    qi[2 * k] = (uint32_t)c[0];
    qi[2 * k + 1] = (uint32_t)c[1];
  }
}

// ------------------------------------------------------------------------------------ K4
// Pack 8 codes of W bits (compile-time W in {2,4,8,16}) and store them at dst (W bytes).
template <int W> __device__ __forceinline__ void pack_store(uint8_t* dst, const uint32_t (&q)[8], bool aligned) {
  if constexpr (W == 2) {
    uint32_t v = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) v |= q[e] << (2 * e);
    if (aligned) __builtin_nontemporal_store((uint16_t)v, reinterpret_cast<uint16_t*>(dst));
    else { dst[0] = (uint8_t)v; dst[1] = (uint8_t)(v >> 8); }
  } else if constexpr (W == 4) {
    uint32_t v = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) v |= q[e] << (4 * e);
    if (aligned) __builtin_nontemporal_store(v, reinterpret_cast<uint32_t*>(dst));
    else {
#pragma unroll
      for (int k = 0; k < 4; ++k) dst[k] = (uint8_t)(v >> (8 * k));
    }
  } else if constexpr (W == 8) {
    const uint32_t lo = q[0] | (q[1] << 8) | (q[2] << 16) | (q[3] << 24);
    const uint32_t hi = q[4] | (q[5] << 8) | (q[6] << 16) | (q[7] << 24);
    if (aligned) __builtin_nontemporal_store(nt_u32x2{lo, hi}, reinterpret_cast<nt_u32x2*>(dst));
    else {
#pragma unroll
      for (int k = 0; k < 8; ++k) dst[k] = (uint8_t)((k < 4 ? lo : hi) >> (8 * (k & 3)));
    }
  } else {  // W == 16
    const uint4 v = make_uint4(q[0] | (q[1] << 16), q[2] | (q[3] << 16), q[4] | (q[5] << 16), q[6] | (q[7] << 16));
    if (aligned) nt_store16(dst, v.x, v.y, v.z, v.w);
    else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t wv = k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
#pragma unroll
        for (int j = 0; j < 4; ++j) dst[4 * k + j] = (uint8_t)(wv >> (8 * j));
      }
    }
  }
}

// ---- per-row pieces of K4, shared by quant_rows_kernel and the fused selection + quantization kernel
// (select_fast.hip).  Row geometry: lane l owns 8-element chunks k*64 + l (k < NCH); FULL: all NCH*64
// chunks exist (F a multiple of 512), else chunk c exists iff c < nch.

// Row min/max (NaN ignored, as fminf/fmaxf), min |x| over nonzero x (bf16/fp32 fast-division gate), and
// whether the row holds a NaN (fp16 only: its native path must not see one).
template <int DT, int NCH, bool FULL>
__device__ __forceinline__ void row_minmax(const Chunk<DT> (&raw)[NCH], int nch, int lane, float& mn, float& mx,
                                         float& anz, bool& row_nan) {
  auto valid = [&](int k) { return FULL || (k * 64 + lane) < nch; };
  mn = INFINITY; mx = -INFINITY; anz = INFINITY;
  row_nan = false;
  if constexpr (DT == RTKV_F16) {  // packed f16 min/max (NaN ignored, as fminf); NaN flagged from the bits
    const _Float16 pinf = (_Float16)INFINITY;
    h2_t mn2 = {pinf, pinf}, mx2 = {-pinf, -pinf};
    u16x2_t ab = {0, 0};
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      if (valid(k)) {
        const uint32_t w4[4] = {raw[k].a.x, raw[k].a.y, raw[k].a.z, raw[k].a.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          mn2 = __builtin_elementwise_min(mn2, as_h2(w4[j]));
          mx2 = __builtin_elementwise_max(mx2, as_h2(w4[j]));
          ab = __builtin_elementwise_max(ab, __builtin_bit_cast(u16x2_t, w4[j] & 0x7fff7fffu));
        }
      }
    }
    mn = fminf((float)mn2[0], (float)mn2[1]);
    mx = fmaxf((float)mx2[0], (float)mx2[1]);
    row_nan = __ballot(ab[0] > 0x7c00 || ab[1] > 0x7c00) != 0ull;
  } else {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      if (valid(k)) {
        float x[8];
        chunk_to_f32<DT>(raw[k], x);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          mn = fminf(mn, x[e]);
          mx = fmaxf(mx, x[e]);
          anz = fminf(anz, x[e] != 0.f ? __builtin_fabsf(x[e]) : INFINITY);
        }
      }
    }
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  if constexpr (DT != RTKV_F16) anz = wave_min(anz);
}

// Quantize, pack, dequantize and store one row (one chunk at a time): packed codes at pk (w bits per
// element) and the dequantized row at orow, either output optional.
//
// stage (fp32, CONTIG && FULL only; null elsewhere): a wave-private 2 KiB LDS buffer through which the
// dequantized chunks are stored.  A lane's 8-element fp32 chunk is 32 B, so two direct 16-byte stores
// per chunk each cover every other 16 B of the wave's 2 KiB span — partial 128-byte lines, which the
// memory side counted as ~8 % extra write and ~5 % extra read traffic (profiles/r03_k4_traffic_split.json).
// Through the stage, each store instruction writes 1 KiB contiguous (lane l: bytes 16l..16l+15).
template <int DT, int NCH, bool CONTIG, bool FULL, bool PK_ONLY = false>
__device__ __forceinline__ void emit_row(const Chunk<DT> (&raw)[NCH], const RowParams& rp, bool row_nan, int w,
                                       typename Dt<DT>::S* orow, const int (&out_off)[NCH], uint8_t* pk, int nch,
                                       int lane, bool emit_deq, bool emit_pk, float4* stage = nullptr) {
  auto valid = [&](int k) { return FULL || (k * 64 + lane) < nch; };
  // ---- quantize, pack, dequantize, store (one chunk at a time)
  // DEQ = false (packed codes only): the code is clamp(rint(t), 0, qmax) as an integer — v_cvt_u32_f32
  // saturates (negative and -0 -> 0, NaN -> 0, as the float clamp followed by the conversion), then an
  // integer min with qmax; the fast quotient skips its e == 0 guard (it only keeps the sign of a zero
  // quotient, which no code sees).  DEQ = true keeps torch.clamp's compare-select (the sign of a zero
  // and NaN reach the dequantized value).
  const uint32_t qmaxU = (uint32_t)rp.qmaxT;
  auto process = [&](auto wtag, auto ftag, auto dtag) {
    constexpr int W = decltype(wtag)::value;
    constexpr bool FASTDIV = decltype(ftag)::value;
    constexpr bool DEQ = decltype(dtag)::value;
    const bool aligned = FULL || (((uintptr_t)pk & 15) == 0 && (nch * W) % 16 == 0);
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = k * 64 + lane;
      __builtin_amdgcn_sched_barrier(0);  // keep one chunk's temporaries live at a time
      if (!valid(k)) continue;
      float x[8];
      chunk_to_f32<DT>(raw[k], x);
      uint32_t qi[8];
      if constexpr (DEQ) {
        float qd[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) qd[e] = FASTDIV ? fast_quotient(x[e], rp.scale, rp.rcp) : x[e] / rp.scale;
        float d[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float q = code_from_quotient<DT>(qd[e], rp);
          d[e] = dequant<DT>(q, rp);
          qi[e] = (uint32_t)q;
        }
        if (emit_pk) pack_store<W>(pk + c * W, qi, aligned);
        if constexpr (DT == RTKV_F32 && CONTIG && FULL) {
          if (stage) {  // 2 KiB of the row (chunks k*64 .. k*64+63) through LDS, stored contiguously
            stage[2 * lane] = make_float4(d[0], d[1], d[2], d[3]);
            stage[2 * lane + 1] = make_float4(d[4], d[5], d[6], d[7]);
            const float4 lo = stage[lane], hi = stage[64 + lane];
            float* blk = reinterpret_cast<float*>(orow) + k * 512;
            nt_store16(blk + 4 * lane, __float_as_uint(lo.x), __float_as_uint(lo.y), __float_as_uint(lo.z),
                       __float_as_uint(lo.w));
            nt_store16(blk + 256 + 4 * lane, __float_as_uint(hi.x), __float_as_uint(hi.y), __float_as_uint(hi.z),
                       __float_as_uint(hi.w));
            continue;
          }
        }
        store_chunk_nt<DT>(reinterpret_cast<Chunk<DT>*>(orow + out_off[k]), f32_to_chunk<DT>(d));
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float qd;
          if constexpr (FASTDIV) {
            const float q0 = x[e] * rp.rcp;
            qd = __builtin_fmaf(__builtin_fmaf(-q0, rp.scale, x[e]), rp.rcp, q0);
          } else {
            qd = x[e] / rp.scale;
          }
          const float t = __builtin_rintf(Dt<DT>::rnd(Dt<DT>::rnd(qd) + rp.zp));
          uint32_t u;
          asm("v_cvt_u32_f32 %0, %1" : "=v"(u) : "v"(t));
          qi[e] = u < qmaxU ? u : qmaxU;
        }
        if (emit_pk) pack_store<W>(pk + c * W, qi, aligned);
      }
    }
  };
  auto by_width = [&](auto ftag) {
    auto go = [&](auto wtag) {
      if constexpr (PK_ONLY) process(wtag, ftag, std::false_type{});
      else if (emit_deq) process(wtag, ftag, std::true_type{});
      else process(wtag, ftag, std::false_type{});
    };
    switch (w) {
      case 2: go(std::integral_constant<int, 2>{}); break;
      case 4: go(std::integral_constant<int, 4>{}); break;
      case 8: go(std::integral_constant<int, 8>{}); break;
      default: go(std::integral_constant<int, 16>{}); break;  // launcher guarantees w in {2,4,8,16}
    }
  };
  if constexpr (DT == RTKV_F16) {
    if (__builtin_amdgcn_readfirstlane((int)(rp.fast && !row_nan))) {
      const _Float16 zph = (_Float16)rp.zp, sh = (_Float16)rp.scale, qmh = (_Float16)rp.qmaxT;
      const h2_t zp2 = {zph, zph}, s2 = {sh, sh};
      auto native = [&](auto wtag, auto dtag) {
        constexpr int W = decltype(wtag)::value;
        constexpr bool DEQ = decltype(dtag)::value;
        const bool aligned = FULL || (((uintptr_t)pk & 15) == 0 && (nch * W) % 16 == 0);
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
          const int c = k * 64 + lane;
          __builtin_amdgcn_sched_barrier(0);  // keep one chunk's temporaries live at a time
          if (!valid(k)) continue;
          uint32_t qi[8], dq[4];
          f16_chunk_codes<DEQ>(raw[k].a, rp.scale, rp.rcp, zp2, s2, qmh, qi, dq);
          if (emit_pk) pack_store<W>(pk + c * W, qi, aligned);
          if constexpr (DEQ) nt_store16(orow + out_off[k], dq[0], dq[1], dq[2], dq[3]);
        }
      };
      auto by_w = [&](auto dtag) {
        switch (w) {
          case 2: native(std::integral_constant<int, 2>{}, dtag); break;
          case 4: native(std::integral_constant<int, 4>{}, dtag); break;
          case 8: native(std::integral_constant<int, 8>{}, dtag); break;
          default: native(std::integral_constant<int, 16>{}, dtag); break;
        }
      };
      if constexpr (PK_ONLY) by_w(std::false_type{});
      else if (emit_deq) by_w(std::true_type{});
      else by_w(std::false_type{});
      return;
    }
  }
  if (__builtin_amdgcn_readfirstlane((int)rp.fast)) by_width(std::true_type{});
  else by_width(std::false_type{});
}

// Layer-level checks of a K4 launch, made before its first row (every workgroup reads the same
// statistics, K2 having finished before this launch):
//  * finish (a.out_rows > 0): the caller sized K'/V' and the code planes from the early statistics;
//    a layer whose S'_max or packed byte count exceeds them is flagged RTKV_FLAG_OUTPUT_OVERFLOW and
//    nothing is written;
//  * a selection that timed out (RTKV_FLAG_SPIN_TIMEOUT, possibly after the early publication) left
//    kept_index unwritten: its rows are written as NaN (scale/zero-point too) so that stale buffers
//    never pass for results;
//  * finish with a host mirror: lane 0 of workgroup 0 publishes the final flags + final_seq there.
// Returns true when the launch must not quantize.
template <int DT>
__device__ __forceinline__ bool k4_layer_gate(const QuantArgs& a) {
  if (!a.stats) return false;
  rtkv_layer_stats* st = const_cast<rtkv_layer_stats*>(a.stats);
  int flags = st->error_flags;
  const int64_t max_kept = st->max_kept, nbytes = st->total_packed_bytes;
  // exact sizing (the drop-in): a size other than the one the device statistics give means the host read a
  // torn or stale early line — raised, never written into
  const int64_t rows_exact = max_kept > 1 ? max_kept : 1, bytes_exact = ((nbytes > 1 ? nbytes : 1) + 255) / 256 * 256;
  const bool over = a.out_rows > 0 &&
                    ((a.out.k_out_dev && (max_kept > a.out_rows || (a.exact_sizes && a.out_rows != rows_exact))) ||
                     (a.out.packed_k_dev &&
                      (nbytes > a.out.packed_capacity || (a.exact_sizes && a.out.packed_capacity != bytes_exact))));
  if (over) flags |= RTKV_FLAG_OUTPUT_OVERFLOW;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (over) atomicOr(&st->error_flags, (int)RTKV_FLAG_OUTPUT_OVERFLOW);
    if (a.final_host)  // one 8-byte store: seq and flags together (no ordering wait)
      __hip_atomic_store(&a.final_host->final_word,
                         ((a.final_seq & ((1ull << 48) - 1)) << 16) | (uint64_t)(uint32_t)(flags & 0xffff),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (over) return true;
  if (!(flags & RTKV_FLAG_SPIN_TIMEOUT)) return false;
  if (a.S_glob != 0 || !a.kept_index) return true;  // shard launches: the host raises; nothing to poison locally
  using S_ = typename Dt<DT>::S;
  const int64_t B = a.kv.B, D = a.kv.D, F = a.kv.H * a.kv.D;
  int64_t R = max_kept < 0 ? 0 : max_kept;
  if (R > a.out.row_capacity) R = a.out.row_capacity;
  if (a.out_rows > 0 && R > a.out_rows) R = a.out_rows;
  const int64_t osb = a.out.o_stride_b >= 0 ? a.out.o_stride_b : R * a.out.o_stride_s;
  const float qnan = __builtin_nanf("");
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < 2 * B * R; t += nw) {
    const int which = (int)(t & 1);
    const int64_t rr = t >> 1, b = rr / R, r = rr - b * R;
    if (a.out.k_out_dev) {
      S_* orow = static_cast<S_*>(which ? a.out.v_out_dev : a.out.k_out_dev) + b * osb + r * a.out.o_stride_s;
      for (int64_t f = lane; f < F; f += 64) orow[(f / D) * a.out.o_stride_h + (f % D)] = Dt<DT>::store(qnan);
    }
    if (a.out.scale_zp_dev && lane < 2) a.out.scale_zp_dev[(b * a.out.row_capacity + r) * 4 + which * 2 + lane] = qnan;
  }
  return true;
}

// rtkv_layer_times.end: only waves that ran one of the layer's last kStampWindow row tasks stamp it (the
// last-dispatched tasks end last; every wave stamping — ~100k atomics per cfg3 layer — cost K4 ~2.9 us,
// rocprofv3 trace of the drop-in)
constexpr int kStampWindow = 2048;

// Contiguous fp32 rows of exactly 4096 elements fit 128 VGPRs (4 waves/SIMD); the gate bookkeeping would push the
// compiler to 129 (3 waves) without the bound.  Wider fp32 rows keep the 256-register budget.
// Row geometry shared by every task of a launch: element f of a row lives at (f / D) * stride_h + f % D.
// CONTIG (stride_h == D on input and output) makes that plain f.  FULL: the row is exactly NCH*64
// chunks of 8 (F a multiple of 512), so no lane is idle and packed rows stay 16-byte aligned.
// PKW > 0 (compile time): packed codes + scale/zero-point only (no dequantized K'/V': the decode and packed
// consumers' mode), the dequantization path compiled out, at a launch bound of PKW waves per SIMD.
// PAIR (packed-only 2-byte rows): one task = a kept row's K AND V rows — one index / class / offset round
// trip for both, and both rows' loads in flight together (twice a task's bytes per wave, half the waves).
template <int DT, int NCH, bool CONTIG, bool FULL, int PKW = 0, bool PAIR = false>
__global__ __launch_bounds__(256, PKW ? PKW : ((DT == RTKV_F32 && NCH == 8 && FULL && CONTIG) ? 4 : 2)) void quant_rows_kernel(QuantArgs a) {
  constexpr bool PK_ONLY = PKW > 0;
  static_assert(!PAIR || PK_ONLY, "the paired task is the packed-only kernel's");
  constexpr int TM = PAIR ? 1 : 2;  // tasks per kept row
  using S_ = typename Dt<DT>::S;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = gridDim.x * (blockDim.x >> 6);
  const int B = (int)a.kv.B;
  const bool shard = a.S_glob != 0;
  const int S = shard ? (int)a.S_glob : (int)a.kv.S;  // tokens of the selection (labels row length)
  const int row0 = (int)a.row0, row1 = (int)(a.row0 + a.kv.S);
  const int F = (int)(a.kv.H * a.kv.D);
  const int nch = FULL ? NCH * 64 : (F + 7) >> 3;
  const int cap = (int)a.out.row_capacity;
  // One batch row (every single-GPU reference configuration): a task's kept count, token index and
  // class are independent loads, issued together — one round trip before the row loads instead of
  // stats → batch row → index.  Rows past the kept count do not exist for B = 1 (no padding rows).
  const bool one_row = B == 1;
  int R = S;  // rows per batch row (B > 1: the runtime maximum, padding rows below it)
  int64_t osb = 0;
  int tasks;
  if (one_row) {
    tasks = TM * (a.kept_index ? (cap < S ? cap : S) : S);
  } else {
    R = a.kept_index ? (int)a.stats->max_kept : S;
    if (R > cap) R = cap;
    tasks = TM * B * R;
    osb = a.out.o_stride_b >= 0 ? a.out.o_stride_b : (int64_t)R * a.out.o_stride_s;
  }
  const rtkv_batch_stats* bst = a.stats ? reinterpret_cast<const rtkv_batch_stats*>(a.stats + 1) : nullptr;
  if (k4_layer_gate<DT>(a)) return;  // buffer sizes, final flags, a timed-out selection
  const bool emit_deq = !PK_ONLY && a.out.k_out_dev != nullptr;
  const bool emit_pk = PK_ONLY || a.out.packed_k_dev != nullptr;
  // per-lane in-row offsets of each chunk (task independent)
  int in_off[NCH], out_off[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int f = (k * 64 + lane) * 8;
    if constexpr (CONTIG) {
      in_off[k] = f;
      out_off[k] = f;
    } else {
      const int D = (int)a.kv.D;
      const int h = f / D, d = f - h * D;
      in_off[k] = (int)(h * a.kv.stride_h) + d;
      out_off[k] = (int)(h * a.out.o_stride_h) + d;
    }
  }
  auto valid = [&](int k) { return FULL || (k * 64 + lane) < nch; };
  float4* stage = nullptr;  // fp32 dequantized rows go out through a wave-private LDS stage (emit_row)
  if constexpr (DT == RTKV_F32 && CONTIG && FULL && !PK_ONLY) {
    __shared__ float4 k4_stage[4][128];  // 256-thread workgroups: 4 waves × 2 KiB
    stage = k4_stage[wave & 3];
  }
  bool wrote = false;
  for (int t = blockIdx.x * (blockDim.x >> 6) + wave; t < tasks; t += nw) {
    const int which0 = PAIR ? 0 : (t & 1);
    const int rr = PAIR ? t : (t >> 1);
    int b, r, kept_b, i, lab;
    int64_t roff = -1;  // packed byte offset of the row, fetched with the index when B = 1
    if (one_row) {
      b = 0;
      r = rr;
      const int rs = r < cap ? r : cap - 1;
      const int i_s = a.kept_index ? a.kept_index[rs] : r;
      const int l_s = a.row_label ? (int)a.row_label[rs] : 0;
      if (emit_pk) roff = a.out.row_offset_dev[rs];
      kept_b = a.kept_index ? (int)bst[0].kept : S;
      if (r >= kept_b) continue;
      i = i_s;
      if ((unsigned)i >= (unsigned)S) continue;  // never read outside the layer (corrupt kept_index)
      lab = a.row_label ? l_s : (int)a.labels[i];
    } else {
      b = rr / R;
      r = rr - b * R;
      kept_b = a.kept_index ? (int)bst[b].kept : S;
      i = (r < kept_b) ? (a.kept_index ? a.kept_index[(int64_t)b * cap + r] : r) : 0;
      if ((unsigned)i >= (unsigned)S) continue;  // never read outside the layer (corrupt kept_index)
      lab = (r < kept_b) ? (a.row_label ? (int)a.row_label[(int64_t)b * cap + r] : (int)a.labels[(int64_t)b * S + i]) : 0;
    }
    i = __builtin_amdgcn_readfirstlane(i);
    lab = __builtin_amdgcn_readfirstlane(lab);
    // shard: skip another rank's token; padding rows' zero scale/zp are written by every rank (the
    // exchange carries kept rows only), their zero dequantized rows by the pad owner alone
    if (shard && r < kept_b && (i < row0 || i >= row1)) continue;
    const int rloc = a.shard_ranges ? r - (int)a.shard_ranges[((int64_t)b * (a.shard_nranks + 1) + a.shard_rank) * 2] : r;
    // (the row lambdas are force-inlined: called twice in the paired kernel, an outlined call took the
    // row arrays through 816 B of scratch per lane — 268 against 60 us)
    auto zero_row = [&](int which) __attribute__((always_inline)) {  // zero padding row (selective_propagation.py:214-222)
      if (emit_deq && (!shard || a.pad_owner)) {
        S_* orow = static_cast<S_*>(which ? a.out.v_out_dev : a.out.k_out_dev) + b * osb + (int64_t)rloc * a.out.o_stride_s;
        const Chunk<DT> z = f32_to_chunk<DT>({0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int k = 0; k < NCH; ++k)
          if (valid(k)) *reinterpret_cast<Chunk<DT>*>(orow + out_off[k]) = z;
      }
      if (a.out.scale_zp_dev && lane < 2) a.out.scale_zp_dev[((int64_t)b * cap + r) * 4 + which * 2 + lane] = 0.f;
    };
    if (r >= kept_b || lab > 2) {
      zero_row(which0);
      if constexpr (PAIR) zero_row(1);
      continue;
    }
    const int bits = lab == 0 ? a.bits[0] : (lab == 1 ? a.bits[1] : a.bits[2]);
    const int w = field_width(DT, bits);
    // ---- load the whole row(s) once (all chunks in flight), min/max
    auto load_row = [&](int which, Chunk<DT> (&raw)[NCH]) __attribute__((always_inline)) {
      const S_* src = static_cast<const S_*>(which ? a.kv.v_dev : a.kv.k_dev) + b * a.kv.stride_b +
                      (int64_t)(i - row0) * a.kv.stride_s;
#pragma unroll
      for (int k = 0; k < NCH; ++k)
        if (valid(k)) raw[k] = load_chunk_nt<DT>(src + in_off[k]);
    };
    auto quant_row = [&](int which, Chunk<DT> (&raw)[NCH]) __attribute__((always_inline)) {
      S_* orow = emit_deq ? static_cast<S_*>(which ? a.out.v_out_dev : a.out.k_out_dev) + b * osb +
                                (int64_t)rloc * a.out.o_stride_s
                          : nullptr;
      float mn, mx, anz;
      bool row_nan;
      row_minmax<DT, NCH, FULL>(raw, nch, lane, mn, mx, anz, row_nan);
      const RowParams rp = row_params<DT>(mn, mx, bits, anz);
      if (a.out.scale_zp_dev && lane < 2)
        a.out.scale_zp_dev[((int64_t)b * cap + r) * 4 + which * 2 + lane] = lane == 0 ? rp.scale : rp.zp;
      if (emit_pk && !one_row) roff = a.out.row_offset_dev[(int64_t)b * cap + r];
      uint8_t* pk = emit_pk ? (which ? a.out.packed_v_dev : a.out.packed_k_dev) + roff : nullptr;
      emit_row<DT, NCH, CONTIG, FULL, PK_ONLY>(raw, rp, row_nan, w, orow, out_off, pk, nch, lane, emit_deq, emit_pk,
                                               stage);
    };
    Chunk<DT> raw[NCH];
    load_row(which0, raw);
    if constexpr (PAIR) {
      Chunk<DT> raw_v[NCH];
      load_row(1, raw_v);
      quant_row(0, raw);
      quant_row(1, raw_v);
    } else {
      quant_row(which0, raw);
    }
    wrote |= t >= (one_row ? TM * kept_b : tasks) - kStampWindow / (3 - TM);  // one of the last tasks
  }
  stamp_end(a.t_end, wrote);
}

// Split-row K4 (one batch row, contiguous rows of NSPLIT·NCHW·512 elements; a sequence shard with its
// rtkv_shard_ranges table too): one workgroup of NSPLIT waves per (kept row, tensor), wave q owning chunks
// [q·NCHW·64, (q+1)·NCHW·64) of the row.  At S = 4096 quant_rows_kernel has ~1.2 waves of kept work
// per wave slot, so its second, mostly empty round of whole-row waves (a full load → min/max →
// store latency chain each) is a third of the kernel; here a task is NSPLIT times shorter.  The
// row's min / max / min |x| / NaN flag are combined through LDS; fminf/fmaxf are order-independent
// (a zero's sign reaches neither scale nor zero-point), so every output equals quant_rows_kernel's.
// Shard (S_glob != 0, shard_ranges set): the rank's kept rows are the contiguous output rows
// [first_row(rank), first_row(rank + 1)) of the global selection, so task t takes row first_row + t/2 and
// the grid is sized by the rank's S_local tokens (a bound on its rows) instead of S_global: no task of
// another rank's rows is launched.  The row's codes and scale/zero-point land at their global positions,
// its dequantized row at local row r − first_row.
template <int DT, int NCHW, int NSPLIT>
__global__ __launch_bounds__(64 * NSPLIT) void quant_rows_split_kernel(QuantArgs a) {
  using S_ = typename Dt<DT>::S;
  const int lane = threadIdx.x & 63;
  const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool shard = a.S_glob != 0;
  const int S = shard ? (int)a.S_glob : (int)a.kv.S;  // tokens of the selection
  const int Sl = (int)a.kv.S;                          // tokens of this launch's K/V rows
  const int cap = (int)a.out.row_capacity;
  const int tasks = 2 * (a.kept_index ? (cap < Sl ? cap : Sl) : Sl);
  const rtkv_batch_stats* bst = a.stats ? reinterpret_cast<const rtkv_batch_stats*>(a.stats + 1) : nullptr;
  if (k4_layer_gate<DT>(a)) return;  // buffer sizes, final flags, a timed-out selection
  int r_first = 0, r_end = cap;
  if (shard) {
    r_first = (int)a.shard_ranges[2 * a.shard_rank];
    r_end = (int)a.shard_ranges[2 * (a.shard_rank + 1)];
  }
  const int row0 = (int)a.row0;
  const bool emit_deq = a.out.k_out_dev != nullptr;
  const bool emit_pk = a.out.packed_k_dev != nullptr;
  __shared__ float xch[NSPLIT][4];
  float4* stage = nullptr;
  if constexpr (DT == RTKV_F32) {
    __shared__ float4 k4_stage[NSPLIT][128];
    stage = k4_stage[q];
  }
  int off[NCHW];
#pragma unroll
  for (int k = 0; k < NCHW; ++k) off[k] = (k * 64 + lane) * 8;
  const int qoff = q * NCHW * 512;  // this wave's first element of the row
  bool wrote = false;
  for (int t = blockIdx.x; t < tasks; t += gridDim.x) {  // every condition below is uniform per task
    const int which = t & 1;
    const int r = r_first + (t >> 1);
    const int rs = r < cap ? r : cap - 1;
    const int i_s = a.kept_index ? a.kept_index[rs] : r;
    const int l_s = a.row_label ? (int)a.row_label[rs] : 0;
    const int64_t roff = emit_pk ? a.out.row_offset_dev[rs] : 0;
    const int kept_b = a.kept_index ? (int)bst[0].kept : S;
    if (r >= kept_b || r >= r_end) continue;
    if ((unsigned)i_s >= (unsigned)S) continue;  // never read outside the layer (corrupt kept_index)
    if ((unsigned)(i_s - row0) >= (unsigned)Sl) continue;  // (shards) another rank's token: inconsistent ranges
    const int i = __builtin_amdgcn_readfirstlane(i_s);
    const int lab = __builtin_amdgcn_readfirstlane(a.row_label ? l_s : (int)a.labels[i]);
    S_* orow = emit_deq ? static_cast<S_*>(which ? a.out.v_out_dev : a.out.k_out_dev) +
                              (int64_t)(r - r_first) * a.out.o_stride_s + qoff
                        : nullptr;
    const int64_t sz_idx = (int64_t)r * 4 + which * 2;
    if (lab > 2) {  // zero row (caller classes outside {0,1,2})
      if (emit_deq) {
        const Chunk<DT> z = f32_to_chunk<DT>({0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int k = 0; k < NCHW; ++k) *reinterpret_cast<Chunk<DT>*>(orow + off[k]) = z;
      }
      if (q == 0 && a.out.scale_zp_dev && lane < 2) a.out.scale_zp_dev[sz_idx + lane] = 0.f;
      continue;
    }
    const int bits = lab == 0 ? a.bits[0] : (lab == 1 ? a.bits[1] : a.bits[2]);
    const int w = field_width(DT, bits);
    const S_* src = static_cast<const S_*>(which ? a.kv.v_dev : a.kv.k_dev) + (int64_t)(i - row0) * a.kv.stride_s + qoff;
    Chunk<DT> raw[NCHW];
#pragma unroll
    for (int k = 0; k < NCHW; ++k) raw[k] = load_chunk_nt<DT>(src + off[k]);
    float mn, mx, anz;
    bool row_nan;
    row_minmax<DT, NCHW, true>(raw, NCHW * 64, lane, mn, mx, anz, row_nan);
    if (lane == 0) {
      xch[q][0] = mn;
      xch[q][1] = mx;
      xch[q][2] = anz;
      xch[q][3] = row_nan ? 1.f : 0.f;
    }
    __syncthreads();
    bool nan_any = false;
#pragma unroll
    for (int p = 0; p < NSPLIT; ++p) {
      mn = fminf(mn, xch[p][0]);
      mx = fmaxf(mx, xch[p][1]);
      anz = fminf(anz, xch[p][2]);
      nan_any |= xch[p][3] != 0.f;
    }
    __syncthreads();  // xch is rewritten by the next task
    const RowParams rp = row_params<DT>(mn, mx, bits, anz);
    if (q == 0 && a.out.scale_zp_dev && lane < 2) a.out.scale_zp_dev[sz_idx + lane] = lane == 0 ? rp.scale : rp.zp;
    uint8_t* pk = emit_pk ? (which ? a.out.packed_v_dev : a.out.packed_k_dev) + roff + (int64_t)q * NCHW * 64 * w
                          : nullptr;
    emit_row<DT, NCHW, true, true>(raw, rp, nan_any, w, orow, off, pk, NCHW * 64, lane, emit_deq, emit_pk, stage);
    wrote |= t >= 2 * kept_b - kStampWindow;  // one of the last tasks
  }
  stamp_end(a.t_end, wrote);
}

// Generic path: any D, any alignment, any F (scalar element access, partial last chunk).
template <int DT>
__global__ __launch_bounds__(256) void quant_rows_generic_kernel(QuantArgs a) {
  using S_ = typename Dt<DT>::S;
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const bool shard = a.S_glob != 0;
  const int64_t B = a.kv.B, S = shard ? a.S_glob : a.kv.S, D = a.kv.D, F = a.kv.H * a.kv.D;
  const int64_t row0 = a.row0, row1 = a.row0 + a.kv.S;
  const int64_t nch = (F + 7) >> 3;
  const int64_t cap = a.out.row_capacity;
  int64_t R = a.kept_index ? a.stats->max_kept : S;
  if (R > cap) R = cap;
  const rtkv_batch_stats* bst = a.stats ? reinterpret_cast<const rtkv_batch_stats*>(a.stats + 1) : nullptr;
  if (k4_layer_gate<DT>(a)) return;
  const bool emit_deq = a.out.k_out_dev != nullptr;
  const bool emit_pk = a.out.packed_k_dev != nullptr;
  const int64_t osb = a.out.o_stride_b >= 0 ? a.out.o_stride_b : R * a.out.o_stride_s;
  for (int64_t t = gw; t < 2 * B * R; t += nw) {
    const int which = (int)(t & 1);
    const int64_t rr = t >> 1, b = rr / R, r = rr - b * R;
    const int64_t kept_b = a.kept_index ? bst[b].kept : S;
    const int64_t i = (r < kept_b) ? (a.kept_index ? a.kept_index[b * cap + r] : r) : 0;
    if (i < 0 || i >= S) continue;  // never read outside the layer (corrupt kept_index)
    const int lab = (r < kept_b) ? a.labels[b * S + i] : 0;
    if (shard && r < kept_b && (i < row0 || i >= row1)) continue;  // padding rows: as quant_rows_kernel
    const int64_t rloc = a.shard_ranges ? r - a.shard_ranges[(b * (a.shard_nranks + 1) + a.shard_rank) * 2] : r;
    S_* orow = emit_deq ? static_cast<S_*>(which ? a.out.v_out_dev : a.out.k_out_dev) + b * osb + rloc * a.out.o_stride_s
                        : nullptr;
    auto oaddr = [&](int64_t f) { return (f / D) * a.out.o_stride_h + (f % D); };
    if (r >= kept_b || lab > 2) {
      if (emit_deq && (!shard || a.pad_owner))
        for (int64_t f = lane; f < F; f += 64) orow[oaddr(f)] = Dt<DT>::store(0.f);
      if (a.out.scale_zp_dev && lane < 2) a.out.scale_zp_dev[(b * cap + r) * 4 + which * 2 + lane] = 0.f;
      continue;
    }
    const int bits = lab == 0 ? a.bits[0] : (lab == 1 ? a.bits[1] : a.bits[2]);
    const int w = field_width(DT, bits);
    const S_* src = static_cast<const S_*>(which ? a.kv.v_dev : a.kv.k_dev) + b * a.kv.stride_b + (i - row0) * a.kv.stride_s;
    auto load = [&](int64_t f) { return Dt<DT>::load(src[(f / D) * a.kv.stride_h + (f % D)]); };
    float mn = INFINITY, mx = -INFINITY;
    for (int64_t f = lane; f < F; f += 64) { const float v = load(f); mn = fminf(mn, v); mx = fmaxf(mx, v); }
    mn = wave_min(mn);
    mx = wave_max(mx);
    const RowParams rp = row_params<DT>(mn, mx, bits);
    if (a.out.scale_zp_dev && lane < 2)
      a.out.scale_zp_dev[(b * cap + r) * 4 + which * 2 + lane] = lane == 0 ? rp.scale : rp.zp;
    uint8_t* pk = emit_pk ? (which ? a.out.packed_v_dev : a.out.packed_k_dev) + a.out.row_offset_dev[b * cap + r] : nullptr;
    for (int64_t c = lane; c < nch; c += 64) {
      const int64_t f0 = c * 8;
      const int nvalid = (F - f0) < 8 ? (int)(F - f0) : 8;
      uint32_t qi[8];
      for (int e = 0; e < 8; ++e) {
        if (e < nvalid) {
          const float q = quant_code<DT>(load(f0 + e), rp);
          qi[e] = (uint32_t)q;
          if (emit_deq) orow[oaddr(f0 + e)] = Dt<DT>::store(dequant<DT>(q, rp));
        } else {
          qi[e] = 0u;
        }
      }
      if (emit_pk) {
        uint64_t p0, p1, p2;
        pack8(qi, w, p0, p1, p2);
        store_bytes(pk + c * w, (nvalid * w + 7) >> 3, p0, p1, p2);
      }
    }
  }
  stamp_end(a.t_end, true);
}

template <int DT, bool CONTIG>
static int launch_quant_vec(const QuantArgs& a, int64_t nch, dim3 grid, hipStream_t st) {
  const int per_lane = (int)((nch + 63) / 64);
  // packed-only: 0 = the runtime-mode kernel, else the compiled-out variant at that wave bound (A/B knob)
  static const int pk_waves = [] {
    const char* e = getenv("RTKV_K4_PK_WAVES");
    return e ? atoi(e) : 4;
  }();
  // RTKV_K4_PK_PAIR (A/B knob): 3 or 4 = a task is a kept row's K and V rows (half the waves), at that
  // many waves per SIMD; 0 = one row per task
  static const int pk_pair = [] {
    const char* e = getenv("RTKV_K4_PK_PAIR");
    return e ? atoi(e) : 0;
  }();
  if (!a.out.k_out_dev && a.out.packed_k_dev && pk_waves > 0 && DT != RTKV_F32) {
    const dim3 pgrid((grid.x + 1) / 2);  // half the tasks (grid = one wave per single-row task)
#define RTKV_QP(N, WV)                                                                                   \
    if (nch == (int64_t)N * 64 && pk_waves == WV) {                                                      \
      if (pk_pair == 3)                                                                                  \
        hipLaunchKernelGGL((quant_rows_kernel<DT, N, CONTIG, true, 3, true>), pgrid, dim3(256), 0, st, a); \
      else if (pk_pair)                                                                                  \
        hipLaunchKernelGGL((quant_rows_kernel<DT, N, CONTIG, true, 4, true>), pgrid, dim3(256), 0, st, a); \
      else                                                                                               \
        hipLaunchKernelGGL((quant_rows_kernel<DT, N, CONTIG, true, WV>), grid, dim3(256), 0, st, a);     \
      RTKV_HIP_CHECK(hipGetLastError());                                                                 \
      return RTKV_OK;                                                                                    \
    }
    RTKV_QP(8, 4) RTKV_QP(10, 4)
#undef RTKV_QP
  }
#define RTKV_Q(N)                                                                              \
  if (nch == (int64_t)N * 64) {                                                                \
    hipLaunchKernelGGL((quant_rows_kernel<DT, N, CONTIG, true>), grid, dim3(256), 0, st, a);   \
    RTKV_HIP_CHECK(hipGetLastError());                                                         \
    return RTKV_OK;                                                                            \
  }
  RTKV_Q(8) RTKV_Q(10) RTKV_Q(16)  // Llama-7B/13B/wide rows; smaller F takes the partial-row variants
#undef RTKV_Q
#define RTKV_Q(N)                                                                              \
  if (per_lane <= N) {                                                                         \
    hipLaunchKernelGGL((quant_rows_kernel<DT, N, CONTIG, false>), grid, dim3(256), 0, st, a);  \
    RTKV_HIP_CHECK(hipGetLastError());                                                         \
    return RTKV_OK;                                                                            \
  }
  RTKV_Q(1) RTKV_Q(2) RTKV_Q(4) RTKV_Q(8) RTKV_Q(16)
#undef RTKV_Q
  hipLaunchKernelGGL((quant_rows_generic_kernel<DT>), grid, dim3(256), 0, st, a);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

template <int DT>
int launch_quant_dt(const QuantArgs& a, hipStream_t st) {
  const rtkv_kv_desc& kv = a.kv;
  const int64_t F = kv.H * kv.D;
  const int64_t nch = (F + 7) / 8;
  const int64_t Sg = a.S_glob ? a.S_glob : kv.S;
  const int64_t R = a.kept_index ? (a.out.row_capacity < Sg ? a.out.row_capacity : Sg) : Sg;
  const int64_t tasks = 2 * kv.B * R;
  int64_t blocks = (tasks + 3) / 4;
  static const int64_t cap_blocks = [] {  // RTKV_K4_BLOCKS: experiment knob; default one wave per task (measured best: 4096 blocks 93 us, 8192 90.5 us at cfg3)
    const char* e = getenv("RTKV_K4_BLOCKS");
    return e ? (int64_t)atol(e) : (int64_t)1 << 20;
  }();
  if (blocks > cap_blocks) blocks = cap_blocks;
  if (blocks < 1) blocks = 1;
  const int esz = Dt<DT>::kBytes;
  auto al16 = [](const void* p) { return p == nullptr || ((uintptr_t)p % 16) == 0; };
  bool vec = (kv.D % 8 == 0) && al16(kv.k_dev) && al16(kv.v_dev) && (kv.stride_s * esz) % 16 == 0 &&
             (kv.stride_h * esz) % 16 == 0 && (kv.stride_b * esz) % 16 == 0;
  if (a.out.k_out_dev)
    vec = vec && al16(a.out.k_out_dev) && al16(a.out.v_out_dev) && (a.out.o_stride_s * esz) % 16 == 0 &&
          (a.out.o_stride_h * esz) % 16 == 0 && (a.out.o_stride_b < 0 || (a.out.o_stride_b * esz) % 16 == 0);
  // every in-row offset (and 2·B·R tasks) must fit in 32 bits for the vector kernel
  const int64_t in_span = (kv.H - 1) * kv.stride_h + kv.D;
  const int64_t out_span = (kv.H - 1) * a.out.o_stride_h + kv.D;
  vec = vec && in_span < ((int64_t)1 << 31) && out_span < ((int64_t)1 << 31) && tasks < ((int64_t)1 << 31) &&
        Sg < ((int64_t)1 << 31) && a.out.row_capacity < ((int64_t)1 << 31);
  const bool contig = (kv.H == 1 || kv.stride_h == kv.D) && (!a.out.k_out_dev || kv.H == 1 || a.out.o_stride_h == kv.D);
  for (int g = 0; g < 3; ++g) {  // the vector kernel packs widths 2/4/8/16 only
    const int w = field_width(DT, a.bits[g]);
    vec = vec && (w == 2 || w == 4 || w == 8 || w == 16 || !a.out.packed_k_dev);
  }
  if (!vec) {
    hipLaunchKernelGGL((quant_rows_generic_kernel<DT>), dim3((unsigned)blocks), dim3(256), 0, st, a);
    RTKV_HIP_CHECK(hipGetLastError());
    return RTKV_OK;
  }
  // single-row layers: split rows (quant_rows_split_kernel) at every S for fp32 with the dequantized
  // outputs (S = 4096: K4 50.5 -> 43.9 us, 8192: 90.3 -> 80.1, 16384 (cfg3): 168.6 -> 155.4, 65536:
  // 635 -> 608; profiles/r04f_k4_split_ab.json, r04ab/r04ac), up to S = 8192 for fp32 packed-only
  // (cfg3 packed-only: 96.4 -> 103.0 us, slower) and up to S = 4096 for the 2-byte dtypes (fp16 S = 8192:
  // 49.9 -> 50.5 us, 16384: 89.6 -> 94.7, slower).  RTKV_K4_SPLIT_MAXS overrides the token bound.
  static const int64_t split_env = [] {
    const char* e = getenv("RTKV_K4_SPLIT_MAXS");
    return e ? (int64_t)atol(e) : (int64_t)-1;
  }();
  const int64_t split_maxs = split_env >= 0 ? split_env
                               : (DT == RTKV_F32 ? (a.out.k_out_dev ? INT64_MAX : (int64_t)8192) : (int64_t)4096);
  // 2-byte dtypes with the dequantized outputs: a row over 2 waves (4 KB each) at every S — fp16 cfg3
  // K4 87.2 -> 82.5 us, S = 4096 29.0 -> 26.8 (against 4 waves), S = 65536 332 -> 317; bf16 cfg3 150.7
  // -> 142.0 (profiles/r05_k4_split2_ab.json).  fp32 (153.3 vs 154.6 us at cfg3, 43.9 vs 45.4 at
  // S = 4096) and fp16 packed-only (59.2 vs 59.9) keep theirs.  (F = 4096 rows: the measured shape.)
  // shards with their ranges table: the split-row kernel over the rank's own rows only (grid 2·S_local)
  const bool split_ok = contig && kv.B == 1 && a.kept_index && (a.S_glob == 0 || a.shard_ranges);
  const int64_t split_tasks = 2 * (a.out.row_capacity < kv.S ? a.out.row_capacity : kv.S);
  if (DT != RTKV_F32 && a.out.k_out_dev && split_env < 0 && split_ok && nch == 512) {
    hipLaunchKernelGGL((quant_rows_split_kernel<DT, 4, 2>), dim3((unsigned)split_tasks), dim3(128), 0, st, a);
    RTKV_HIP_CHECK(hipGetLastError());
    return RTKV_OK;
  }
  // (packed-only 2-byte rows over 2 waves, compile-time packed-only at 4 or 5 waves per SIMD: 60.3 / 60.5
  // against 59.7 us for the whole-row kernel at cfg3 fp16, profiles/r05_k4_split2_ab.json: not used)
  if (split_ok && Sg <= split_maxs && (nch % 64) == 0) {
    const unsigned g = (unsigned)split_tasks;
#define RTKV_QS(NCHT, NCHW, NSPLIT)                                                                       \
    if (nch == (int64_t)NCHT * 64) {                                                                      \
      hipLaunchKernelGGL((quant_rows_split_kernel<DT, NCHW, NSPLIT>), dim3(g), dim3(64 * NSPLIT), 0, st, a); \
      RTKV_HIP_CHECK(hipGetLastError());                                                                  \
      return RTKV_OK;                                                                                     \
    }
    // 4 waves per F = 4096 row; 8 waves of one chunk each measured slower (s4096 K4 43.7 -> 48.9 us,
    // profiles/r04m_k4_split8_ab.json)
    RTKV_QS(8, 2, 4) RTKV_QS(10, 2, 5)  // Llama-7B / 13B rows
#undef RTKV_QS
  }
  if (contig) return launch_quant_vec<DT, true>(a, nch, dim3((unsigned)blocks), st);
  return launch_quant_vec<DT, false>(a, nch, dim3((unsigned)blocks), st);
}

}  // namespace rtkv
