// attn_f32.hip — the model-side kernels of the fused importance mode for fp32 states, the reference
// model's precision (modified_llama.py:368 builds CompressedLlamaForCausalLM with fp32 parameters):
//
//   lse[b,h,i] = log Σ_j exp(q·k_j·scale + kbias[b,j])             (j ≤ i when causal)   attn_lse_f32_kernel
//   A[b,i]     = Σ_{p<P} (1/H) Σ_h exp(q·k_p·scale + kbias[b,p] − lse)                      qk_head_f32_kernel
//
// on gfx950's f32-input MFMA (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation; 155
// TF/s, 1/16 of the bf16 rate, so these kernels are matrix-core bound where the f16/bf16 ones
// (attn_lse.hip, qk_importance.hip) are not).  head_dim 128.
//
// Fragments (cdna_hip_programming.md, f32 16x16x4): lane l supplies A[row l&15][k = l>>4] and
// B[k = l>>4][col l&15]; the accumulator holds col l&15, rows 4(l>>4) + reg.  The k order is permuted
// so that every operand comes from 16-byte loads: k-step (j, e) covers head dims 16j + 4kg + e for
// the lane group kg = l>>4 (a dot product's order of terms is the only thing that changes: parity is a
// tolerance against the fp32 restatement, tests/test_gpu_model_side.py).  Key rows sit in LDS with
// their 16-byte chunks XOR-swizzled by row (chunk c of row r at c ^ (r & 31)).
#include <cstdlib>

#include "common.h"

namespace rtkv {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kD = 128;            // head_dim
constexpr int kRB = kD * 4;        // bytes per key row
constexpr int kCH = kRB / 16;      // 16-byte chunks per row (32)
constexpr int kKS = kD / 16;       // 16-dim groups per row (8): 4 k-steps each
constexpr float kL2E = 1.4426950408889634f;

__device__ __forceinline__ void dma16(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// 16 rows × 16 keys of q·k (raw dot products) for key rows kr = 16t + (l & 15) of an LDS tile
__device__ __forceinline__ f32x4 dot_tile(const f32x4 (&a)[kKS], const uint8_t* tile, int kr, int kg) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const uint8_t* krow = tile + kr * kRB;
#pragma unroll
  for (int j = 0; j < kKS; ++j) {
    const f32x4 b = *reinterpret_cast<const f32x4*>(krow + (((4 * j + kg) ^ (kr & (kCH - 1))) * 16));
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][e], b[e], acc, 0, 0, 0);
  }
  return acc;
}

__device__ __forceinline__ float kb_raw(const rtkv_qk_desc& q, int b, int64_t j, float inv_scale) {
  return q.kbias_dev ? key_bias_raw(q, b, j, inv_scale) : 0.f;
}

struct LseF32Args {
  rtkv_qk_desc q;
  float* lse;
  int nblk;
};

constexpr int kLKeysF = 64;  // keys per LDS tile (32 KiB)

// One workgroup: 64 query rows (16 per wave) of one (b, h); key tiles double-buffered in LDS by
// LDS-DMA, walked up to the causal diagonal; 4 column tiles per key tile = 4 independent accumulator
// chains per wave (the f32 MFMA's 40-cycle dependent latency hides behind 32-cycle issue).
__global__ __launch_bounds__(256) void attn_lse_f32_kernel(LseF32Args g) {
  constexpr int TILE = kLKeysF * kRB;
  constexpr int KI = TILE / 1024 / 4;  // DMA instructions per wave per tile
  constexpr int RPI = 1024 / kRB;      // key rows per DMA instruction
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];  // 2 × TILE
  const rtkv_qk_desc& q = g.q;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, kg = lane >> 4;
  // XCD-aware order, as attn_lse32.hip: each XCD runs whole heads (longest query block first), so a
  // head's keys stay in one L2
  int qb, h, b;
  {
    const int nwg = (int)(gridDim.x * gridDim.y * gridDim.z);
    int bid = (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
    if ((nwg & 7) == 0) bid = (bid & 7) * (nwg >> 3) + (bid >> 3);
    const int unit = bid / g.nblk;
    qb = g.nblk - 1 - (bid - unit * g.nblk);
    h = unit % (int)gridDim.y;
    b = unit / (int)gridDim.y;
  }
  const int S = (int)q.S, grp = (int)(q.H / q.Hkv);
  const int i0 = qb * 64, wrow0 = i0 + wave * 16, crow0 = wrow0 + 4 * kg;
  const float sc = q.scale * kL2E, inv_scale = 1.f / q.scale;
  const float* Kh = static_cast<const float*>(q.k_dev) + b * q.k_stride_b + (int64_t)(h / grp) * q.k_stride_h;
  int64_t kend = q.causal ? q.row0 + i0 + 64 : S;
  if (kend > S) kend = S;
  const int ntiles = (int)((kend + kLKeysF - 1) / kLKeysF);
  const int lrow = lane / kCH, lpc = lane % kCH;
  auto issue = [&](int kt) {
    uint8_t* st = lds + (kt & 1) * TILE;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      const int r = (wave * KI + k) * RPI + lrow;
      const int c = lpc ^ (r & (kCH - 1));
      int kr = kt * kLKeysF + r;
      kr = kr < S ? kr : S - 1;
      dma16(Kh + (int64_t)kr * q.k_stride_s + c * 4, st + (wave * KI + k) * 1024);
    }
  };
  f32x4 a[kKS];
  {
    const int qr = wrow0 + c16 < S ? wrow0 + c16 : S - 1;
    const float* qrow = static_cast<const float*>(q.q_dev) + b * q.q_stride_b + (int64_t)h * q.q_stride_h +
                        (int64_t)qr * q.q_stride_s;
#pragma unroll
    for (int j = 0; j < kKS; ++j) a[j] = *reinterpret_cast<const f32x4*>(qrow + 16 * j + 4 * kg);
  }
  float m[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { m[r] = -1e30f; l[r] = 0.f; }
  issue(0);
  for (int kt = 0; kt < ntiles; ++kt) {
    if (kt + 1 < ntiles) {
      issue(kt + 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KI) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // every wave's pieces of tile kt landed
    const uint8_t* st = lds + (kt & 1) * TILE;
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = dot_tile(a, st, 16 * t + c16, kg);
    __builtin_amdgcn_s_barrier();  // every wave has read tile kt: its slot is free for tile kt+2
    const bool edge = (int64_t)(kt + 1) * kLKeysF > (q.causal ? q.row0 + wrow0 : (int64_t)S) || (kt + 1) * kLKeysF > S;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int64_t j = (int64_t)kt * kLKeysF + 16 * t + c16;
      const float kb = (q.kbias_dev && j < S) ? kb_raw(q, b, j, inv_scale) : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = !edge || (j < S && (!q.causal || j <= q.row0 + crow0 + r));
        acc[t][r] = ok ? acc[t][r] + kb : -INFINITY;
      }
    }
    bool up = false;
    float mt[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mt[r] = fmaxf(fmaxf(acc[0][r], acc[1][r]), fmaxf(acc[2][r], acc[3][r])) * sc;
      up |= mt[r] > m[r] + 8.f;
    }
    if (__ballot(up)) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float mn = mt[r] > m[r] + 8.f ? mt[r] : m[r];
        l[r] *= __builtin_amdgcn_exp2f(m[r] - mn);
        m[r] = mn;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int t = 0; t < 4; ++t) l[r] += __builtin_amdgcn_exp2f(__builtin_fmaf(acc[t][r], sc, -m[r]));
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float M = m[r];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) M = fmaxf(M, __shfl_xor(M, o, 64));
    float L = l[r] * __builtin_amdgcn_exp2f(m[r] - M);
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) L += __shfl_xor(L, o, 64);
    const int i = crow0 + r;
    if (c16 == 0 && i < S)
      g.lse[b * q.lse_stride_b + (int64_t)h * q.lse_stride_h + i] = L > 0.f ? (M + __log2f(L)) * 0.6931471805599453f : -INFINITY;
  }
}

// Head-major K1' (as qk_head_kernel): a workgroup owns ONE head and 4·rpw query rows; the head's
// P ≤ 128 prompt keys stay in LDS (64 KiB); each wave walks its rows in 16-row tiles and writes the
// per-head prompt mass of each row to part[b][h][i] (qk_head_reduce_kernel sums the heads in order).
__global__ __launch_bounds__(256) void qk_head_f32_kernel(rtkv_qk_desc q, int P, float* __restrict__ part, int rpw,
                                                          unsigned long long* t_begin) {
  stamp_begin(t_begin);
  constexpr int PT = 128;
  constexpr int KEY_BYTES = PT * kRB;
  constexpr int KI = KEY_BYTES / 1024 / 4;
  constexpr int RPI = 1024 / kRB;
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];  // KEY_BYTES
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, kg = lane >> 4;
  const int h = blockIdx.y, b = blockIdx.z;
  const int S = (int)q.S, grp = (int)(q.H / q.Hkv);
  const int wrow = (blockIdx.x * 4 + wave) * rpw;
  const float sc = q.scale * kL2E, inv_scale = 1.f / q.scale;
  const float* Qh = static_cast<const float*>(q.q_dev) + b * q.q_stride_b + (int64_t)h * q.q_stride_h;
  const float* Lh = q.lse_dev + b * q.lse_stride_b + (int64_t)h * q.lse_stride_h;
  float* Ph = part + ((int64_t)b * q.H + h) * S;
  {
    const float* kh = static_cast<const float*>(q.k_dev) + b * q.k_stride_b + (int64_t)(h / grp) * q.k_stride_h;
    const int lrow = lane / kCH, lpc = lane % kCH;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      const int r = (wave * KI + k) * RPI + lrow;
      const int c = lpc ^ (r & (kCH - 1));
      const int pr = r < P ? r : P - 1;
      dma16(kh + (int64_t)pr * q.k_stride_s + c * 4, lds + (wave * KI + k) * 1024);
    }
  }
  // the prompt columns' key bias (raw units), the same for every row
  float kb[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) kb[t] = (16 * t + c16 < P) ? kb_raw(q, b, 16 * t + c16, inv_scale) : 0.f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int ntile = rpw / 16;
  for (int k = 0; k < ntile; ++k) {
    const int r0 = wrow + 16 * k;
    if (r0 >= S) break;
    const int crow0 = r0 + 4 * kg;
    f32x4 a[kKS];
    {
      const int qr = r0 + c16 < S ? r0 + c16 : S - 1;
      const float* qp = Qh + (int64_t)qr * q.q_stride_s;
#pragma unroll
      for (int j = 0; j < kKS; ++j) a[j] = *reinterpret_cast<const f32x4*>(qp + 16 * j + 4 * kg);
    }
    float lv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) lv[r] = crow0 + r < S ? Lh[crow0 + r] : 0.f;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      if (16 * t >= P) break;
      const f32x4 acc = dot_tile(a, lds, 16 * t + c16, kg);
      const int p = 16 * t + c16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = crow0 + r;
        const bool ok = p < P && i < S && (!q.causal || (int64_t)p <= q.row0 + i);
        const float w = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[r] + kb[t], sc, -lv[r] * kL2E));
        v[r] += ok ? w : 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) v[r] += __shfl_xor(v[r], o, 64);
      // a row that sees no key at all (lse = -inf): the reference's all-masked softmax row is uniform
      if (lv[r] == -INFINITY) v[r] = (float)P / (float)S;
    }
    if (c16 == 0 && crow0 < S) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (crow0 + r < S) Ph[crow0 + r] = v[r];
    }
  }
}

// ---- The fp32 LSE on the bf16 matrix cores (round 5).  Each fp32 operand is split into three bf16
// parts, x = x_h + x_l + x_ll (round-to-nearest splits: every part holds the next 8 significant bits, the
// residual is below 2^-27 |x|), and q·k is the sum of the six part products down to order 2^-18:
// h·h, h·l, l·h, h·ll, ll·h, l·l — the dropped l·ll, ll·l, ll·ll are below 2^-27 |q||k| each, under
// fp32's own 2^-24 rounding of a product.  Six v_mfma_f32_16x16x32_bf16 (fp32 accumulation) per
// 16 × 16 × 32 block take 6 × 16 cycles where the exact f32 MFMA takes 8 × 32 (v_mfma_f32_16x16x4_f32 at
// 1/16 of the bf16 rate): 2.7× fewer matrix cycles for the same logits to fp32 accuracy (not bit for
// bit: the f32 kernel above stays as RTKV_LSE_F32_EXACT).
//
// Work decomposition (attn_lse_f32x3s_kernel below): a workgroup of 16 waves owns 256 query rows of one
// (b, h), 16 per wave (Q split once into registers: 3 planes × 4 k-steps, 48 registers, so four waves
// per SIMD overlap one another's bookkeeping and MFMAs); key tiles of 64 rows are loaded by all 1024
// threads into registers a full iteration ahead, split, and written to LDS as three swizzled bf16 planes
// (double-buffered, 2 × 48 KiB, one barrier per tile), the split of tile kt + 1 issuing inside tile kt's
// MFMA block.  Softmax bookkeeping as attn_lse_f32_kernel: a checked lazy max (raised by 8 log2 units at
// most once per tile and row), so no fix-up pass.  Measured (S = 16384, 32 heads): 5.2 ms against 10.5
// for the exact kernel; a 32-row tiling on 32x32x16 (96 registers of Q planes: one wave per SIMD) 6.8 ms,
// this tiling at 8 waves per workgroup (two per SIMD) 6.3 ms.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kX3Keys = 64;              // key rows per tile
constexpr int kX3Plane = kX3Keys * 256;  // one bf16 plane of a tile (16 KiB)

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& l, __bf16& ll) {
  h = (__bf16)x;
  // exact (x and h share the leading bits).  A value with no finite bf16 head (±inf, or finite above the
  // bf16 maximum ≈ 3.39e38, which rounds to inf) keeps l = ll = 0: its products with the other operand's
  // parts are ±inf or NaN, as the exact kernel's product with an overflowing operand is
  const float r1 = __builtin_isfinite((float)h) ? x - (float)h : 0.f;
  l = (__bf16)r1;
  const float r2 = r1 - (float)l;                               // exact
  ll = (__bf16)r2;
}

// 8 consecutive fp32 values → their three bf16x8 parts
__device__ __forceinline__ void split8(const f32x4& x0, const f32x4& x1, bf16x8& h, bf16x8& l, bf16x8& ll) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    __bf16 a, b, c;
    split3(e < 4 ? x0[e] : x1[e - 4], a, b, c);
    h[e] = a;
    l[e] = b;
    ll[e] = c;
  }
}

// The split-bf16 LSE on 16-row wave tiles (v_mfma_f32_16x16x32_bf16): Q's three planes take 48
// registers, so NW = 16 waves (four per SIMD, 128 registers) share a workgroup of 256 query rows and the
// waves' bookkeeping overlaps one another's MFMAs.  Fragments (cdna_hip_programming.md §3): lane l supplies
// A[row l & 15][k = 8 (l >> 4) + j] and B[k = 8 (l >> 4) + j][col l & 15]; k-step s covers the 16-byte
// chunk 4s + (l >> 4) of a row (A and B alike); the accumulator holds key column l & 15 of rows
// 4 (l >> 4) + r.  Bookkeeping as attn_lse_f32_kernel (4 rows per lane, 16 lanes per row group).
template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_lse_f32x3s_kernel(LseF32Args g) {
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];  // 2 buffers × 3 planes × kX3Plane
  constexpr int ROWS = 16 * NW;
  constexpr int EPT = kX3Keys * 128 / (64 * NW);  // key elements per thread and tile
  static_assert(EPT % 8 == 0, "whole 16-byte chunks per thread");
  constexpr int CPT = EPT / 8;                      // chunks per thread and plane
  const rtkv_qk_desc& q = g.q;
  const int t = threadIdx.x;
  const int lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int c16 = lane & 15, kg = lane >> 4;
  int qb, hd, b;  // XCD-aware order, as attn_lse32.hip
  {
    const int nwg = (int)(gridDim.x * gridDim.y * gridDim.z);
    int bid = (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
    if ((nwg & 7) == 0) bid = (bid & 7) * (nwg >> 3) + (bid >> 3);
    const int unit = bid / g.nblk;
    qb = g.nblk - 1 - (bid - unit * g.nblk);
    hd = unit % (int)gridDim.y;
    b = unit / (int)gridDim.y;
  }
  const int S = (int)q.S, grp = (int)(q.H / q.Hkv);
  const int i0 = qb * ROWS, wrow0 = i0 + 16 * wave, crow0 = wrow0 + 4 * kg;
  const float sc = q.scale * kL2E, inv_scale = 1.f / q.scale;
  const float* Kh = static_cast<const float*>(q.k_dev) + b * q.k_stride_b + (int64_t)(hd / grp) * q.k_stride_h;
  int64_t kend = q.causal ? q.row0 + i0 + ROWS : S;
  if (kend > S) kend = S;
  const int ntiles = (int)((kend + kX3Keys - 1) / kX3Keys);
  // this thread's share of a key tile: key row kr, EPT consecutive dims from kd
  constexpr int TPR = 128 / EPT;  // threads per key row
  const int kr = t / TPR, kd = (t % TPR) * EPT;
  f32x4 kreg[EPT / 4], knext[EPT / 4];
  auto load_tile = [&](int kt, f32x4 (&dst)[EPT / 4]) {  // (rows clamped: a tile past the end is a harmless re-read)
    int r = kt * kX3Keys + kr;
    r = r < S ? r : S - 1;
    const float* src = Kh + (int64_t)r * q.k_stride_s + kd;
#pragma unroll
    for (int e = 0; e < EPT / 4; ++e) dst[e] = *reinterpret_cast<const f32x4*>(src + 4 * e);
  };
  load_tile(0, kreg);
  bf16x8 ah[4], al[4], all[4];  // Q row c16 of the wave's 16, k-step s = chunk 4s + kg
  {
    const int qr = wrow0 + c16 < S ? wrow0 + c16 : S - 1;
    const float* qrow = static_cast<const float*>(q.q_dev) + b * q.q_stride_b + (int64_t)hd * q.q_stride_h +
                        (int64_t)qr * q.q_stride_s;
#pragma unroll
    for (int s_ = 0; s_ < 4; ++s_) {
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(qrow + (4 * s_ + kg) * 8);
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(qrow + (4 * s_ + kg) * 8 + 4);
      split8(x0, x1, ah[s_], al[s_], all[s_]);
    }
  }
  float m[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { m[r] = -1e30f; l[r] = 0.f; }
  auto split_store = [&](int kt) {
    uint8_t* buf = lds + (kt & 1) * 3 * kX3Plane;
    const int sw = kr & 15;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      bf16x8 h, lo, ll;
      split8(kreg[2 * c], kreg[2 * c + 1], h, lo, ll);
      const int off = kr * 256 + ((((kd >> 3) + c) ^ sw) * 16);
      *reinterpret_cast<bf16x8*>(buf + off) = h;
      *reinterpret_cast<bf16x8*>(buf + kX3Plane + off) = lo;
      *reinterpret_cast<bf16x8*>(buf + 2 * kX3Plane + off) = ll;
    }
  };
  split_store(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  load_tile(1, kreg);
  for (int kt = 0; kt < ntiles; ++kt) {
    load_tile(kt + 2, knext);  // a whole iteration ahead of its split
    const uint8_t* buf = lds + (kt & 1) * 3 * kX3Plane;
    f32x4 acc[4];
#pragma unroll
    for (int tc = 0; tc < 4; ++tc) {  // 16-key column tiles
      const int kro = 16 * tc + c16;
      const uint8_t* krow = buf + kro * 256;
      const int sw = kro & 15;
      acc[tc] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s_ = 0; s_ < 4; ++s_) {
        const int c = ((4 * s_ + kg) ^ sw) * 16;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(krow + c);
        const bf16x8 bl = *reinterpret_cast<const bf16x8*>(krow + kX3Plane + c);
        const bf16x8 bll = *reinterpret_cast<const bf16x8*>(krow + 2 * kX3Plane + c);
        acc[tc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[s_], bl, acc[tc], 0, 0, 0);
        acc[tc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[s_], bll, acc[tc], 0, 0, 0);
        acc[tc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(all[s_], bh, acc[tc], 0, 0, 0);
        acc[tc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[s_], bl, acc[tc], 0, 0, 0);
        acc[tc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[s_], bh, acc[tc], 0, 0, 0);
        acc[tc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[s_], bh, acc[tc], 0, 0, 0);
      }
    }
    if constexpr (NW > 8) {  // a k-step's 3 fragment reads just ahead of its 6 MFMAs (registers)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
      }
    }
    split_store(kt + 1);
    const bool edge = (int64_t)(kt + 1) * kX3Keys > (q.causal ? q.row0 + wrow0 : (int64_t)S) || (kt + 1) * kX3Keys > S;
#pragma unroll
    for (int tc = 0; tc < 4; ++tc) {
      const int64_t j = (int64_t)kt * kX3Keys + 16 * tc + c16;
      const float kb = (q.kbias_dev && j < S) ? kb_raw(q, b, j, inv_scale) : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = !edge || (j < S && (!q.causal || j <= q.row0 + crow0 + r));
        acc[tc][r] = ok ? acc[tc][r] + kb : -INFINITY;
      }
    }
    bool up = false;
    float mt[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mt[r] = fmaxf(fmaxf(acc[0][r], acc[1][r]), fmaxf(acc[2][r], acc[3][r])) * sc;
      up |= mt[r] > m[r] + 8.f;
    }
    if (__ballot(up)) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float mn = mt[r] > m[r] + 8.f ? mt[r] : m[r];
        l[r] *= __builtin_amdgcn_exp2f(m[r] - mn);
        m[r] = mn;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int tc = 0; tc < 4; ++tc) l[r] += __builtin_amdgcn_exp2f(__builtin_fmaf(acc[tc][r], sc, -m[r]));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int e = 0; e < EPT / 4; ++e) kreg[e] = knext[e];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float M = m[r];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) M = fmaxf(M, __shfl_xor(M, o, 64));
    float L = l[r] * __builtin_amdgcn_exp2f(m[r] - M);
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) L += __shfl_xor(L, o, 64);
    const int i = crow0 + r;
    if (c16 == 0 && i < S)
      g.lse[b * q.lse_stride_b + (int64_t)hd * q.lse_stride_h + i] = L > 0.f ? (M + __log2f(L)) * 0.6931471805599453f : -INFINITY;
  }
}

// Head-major K1' for fp32 states on the bf16 matrix cores, with the LSE kernel's three-way split: the
// head's P ≤ 128 prompt keys are split once per workgroup into three bf16 planes in LDS (96 KiB); 16 waves
// (1024 threads, four per SIMD at 128 registers) each walk their rows in 16-row tiles, the tile's queries
// split into registers (48), 8 column tiles × 4 k-steps × 6 part products on v_mfma_f32_16x16x32_bf16,
// then exp2(x·scale·log2e − lse·log2e) (+ key bias) summed over the prompt columns and written to
// part[b][h][i] as qk_head_f32_kernel does (qk_head_reduce_kernel sums the heads).
template <int NW>
__global__ __launch_bounds__(64 * NW) void qk_head_f32x3_kernel(rtkv_qk_desc q, int P, float* __restrict__ part, int rpw,
                                                               unsigned long long* t_begin) {
  stamp_begin(t_begin);
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];  // 3 planes × 128 rows × 256 B
  constexpr int PL = 128 * 256;                                     // one plane
  const int t = threadIdx.x;
  const int lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int c16 = lane & 15, kg = lane >> 4;
  const int h = blockIdx.y, b = blockIdx.z;
  const int S = (int)q.S, grp = (int)(q.H / q.Hkv);
  const int wrow = (blockIdx.x * NW + wave) * rpw;
  const float sc = q.scale * kL2E, inv_scale = 1.f / q.scale;
  const float* Qh = static_cast<const float*>(q.q_dev) + b * q.q_stride_b + (int64_t)h * q.q_stride_h;
  const float* Lh = q.lse_dev + b * q.lse_stride_b + (int64_t)h * q.lse_stride_h;
  float* Ph = part + ((int64_t)b * q.H + h) * S;
  {  // the head's prompt keys: thread t splits EPT dims of key row kr (rows past P: row P - 1)
    constexpr int EPT = 128 * 128 / (64 * NW), TPR = 128 / EPT;
    const float* kh = static_cast<const float*>(q.k_dev) + b * q.k_stride_b + (int64_t)(h / grp) * q.k_stride_h;
    const int kr = t / TPR, kd = (t % TPR) * EPT;
    const float* src = kh + (int64_t)(kr < P ? kr : P - 1) * q.k_stride_s + kd;
    f32x4 x[EPT / 4];
#pragma unroll
    for (int e = 0; e < EPT / 4; ++e) x[e] = *reinterpret_cast<const f32x4*>(src + 4 * e);
    const int sw = kr & 15;
#pragma unroll
    for (int c = 0; c < EPT / 8; ++c) {
      bf16x8 hi, lo, ll;
      split8(x[2 * c], x[2 * c + 1], hi, lo, ll);
      const int off = kr * 256 + ((((kd >> 3) + c) ^ sw) * 16);
      *reinterpret_cast<bf16x8*>(lds + off) = hi;
      *reinterpret_cast<bf16x8*>(lds + PL + off) = lo;
      *reinterpret_cast<bf16x8*>(lds + 2 * PL + off) = ll;
    }
  }
  // the prompt columns' key bias (raw units), the same for every row: a 128-entry LDS table
  float* kbl = reinterpret_cast<float*>(lds + 3 * PL);
  if (t < 128) kbl[t] = t < P ? kb_raw(q, b, t, inv_scale) : 0.f;
  __syncthreads();
  const int ntile = rpw / 16;
  for (int k = 0; k < ntile; ++k) {
    const int r0 = wrow + 16 * k;
    if (r0 >= S) break;
    const int crow0 = r0 + 4 * kg;
    bf16x8 ah[4], al[4], all[4];  // row c16 of the tile, k-step s = chunk 4s + kg
    {
      const int qr = r0 + c16 < S ? r0 + c16 : S - 1;
      const float* qp = Qh + (int64_t)qr * q.q_stride_s;
#pragma unroll
      for (int s_ = 0; s_ < 4; ++s_) {
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(qp + (4 * s_ + kg) * 8);
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(qp + (4 * s_ + kg) * 8 + 4);
        split8(x0, x1, ah[s_], al[s_], all[s_]);
      }
    }
    float lv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) lv[r] = crow0 + r < S ? Lh[crow0 + r] : 0.f;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tc = 0; tc < 8; ++tc) {
      if (16 * tc >= P) break;
      const int kro = 16 * tc + c16;
      const uint8_t* krow = lds + kro * 256;
      const int sw = kro & 15;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s_ = 0; s_ < 4; ++s_) {
        const int c = ((4 * s_ + kg) ^ sw) * 16;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(krow + c);
        const bf16x8 bl = *reinterpret_cast<const bf16x8*>(krow + PL + c);
        const bf16x8 bll = *reinterpret_cast<const bf16x8*>(krow + 2 * PL + c);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[s_], bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[s_], bll, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(all[s_], bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[s_], bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[s_], bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[s_], bh, acc, 0, 0, 0);
      }
      // a k-step's 3 fragment reads just ahead of its 6 MFMAs (registers)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
      }
      const int p = kro;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = crow0 + r;
        const bool ok = p < P && i < S && (!q.causal || (int64_t)p <= q.row0 + i);
        const float w = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[r] + kbl[kro], sc, -lv[r] * kL2E));
        v[r] += ok ? w : 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) v[r] += __shfl_xor(v[r], o, 64);
      if (lv[r] == -INFINITY) v[r] = (float)P / (float)S;  // a row that sees no key: the uniform row
    }
    if (c16 == 0 && crow0 < S) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (crow0 + r < S) Ph[crow0 + r] = v[r];
    }
  }
}

}  // namespace

int launch_attention_lse_f32(const rtkv_qk_desc& q, float* lse, hipStream_t st) {
  RTKV_REQUIRE(q.D == kD, "attention_lse (fp32): head_dim must be 128");
  RTKV_REQUIRE(q.q_stride_s % 4 == 0 && q.q_stride_h % 4 == 0 && q.q_stride_b % 4 == 0 && q.k_stride_s % 4 == 0 &&
                   q.k_stride_h % 4 == 0 && q.k_stride_b % 4 == 0 && ((uintptr_t)q.q_dev % 16) == 0 &&
                   ((uintptr_t)q.k_dev % 16) == 0,
               "attention_lse (fp32): Q/K rows must be 16-byte aligned");
  // default: the split-bf16 kernel (fp32-accurate, not bit-identical); RTKV_LSE_F32_EXACT: the exact
  // f32-MFMA kernel
  static const bool exact = getenv("RTKV_LSE_F32_EXACT") != nullptr;
  if (!exact) {
    constexpr size_t lds3 = 6 * (size_t)kX3Plane;
    static bool attr3 = false;
    if (!attr3) {
      RTKV_HIP_CHECK(hipFuncSetAttribute((const void*)attn_lse_f32x3s_kernel<16>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds3));
      attr3 = true;
    }
    LseF32Args a;
    a.q = q;
    a.lse = lse;
    a.nblk = (int)((q.S + 255) / 256);
    hipLaunchKernelGGL(attn_lse_f32x3s_kernel<16>, dim3((unsigned)a.nblk, (unsigned)q.H, (unsigned)q.B), dim3(1024),
                       lds3, st, a);
    RTKV_HIP_CHECK(hipGetLastError());
    return RTKV_OK;
  }
  constexpr size_t lds = 2 * (size_t)kLKeysF * kRB;
  static bool attr = false;
  if (!attr) {
    RTKV_HIP_CHECK(hipFuncSetAttribute((const void*)attn_lse_f32_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds));
    attr = true;
  }
  LseF32Args a;
  a.q = q;
  a.lse = lse;
  a.nblk = (int)((q.S + 63) / 64);
  hipLaunchKernelGGL(attn_lse_f32_kernel, dim3((unsigned)a.nblk, (unsigned)q.H, (unsigned)q.B), dim3(256), lds, st, a);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

int launch_qk_head_f32(const rtkv_qk_desc& q, int P, float* part, hipStream_t st, unsigned long long* t_begin) {
  RTKV_REQUIRE(q.D == kD, "importance_qk_lse (fp32): head_dim must be 128");
  RTKV_REQUIRE(q.q_stride_s % 4 == 0 && q.q_stride_h % 4 == 0 && q.q_stride_b % 4 == 0 && q.k_stride_s % 4 == 0 &&
                   q.k_stride_h % 4 == 0 && q.k_stride_b % 4 == 0 && ((uintptr_t)q.q_dev % 16) == 0 &&
                   ((uintptr_t)q.k_dev % 16) == 0,
               "importance_qk_lse (fp32): Q/K rows must be 16-byte aligned");
  // default: the split-bf16 kernel; RTKV_LSE_F32_EXACT also selects the exact f32-MFMA K1'
  static const bool exact = getenv("RTKV_LSE_F32_EXACT") != nullptr;
  if (!exact) {
    constexpr size_t lds3 = (size_t)3 * 128 * 256 + 128 * sizeof(float);
    // 16 waves per workgroup (four per SIMD; 6 registers spilled): 113.6 against 120.8 us per cfg3 fp32
    // layer for 8 waves without spills (profiles/r05_qkf32_ab.json)
    constexpr int nw = 16;
    static bool attr3 = false;
    if (!attr3) {
      RTKV_HIP_CHECK(hipFuncSetAttribute((const void*)qk_head_f32x3_kernel<16>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds3));
      attr3 = true;
    }
    // rows per wave (16-row tiles): about 512 workgroups (two rounds of one per CU)
    int rpw = 256;
    while (rpw > 16 && (q.S + nw * rpw - 1) / (nw * rpw) * q.H * q.B < 512) rpw /= 2;
    const dim3 grid((unsigned)((q.S + nw * rpw - 1) / (nw * rpw)), (unsigned)q.H, (unsigned)q.B);
    hipLaunchKernelGGL(qk_head_f32x3_kernel<nw>, grid, dim3(64 * nw), lds3, st, q, P, part, rpw, t_begin);
    RTKV_HIP_CHECK(hipGetLastError());
    return RTKV_OK;
  }
  constexpr size_t lds = (size_t)128 * kRB;
  static bool attr = false;
  if (!attr) {
    RTKV_HIP_CHECK(hipFuncSetAttribute((const void*)qk_head_f32_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds));
    attr = true;
  }
  int rpw = 256;
  while (rpw > 16 && (q.S + 4 * rpw - 1) / (4 * rpw) * q.H * q.B < 2048) rpw /= 2;
  const dim3 grid((unsigned)((q.S + 4 * rpw - 1) / (4 * rpw)), (unsigned)q.H, (unsigned)q.B);
  hipLaunchKernelGGL(qk_head_f32_kernel, grid, dim3(256), lds, st, q, P, part, rpw, t_begin);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

}  // namespace rtkv
