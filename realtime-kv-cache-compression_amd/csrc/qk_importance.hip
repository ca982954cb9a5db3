// qk_importance.hip — K1': the fused importance mode.  The prompt-attention mass of every token is
// computed from the queries, the prompt keys and the row log-sum-exp instead of reading a
// materialised attention matrix:
//
//   A[b,i] = Σ_{p<P} (1/H) Σ_h exp(q[b,h,i]·k[b,h/g,p]·scale − lse[b,h,i])        (p ≤ i if causal)
//
// which is the reference's compute_attention_aggregation (token_importance.py:21-47) applied to
// W = softmax(Q·Kᵀ/√d + mask) (modified_llama.py:88-94) restricted to the first P key columns.
// The reference model runs in fp32, so W is kept in fp32 here (no rounding to the
// input dtype) and A is produced as fp32; parity is a tolerance (north_star: 1e-3 rel on scores).
//
// Work decomposition (gfx950, wave64): a workgroup owns 64 query rows of one batch row, one wave
// per 16 rows, and walks the heads.  Per head the P×D prompt-key tile is staged in LDS once
// (double-buffered, shared by the 4 waves) and each wave computes its 16 × P logits with
// v_mfma_f32_16x16x32_{f16,bf16} (NT column tiles of 16, KS k-steps of 32), then
// exp2(x·scale·log2e − lse·log2e) and the head sum in registers.  Next head's keys and query
// fragments are loaded from HBM while the current head computes.  Fragment maps
// (cdna_hip_programming.md §3): lane l holds A[row l&15][k 8(l>>4)..+7] and
// B[k 8(l>>4)..+7][col l&15]; the accumulator holds col l&15, rows 4(l>>4) + reg.
// Waves own disjoint rows, so the only reduction is over the 16 columns held across lanes.
#include <cstdlib>

#include "common.h"

namespace rtkv {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct QKArgs {
  rtkv_qk_desc q;
  int P;
  float* A;
  AggExtras ex;
};

template <int DT> struct Frag;
template <> struct Frag<RTKV_F16> {
  using T = f16x8;
  __device__ __forceinline__ static f32x4 mfma(T a, T b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
template <> struct Frag<RTKV_BF16> {
  using T = bf16x8;
  __device__ __forceinline__ static f32x4 mfma(T a, T b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};

constexpr int kQKRows = 64;   // query rows per workgroup (4 waves × 16)
constexpr int kQKStages = 3;  // LDS ring depth (heads in flight)

// LDS-DMA of one 16-byte chunk per lane: the wave writes 1 KiB lane-linear at lds_base (M0).
__device__ __forceinline__ void glds16(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_base, 4, 0, 0);
}

// NT: column tiles of 16 (P ≤ 16·NT); KS: k-steps of 32 (D = 32·KS).
//
// Per head h the workgroup stages, by LDS-DMA into ring slot h % 3: the P×D prompt keys (kv head
// h/g), its 64 query rows and their 64 LSE values.  Rows are 2·D bytes, chunk c of row r sits at
// physical chunk c ^ (r & (CH-1)) (the swizzle is applied on the global source address: the DMA
// writes lane-linear), which makes the fragment reads conflict-free.  Two heads stay in flight while
// one is computed (counted vmcnt, raw s_barrier: a __syncthreads would drain the DMA queue).
template <int DT, int NT, int KS>
__global__ __launch_bounds__(256) void qk_importance_kernel(QKArgs g) {
  using FT = typename Frag<DT>::T;
  using S_ = typename Dt<DT>::S;
  constexpr int D = 32 * KS;
  constexpr int PT = 16 * NT;                      // padded prompt rows
  constexpr int RB = 2 * D;                        // bytes per row
  constexpr int CH = RB / 16;                      // 16-byte chunks per row
  constexpr int RPI = 1024 / RB;                   // rows per DMA wave-instruction
  constexpr int KEY_BYTES = PT * RB, Q_BYTES = kQKRows * RB;
  constexpr int STAGE = KEY_BYTES + Q_BYTES + kQKRows * 4;
  constexpr int KI = KEY_BYTES / 1024 / 4;         // key DMA instructions per wave per head
  constexpr int QI = Q_BYTES / 1024 / 4;           // query DMA instructions per wave per head
  constexpr int OPS = KI + QI + 1;                 // DMA ops per wave per head (+1: LSE)
  static_assert(KI >= 1 && QI >= 1, "tile too small for 4 waves");
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];  // kQKStages × STAGE
  __shared__ float tokA[kQKRows];
  const rtkv_qk_desc& q = g.q;
  zero_regions(g.ex);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, kg = lane >> 4;
  const int b = blockIdx.y;
  const int S = (int)q.S, H = (int)q.H, grp = (int)(q.H / q.Hkv), P = g.P;
  const int i0 = blockIdx.x * kQKRows;
  const int wrow0 = i0 + wave * 16;                 // first row of this wave
  const int crow0 = wrow0 + 4 * kg;                 // accumulator rows crow0 + reg
  const float l2e = 1.4426950408889634f;
  const float sc = q.scale * l2e;
  const bool masked = (q.causal && q.row0 + wrow0 < PT - 1) || wrow0 + 16 > S || P < PT;

  const S_* Qb = static_cast<const S_*>(q.q_dev) + b * q.q_stride_b;
  const S_* Kb = static_cast<const S_*>(q.k_dev) + b * q.k_stride_b;
  const float* Lb = q.lse_dev + b * q.lse_stride_b;
  // this lane's DMA source row/chunk within an instruction (lane-linear destination)
  const int lrow = lane / CH, lpc = lane % CH;

  auto issue = [&](int h) {
    uint8_t* st = lds + (h % kQKStages) * STAGE;
    const S_* kh = Kb + (int64_t)(h / grp) * q.k_stride_h;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      const int r = (wave * KI + k) * RPI + lrow;          // key row (prompt position)
      const int c = lpc ^ (r & (CH - 1));                  // logical chunk stored at slot lpc
      const int pr = r < P ? r : P - 1;                    // rows past P: any valid row (masked)
      glds16(kh + (int64_t)pr * q.k_stride_s + c * 8, st + (wave * KI + k) * 1024);
    }
    const S_* qh = Qb + (int64_t)h * q.q_stride_h;
#pragma unroll
    for (int k = 0; k < QI; ++k) {
      const int r = (wave * QI + k) * RPI + lrow;          // query row within the block
      const int c = lpc ^ (r & (CH - 1));
      const int gr = i0 + r < S ? i0 + r : S - 1;
      glds16(qh + (int64_t)gr * q.q_stride_s + c * 8, st + KEY_BYTES + (wave * QI + k) * 1024);
    }
    {  // this wave's 16 LSE values (lanes 16..63 idle)
      const int gr = wrow0 + c16 < S ? wrow0 + c16 : S - 1;
      if (lane < 16) glds4(Lb + (int64_t)h * q.lse_stride_h + gr, st + KEY_BYTES + Q_BYTES + wave * 64);
    }
  };

  f32x4 hs[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) hs[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0);
  if (H > 1) issue(1);
  for (int h = 0; h < H; ++h) {
    __builtin_amdgcn_s_barrier();      // every wave is done with head h-1: its slot is free
    if (h + 2 < H) {
      issue(h + 2);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * OPS) : "memory");  // head h landed (this wave)
    } else if (h + 1 < H) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();      // ... and every other wave's pieces of head h too
    const uint8_t* st = lds + (h % kQKStages) * STAGE;
    const uint8_t* qrow = st + KEY_BYTES + (wave * 16 + c16) * RB;
    const int qsw = (wave * 16 + c16) & (CH - 1);
    FT a[KS];
#pragma unroll
    for (int s_ = 0; s_ < KS; ++s_) a[s_] = *reinterpret_cast<const FT*>(qrow + (((4 * s_ + kg) ^ qsw) * 16));
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int kr = 16 * t + c16;
      const uint8_t* krow = st + kr * RB;
#pragma unroll
      for (int s_ = 0; s_ < KS; ++s_) {
        const FT bf = *reinterpret_cast<const FT*>(krow + (((4 * s_ + kg) ^ (kr & (CH - 1))) * 16));
        acc[t] = Frag<DT>::mfma(a[s_], bf, acc[t]);
      }
    }
    const f32x4 lse = *reinterpret_cast<const f32x4*>(st + KEY_BYTES + Q_BYTES + wave * 64 + kg * 16);
    float nl2[4];  // −lse·log2(e): one FMA + exp2 + add per logit
#pragma unroll
    for (int r = 0; r < 4; ++r) nl2[r] = -lse[r] * l2e;
    if (!masked) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) hs[t][r] += __builtin_amdgcn_exp2f(__builtin_fmaf(acc[t][r], sc, nl2[r]));
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int p = 16 * t + c16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = crow0 + r;
          const bool ok = p < P && i < S && (!q.causal || (int64_t)p <= q.row0 + i);
          const float w = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[t][r], sc, nl2[r]));
          hs[t][r] += ok ? w : 0.f;
        }
      }
    }
  }
  // Σ over the P columns: tiles in-lane, then the 16 lanes of each row group
  float rs[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) v += hs[t][r];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
    rs[r] = v / (float)H;
  }
  if (c16 == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = crow0 + r;
      tokA[wave * 16 + 4 * kg + r] = rs[r];
      if (i < S) {
        g.A[(int64_t)b * S + i] = rs[r];
        if (g.ex.t2 && b == 0) {
          const int64_t n = g.ex.row0 + i + 1;  // global position (sequence shards)
          g.ex.t2[i] = g.ex.beta * ((g.ex.S_total > 1) ? torch_logf((uint32_t)n) / g.ex.logS : 0.f);
        }
      }
    }
  }
  if (g.ex.part) {
    __syncthreads();
    if (threadIdx.x == 0) {
      float mn = INFINITY, mx = -INFINITY;
      for (int t = 0; t < kQKRows && i0 + t < S; ++t) { mn = fminf(mn, tokA[t]); mx = fmaxf(mx, tokA[t]); }
      g.ex.part[((int64_t)b * gridDim.x + blockIdx.x) * 2] = mn;
      g.ex.part[((int64_t)b * gridDim.x + blockIdx.x) * 2 + 1] = mx;
    }
  }
}

// Head-major variant (S % 4 == 0, with a [B][H][S] fp32 scratch): a workgroup owns ONE head and a
// block of 4·RPW query rows.  The head's P×D prompt keys are staged in LDS once (32 KiB) and stay
// there; each wave then streams its RPW rows in 16-row tiles, the query fragments and LSE going
// straight to registers in the MFMA A-fragment layout (the next tile in flight while one computes),
// no barrier after the key tile, and writes the 16 rows' per-head sums to the scratch.  qk_head_reduce_kernel sums
// the H heads of each row in head order (deterministic) and does K1's epilogue (β·pos, per-block
// min/max, zeroing).  Against the head-walking kernel above: the keys are staged once per
// workgroup instead of once per head, and 8-16 waves per CU keep queries in flight.
// 4 waves per SIMD: the register budget becomes 128 (no AGPR accumulators, no spills) and 16 waves
// per CU keep their next query tiles in flight (3 waves per SIMD without the bound: 159 registers).
#ifndef QK_HEAD_WPE
#define QK_HEAD_WPE 4
#endif
// (Row-contiguous query loads through a wave-private LDS transpose measured slower: 60 against 49 us per cfg3
// f16 layer at 3 waves per SIMD, profiles/r05_qk_coal_ab.json.)
template <int DT, int NT, int KS>
__global__ __launch_bounds__(256, QK_HEAD_WPE) void qk_head_kernel(QKArgs g, float* __restrict__ part, int rpw) {
  using FT = typename Frag<DT>::T;
  using S_ = typename Dt<DT>::S;
  constexpr int D = 32 * KS;
  constexpr int PT = 16 * NT;
  constexpr int RB = 2 * D;
  constexpr int CH = RB / 16;
  constexpr int RPI = 1024 / RB;
  constexpr int KEY_BYTES = PT * RB;
  constexpr int KI = KEY_BYTES / 1024 / 4;
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];  // KEY_BYTES
  const rtkv_qk_desc& q = g.q;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, kg = lane >> 4;
  const int h = blockIdx.y, b = blockIdx.z;
  const int S = (int)q.S, grp = (int)(q.H / q.Hkv), P = g.P;
  stamp_begin(g.ex.t_begin);
  const int wrow = (blockIdx.x * 4 + wave) * rpw;  // this wave's first row
  const float l2e = 1.4426950408889634f;
  const float sc = q.scale * l2e;
  const S_* Qh = static_cast<const S_*>(q.q_dev) + b * q.q_stride_b + (int64_t)h * q.q_stride_h;
  const float* Lh = q.lse_dev + b * q.lse_stride_b + (int64_t)h * q.lse_stride_h;
  float* Ph = part + ((int64_t)b * q.H + h) * S;
  {  // the head's prompt keys into LDS, swizzled as in qk_importance_kernel
    const S_* kh = static_cast<const S_*>(q.k_dev) + b * q.k_stride_b + (int64_t)(h / grp) * q.k_stride_h;
    const int lrow = lane / CH, lpc = lane % CH;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      const int r = (wave * KI + k) * RPI + lrow;
      const int c = lpc ^ (r & (CH - 1));
      const int pr = r < P ? r : P - 1;
      glds16(kh + (int64_t)pr * q.k_stride_s + c * 8, lds + (wave * KI + k) * 1024);
    }
  }
  // the prompt columns' key bias (raw units; 0 without one), the same for every row
  float kb[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
    kb[t] = (q.kbias_dev && 16 * t + c16 < P) ? key_bias_raw(q, b, 16 * t + c16, 1.f / q.scale) : 0.f;
  const int ntile = rpw / 16;
  auto load_tile = [&](int k, FT (&a)[KS], f32x4& l) {  // tile k of this wave (clamped rows)
    const int r0 = wrow + 16 * (k < ntile ? k : ntile - 1);
    const int qr = r0 + c16 < S ? r0 + c16 : S - 1;
    const S_* qp = Qh + (int64_t)qr * q.q_stride_s;
#pragma unroll
    for (int s_ = 0; s_ < KS; ++s_) a[s_] = *reinterpret_cast<const FT*>(qp + (4 * s_ + kg) * 8);
    const int lr = r0 + 4 * kg < S ? r0 + 4 * kg : S - 4;
    l = *reinterpret_cast<const f32x4*>(Lh + lr);
  };
  FT qa[KS], qn[KS];
  f32x4 ql, qln;
  load_tile(0, qa, ql);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KS + 1) : "memory");  // this wave's key pieces landed
  __syncthreads();                                               // ... and every wave's
  for (int k = 0; k < ntile; ++k) {
    load_tile(k + 1, qn, qln);  // the next tile in flight while this one computes (clamped at the end)
    const int r0 = wrow + 16 * k;
    const int crow0 = r0 + 4 * kg;
    // the key fragments are re-read from LDS for every tile: kept in registers (the compiler would
    // hoist them) they cost 128 VGPRs, and occupancy is what hides the query loads here
    uint32_t kofs = 0;  // opaque zero offset: the LDS reads stay in the loop (and ds_read, not flat)
    asm volatile("" : "+v"(kofs));
    const uint8_t* kt = lds + kofs;
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int kr = 16 * t + c16;
      const uint8_t* krow = kt + kr * RB;
#pragma unroll
      for (int s_ = 0; s_ < KS; ++s_) {
        const FT bf = *reinterpret_cast<const FT*>(krow + (((4 * s_ + kg) ^ (kr & (CH - 1))) * 16));
        acc[t] = Frag<DT>::mfma(qa[s_], bf, acc[t]);
      }
    }
    const int lr = crow0 < S ? crow0 : S - 4;
    float nl2[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = crow0 + r - lr;  // 0..3 except in the clamped tail
      const float lv = e == 0 ? ql[0] : (e == 1 ? ql[1] : (e == 2 ? ql[2] : ql[3]));
      nl2[r] = -lv * l2e;
    }
    const bool masked = (q.causal && q.row0 + r0 < PT - 1) || r0 + 16 > S || P < PT;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (!masked) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += __builtin_amdgcn_exp2f(__builtin_fmaf(acc[t][r] + kb[t], sc, nl2[r]));
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int p = 16 * t + c16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = crow0 + r;
          const bool ok = p < P && i < S && (!q.causal || (int64_t)p <= q.row0 + i);
          const float w = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[t][r] + kb[t], sc, nl2[r]));
          v[r] += ok ? w : 0.f;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) v[r] += __shfl_xor(v[r], o, 64);
      // a row that sees no key (lse = -inf, padding): the reference's all-masked row is uniform over S
      if (nl2[r] == INFINITY) v[r] = (float)P / (float)S;
    }
    if (c16 == 0 && crow0 < S) *reinterpret_cast<f32x4*>(Ph + crow0) = f32x4{v[0], v[1], v[2], v[3]};
#pragma unroll
    for (int s_ = 0; s_ < KS; ++s_) qa[s_] = qn[s_];
    ql = qln;
  }
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
template <int DT> struct Frag32;
template <> struct Frag32<RTKV_F16> {
  using T = f16x8;
  __device__ __forceinline__ static f32x16 mfma(T a, T b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};
template <> struct Frag32<RTKV_BF16> {
  using T = bf16x8;
  __device__ __forceinline__ static f32x16 mfma(T a, T b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};

// Transposed head-major K1' on v_mfma_f32_32x32x16 (D = 128, P <= 128).  The head's prompt keys are
// the A operand (32 prompt columns per MFMA row block, from LDS) and a wave's 32-row query tile the B
// operand (straight from HBM into registers), so the accumulator holds ONE query row per lane (column
// lane & 31) and 16 prompt columns in its registers: the row's LSE is one value per lane, the P-sum is
// in-lane plus one add across the two lane halves (the 16x16x32 kernel above: 4 rows x 4 shuffle
// steps per 16 rows), and every key fragment read from LDS serves 32 query rows instead of 16.
// k order: k-step s takes the 16-byte chunk 2s + h of the row in lane half h, for A and B alike (the
// dot product is the same sum), so a query load instruction reads 32 contiguous bytes of each of 32 rows.
// The wave keeps NB − 1 query tiles in flight beyond the one it computes, in registers (the loop is
// unrolled over the tile buffers, no register copies).  Without a key bias: four waves per SIMD (128
// VGPRs) with one tile ahead, 1024 workgroups — head + reduce 41.6 → 39.0 us per cfg3 f16 layer against
// two waves with two tiles ahead (three waves: 39.5; profiles/r06x_qk_occupancy_ab.txt); with a key bias
// the 128-register form spills (48–89 VGPRs), so that variant keeps two waves per SIMD, two tiles ahead.
// KB: a key bias (padding), kept in LDS as kb[p]·scale·log2(e), added to the row's −lse·log2(e).
template <int DT, bool KB, int NTILE, int NB>
__global__ __launch_bounds__(256, KB ? 2 : 4) void qk_head32_kernel(QKArgs g, float* __restrict__ part) {
  using FT = typename Frag32<DT>::T;
  using S_ = typename Dt<DT>::S;
  constexpr int RB = 256, CH = 16, PT = 128, NT = 4, KS = 8;  // NB query tile buffers (NB - 1 ahead)
  constexpr int KEY_BYTES = PT * RB;
  constexpr int RPI = 1024 / RB;
  constexpr int KI = KEY_BYTES / 1024 / 4;
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];  // keys, then (KB) PT key-bias terms
  float* kbl = reinterpret_cast<float*>(lds + KEY_BYTES);
  const rtkv_qk_desc& q = g.q;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int h = blockIdx.y, b = blockIdx.z;
  const int S = (int)q.S, grp = (int)(q.H / q.Hkv), P = g.P;
  stamp_begin(g.ex.t_begin);
  const int wrow = (blockIdx.x * 4 + wave) * (32 * NTILE);  // this wave's first row
  const float l2e = 1.4426950408889634f;
  const float sc = q.scale * l2e;
  const S_* Qh = static_cast<const S_*>(q.q_dev) + b * q.q_stride_b + (int64_t)h * q.q_stride_h;
  const float* Lh = q.lse_dev + b * q.lse_stride_b + (int64_t)h * q.lse_stride_h;
  float* Ph = part + ((int64_t)b * q.H + h) * S;
  // the head's prompt keys: loaded into registers here, written to LDS below (chunk c of row r at
  // c ^ (r & 15), as qk_head_kernel's LDS-DMA).  Not by LDS-DMA: the compiler then makes the first LDS
  // read wait for every vector load in flight (vmcnt(0)), i.e. for all the query tiles issued ahead.
  FT kreg[KI];
  {
    const S_* kh = static_cast<const S_*>(q.k_dev) + b * q.k_stride_b + (int64_t)(h / grp) * q.k_stride_h;
    const int lrow = lane / CH, lpc = lane % CH;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      const int r = (wave * KI + k) * RPI + lrow;
      const int c = lpc ^ (r & (CH - 1));
      const int pr = r < P ? r : P - 1;
      kreg[k] = *reinterpret_cast<const FT*>(kh + (int64_t)pr * q.k_stride_s + c * 8);
    }
  }
  if constexpr (KB) {
    if (threadIdx.x < PT)
      kbl[threadIdx.x] = (int)threadIdx.x < P ? key_bias_raw(q, b, threadIdx.x, 1.f / q.scale) * sc : 0.f;
  }
  FT qb[NB][KS];
  float ql[NB];
  auto load_tile = [&](int k, FT (&a)[KS], float& l) {  // tile k of this wave (rows clamped to S - 1)
    const int qr = wrow + 32 * k + r32 < S ? wrow + 32 * k + r32 : S - 1;
    const S_* qp = Qh + (int64_t)qr * q.q_stride_s + 8 * hh;
#pragma unroll
    for (int s_ = 0; s_ < KS; ++s_) a[s_] = *reinterpret_cast<const FT*>(qp + 16 * s_);
    l = Lh[qr];
  };
#pragma unroll
  for (int k = 0; k < NB && k < NTILE; ++k) load_tile(k, qb[k], ql[k]);
#pragma unroll
  for (int k = 0; k < KI; ++k) *reinterpret_cast<FT*>(lds + (wave * KI + k) * 1024 + lane * 16) = kreg[k];
  // every wave's key pieces (and key-bias terms) in LDS: a raw barrier after the LDS writes, since
  // __syncthreads would also wait for the query tiles in flight
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  // fully unrolled over the wave's NTILE tiles: the buffer of tile k is k % NB at compile time, and the
  // compiler's wait counts stay exact (a runtime loop over the buffers merged into vmcnt(0))
#pragma unroll
  for (int k = 0; k < NTILE; ++k) {
    const FT (&cur)[KS] = qb[k % NB];
    const int r0 = wrow + 32 * k;
    const int i = r0 + r32;
    const float nl2 = -ql[k % NB] * l2e;
    // columns this lane's row may see: p < P, p <= row0 + i when causal, none past S
    const int lim = i >= S ? 0 : (q.causal && q.row0 + i + 1 < P ? (int)(q.row0 + i + 1) : P);
    const bool masked = (q.causal && q.row0 + r0 < PT - 1) || r0 + 32 > S || P < PT;
    uint32_t kofs = 0;  // opaque zero offset: the LDS reads stay here (and ds_read, not flat)
    asm volatile("" : "+v"(kofs));
    const uint8_t* kt = lds + kofs;
    float hs = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      // a compiler fence per column block: its 8 key fragments (32 VGPRs) are read from LDS just
      // before its MFMAs, not all 32 hoisted together
      asm volatile("" ::: "memory");
      f32x16 acc;
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] = 0.f;
      const int kr = 32 * t + r32;
      const uint8_t* krow = kt + kr * RB;
#pragma unroll
      for (int s_ = 0; s_ < KS; ++s_) {
        const FT af = *reinterpret_cast<const FT*>(krow + (((2 * s_ + hh) ^ (kr & (CH - 1))) * 16));
        acc = Frag32<DT>::mfma(af, cur[s_], acc);
      }
      // acc[j]: prompt column p = 32t + (j & 3) + 8 (j >> 2) + 4 hh of query row i
      float off[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) off[j] = nl2;
      if constexpr (KB) {
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const f32x4 kb4 = *reinterpret_cast<const f32x4*>(kt + 4 * (32 * t + 8 * gq + 4 * hh) + KEY_BYTES);
#pragma unroll
          for (int e = 0; e < 4; ++e) off[4 * gq + e] = nl2 + kb4[e];
        }
      }
      if (!masked) {
#pragma unroll
        for (int j = 0; j < 16; ++j) hs += __builtin_amdgcn_exp2f(__builtin_fmaf(acc[j], sc, off[j]));
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int p = 32 * t + (j & 3) + 8 * (j >> 2) + 4 * hh;
          const float w = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[j], sc, off[j]));
          hs += p < lim ? w : 0.f;
        }
      }
    }
    if (k + NB < NTILE) load_tile(k + NB, qb[k % NB], ql[k % NB]);  // (compile-time condition)
    hs += __shfl_xor(hs, 32, 64);
    // a row that sees no key (lse = -inf, padding): the reference's all-masked row is uniform over S
    if (nl2 == INFINITY) hs = (float)P / (float)S;
    if (hh == 0 && i < S) Ph[i] = hs;
  }
}

// A[b,i] = (Σ_h part[b,h,i]) / H in head order, plus K1's epilogue (β·pos, block min/max, zeroing).
__global__ __launch_bounds__(256) void qk_head_reduce_kernel(const float* __restrict__ part, int64_t H, int64_t S,
                                                             float* __restrict__ A, AggExtras ex) {
  __shared__ float red[2][4];
  zero_regions(ex);
  const int b = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float mn = INFINITY, mx = -INFINITY;
  if (i < S) {
    const float* pp = part + (int64_t)b * H * S + i;
    float s = 0.f;
    int64_t h = 0;
    for (; h + 32 <= H; h += 32) {  // 32 loads in flight, summed in head order
      float v[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) v[j] = __builtin_nontemporal_load(pp + (h + j) * S);
#pragma unroll
      for (int j = 0; j < 32; ++j) s += v[j];
    }
    for (; h + 8 <= H; h += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __builtin_nontemporal_load(pp + (h + j) * S);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; h < H; ++h) s += pp[h * S];
    const float Ai = s / (float)H;
    A[(int64_t)b * S + i] = Ai;
    if (ex.t2 && b == 0) {
      const int64_t n = ex.row0 + i + 1;
      ex.t2[i] = ex.beta * ((ex.S_total > 1) ? torch_logf((uint32_t)n) / ex.logS : 0.f);
    }
    mn = mx = Ai;
  }
  if (ex.part) {
    mn = wave_min(mn);
    mx = wave_max(mx);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) { red[0][wave] = mn; red[1][wave] = mx; }
    __syncthreads();
    if (threadIdx.x == 0) {
      float a = red[0][0], z = red[1][0];
      for (int w = 1; w < (int)(blockDim.x >> 6); ++w) { a = fminf(a, red[0][w]); z = fmaxf(z, red[1][w]); }
      ex.part[((int64_t)b * gridDim.x + blockIdx.x) * 2] = a;
      ex.part[((int64_t)b * gridDim.x + blockIdx.x) * 2 + 1] = z;
    }
  }
}

// one wave per 64 tokens: every token's H loads in flight at once, over S/64 CUs
static int launch_qk_head_reduce(const QKArgs& a, float* part, hipStream_t st, int* nparts) {
  const dim3 rgrid((unsigned)((a.q.S + 63) / 64), (unsigned)a.q.B);
  if (nparts) *nparts = (int)rgrid.x;
  hipLaunchKernelGGL(qk_head_reduce_kernel, rgrid, dim3(64), 0, st, part, a.q.H, a.q.S, a.A, a.ex);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

template <int DT, int NT, int KS>
static int launch_qk_head(const QKArgs& a, float* part, hipStream_t st, int* nparts) {
  const size_t lds = (size_t)(16 * NT) * (64 * KS);
  const int64_t S = a.q.S;
  // rows per wave: 16-row tiles, enough workgroups to fill the chip (>= 1024 with the heads)
  // RTKV_QK_WGS: workgroups to aim for.  1024 (128 rows per wave: the head's 32 KB of keys staged once per
  // 512 rows) measured 47.3 us per cfg3 f16 layer against 49.8 for 2048 and 53.2 for 4096; 8-wave
  // workgroups (the keys once per 8 waves) 54.4 (profiles/r04p_qk_grid_ab.json)
  static const int target = [] {
    const char* e = getenv("RTKV_QK_WGS");
    return e ? atoi(e) : 1024;
  }();
  int rpw = 256;
  while (rpw > 16 && (S + 4 * rpw - 1) / (4 * rpw) * a.q.H * a.q.B < target) rpw /= 2;
  const dim3 grid((unsigned)((S + 4 * rpw - 1) / (4 * rpw)), (unsigned)a.q.H, (unsigned)a.q.B);
  hipLaunchKernelGGL((qk_head_kernel<DT, NT, KS>), grid, dim3(256), lds, st, a, part, rpw);
  RTKV_HIP_CHECK(hipGetLastError());
  QKArgs r = a;
  r.ex.t_begin = nullptr;  // the layer started with the head kernel
  return launch_qk_head_reduce(r, part, st, nparts);
}

template <int DT, int NTILE>
static void launch_qk_head32_n(const QKArgs& a, float* part, hipStream_t st, dim3 grid, size_t lds) {
  // key bias: 3 tile buffers (2 tiles ahead) at two waves per SIMD — 4 buffers measured 43.6 against 42.6 us
  // per cfg3 f16 layer (profiles/r05_qk32_ab.json); none: 2 buffers at four waves per SIMD (above)
  if (a.q.kbias_dev) hipLaunchKernelGGL((qk_head32_kernel<DT, true, NTILE, 3>), grid, dim3(256), lds, st, a, part);
  else hipLaunchKernelGGL((qk_head32_kernel<DT, false, NTILE, 2>), grid, dim3(256), lds, st, a, part);
}

template <int DT>
static int launch_qk_head32(const QKArgs& a, float* part, hipStream_t st, int* nparts) {
  const size_t lds = (size_t)128 * 256 + (a.q.kbias_dev ? 128 * sizeof(float) : 0);
  const int64_t S = a.q.S;
  // 32-row tiles per wave (8, 4, 2 or 1): the most that still gives about RTKV_QK32_WGS workgroups
  // (default: four per CU without a key bias, two with one — the occupancy each variant's registers allow)
  static const int env_target = [] {
    const char* e = getenv("RTKV_QK32_WGS");
    return e ? atoi(e) : 0;
  }();
  const int target = env_target > 0 ? env_target : (a.q.kbias_dev ? 512 : 1024);
  int nt = 8;
  while (nt > 1 && (S + 128 * nt - 1) / (128 * nt) * a.q.H * a.q.B < target) nt /= 2;
  const dim3 grid((unsigned)((S + 128 * nt - 1) / (128 * nt)), (unsigned)a.q.H, (unsigned)a.q.B);
  if (nt == 8) launch_qk_head32_n<DT, 8>(a, part, st, grid, lds);
  else if (nt == 4) launch_qk_head32_n<DT, 4>(a, part, st, grid, lds);
  else if (nt == 2) launch_qk_head32_n<DT, 2>(a, part, st, grid, lds);
  else launch_qk_head32_n<DT, 1>(a, part, st, grid, lds);
  RTKV_HIP_CHECK(hipGetLastError());
  QKArgs r = a;
  r.ex.t_begin = nullptr;  // the layer started with the head kernel
  return launch_qk_head_reduce(r, part, st, nparts);
}

template <int DT, int NT, int KS>
static int launch_qk_tpl(const QKArgs& a, dim3 grid, hipStream_t st) {
  constexpr size_t lds = (size_t)kQKStages * ((size_t)(16 * NT) * (64 * KS) + (size_t)kQKRows * (64 * KS) + kQKRows * 4);
  static bool attr = false;
  if (!attr) {
    RTKV_HIP_CHECK(hipFuncSetAttribute((const void*)qk_importance_kernel<DT, NT, KS>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  hipLaunchKernelGGL((qk_importance_kernel<DT, NT, KS>), grid, dim3(256), lds, st, a);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

template <int DT>
static int launch_qk_dt(const QKArgs& a, dim3 grid, hipStream_t st) {
  const int ks = (int)(a.q.D / 32);
  int nt = a.P <= 32 ? 2 : (a.P <= 64 ? 4 : 8);
  if (nt * ks < 4) nt = 4 / ks;  // at least one 4 KiB key DMA round per head
#define RTKV_QK(N, K) \
  if (nt == N && ks == K) return launch_qk_tpl<DT, N, K>(a, grid, st);
  RTKV_QK(4, 1) RTKV_QK(8, 1)
  RTKV_QK(2, 2) RTKV_QK(4, 2) RTKV_QK(8, 2)
  RTKV_QK(2, 4) RTKV_QK(4, 4) RTKV_QK(8, 4)
#undef RTKV_QK
  RTKV_REQUIRE(false, "importance_qk_lse: unsupported head_dim");
}

size_t qk_scratch_bytes(int64_t B, int64_t H, int64_t S) { return (size_t)(B * H * S) * sizeof(float); }

int launch_qk_importance(const rtkv_qk_desc& q, int P, float* A, hipStream_t st, const AggExtras& x, int* nparts,
                         float* scratch, size_t scratch_bytes) {
  RTKV_REQUIRE(q.q_dev && q.k_dev && q.lse_dev && A, "importance_qk_lse: null pointer");
  RTKV_REQUIRE(q.B >= 1 && q.B <= 65535 && q.H >= 1 && q.S >= 4 && q.Hkv >= 1, "importance_qk_lse: bad shape (S >= 4)");
  RTKV_REQUIRE(q.H % q.Hkv == 0, "importance_qk_lse: H must be a multiple of Hkv");
  RTKV_REQUIRE(q.D == 32 || q.D == 64 || q.D == 128, "importance_qk_lse: head_dim must be 32, 64 or 128");
  RTKV_REQUIRE(P >= 1 && P <= 128, "importance_qk_lse: prompt_len must be in [1, 128]");
  RTKV_REQUIRE(q.dtype == RTKV_F16 || q.dtype == RTKV_BF16 || q.dtype == RTKV_F32,
               "importance_qk_lse: Q/K must be float16, bfloat16 or float32");
  RTKV_REQUIRE(((uintptr_t)q.lse_dev % 16) == 0 && q.lse_stride_h % 4 == 0 && q.lse_stride_b % 4 == 0,
               "importance_qk_lse: lse rows must be 16-byte aligned");
  RTKV_REQUIRE(q.S < ((int64_t)1 << 31) && q.row0 >= 0, "importance_qk_lse: bad row range");
  RTKV_REQUIRE(!q.kbias_dev || q.row0 == 0, "importance_qk_lse: key bias with row0 != 0");
  QKArgs a;
  a.q = q;
  a.P = P;
  a.A = A;
  a.ex = x;
  const bool head_ok = scratch && scratch_bytes >= qk_scratch_bytes(q.B, q.H, q.S) && q.H <= 65535 && q.D == 128;
  if (q.dtype == RTKV_F32) {  // fp32 states: the head-major kernel on the f32 MFMA (attn_f32.hip)
    RTKV_REQUIRE(head_ok, "importance_qk_lse (fp32): needs head_dim 128 and the head-major scratch "
                          "(rtkv_importance_qk_lse_ws / rtkv_workspace_size_qk)");
    const int rc = launch_qk_head_f32(q, P, scratch, st, a.ex.t_begin);
    if (rc) return rc;
    QKArgs r = a;
    r.ex.t_begin = nullptr;  // the layer started with the head kernel
    return launch_qk_head_reduce(r, scratch, st, nparts);
  }
  RTKV_REQUIRE(q.q_stride_s % 8 == 0 && q.q_stride_h % 8 == 0 && q.q_stride_b % 8 == 0 && q.k_stride_s % 8 == 0 &&
                   q.k_stride_h % 8 == 0 && q.k_stride_b % 8 == 0 && ((uintptr_t)q.q_dev % 16) == 0 &&
                   ((uintptr_t)q.k_dev % 16) == 0,
               "importance_qk_lse: Q/K rows must be 16-byte aligned");
  // head-major kernel when a scratch is given (the C ABI entries that take a workspace); RTKV_QK_RING
  // forces the head-walking kernel (cross-check knob).  A key bias (padding) is applied by the
  // head-major kernel only.
  static const bool ring = getenv("RTKV_QK_RING") != nullptr;
  if (q.kbias_dev)
    RTKV_REQUIRE(head_ok && q.S % 4 == 0, "importance_qk_lse: a key bias needs head_dim 128, S % 4 == 0 and the "
                                          "head-major scratch");
  if (head_ok && q.S % 4 == 0 && ((!ring && P > 64) || q.kbias_dev)) {
    // the 32x32x16 transposed kernel: 42.6 against 47.6 us per cfg3 f16 layer for the 16x16x32 one
    // (head + reduce, profiles/r05_qk32_ab.json); RTKV_QK16 keeps the latter as a cross-check
    static const bool k16 = getenv("RTKV_QK16") != nullptr;
    if (!k16) {
      if (q.dtype == RTKV_F16) return launch_qk_head32<RTKV_F16>(a, scratch, st, nparts);
      return launch_qk_head32<RTKV_BF16>(a, scratch, st, nparts);
    }
    if (q.dtype == RTKV_F16) return launch_qk_head<RTKV_F16, 8, 4>(a, scratch, st, nparts);
    return launch_qk_head<RTKV_BF16, 8, 4>(a, scratch, st, nparts);
  }
  const dim3 grid((unsigned)((q.S + kQKRows - 1) / kQKRows), (unsigned)q.B);
  if (nparts) *nparts = (int)grid.x;
  if (q.dtype == RTKV_F16) return launch_qk_dt<RTKV_F16>(a, grid, st);
  return launch_qk_dt<RTKV_BF16>(a, grid, st);
}

}  // namespace rtkv
