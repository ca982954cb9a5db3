// attn_lse.hip — the row log-sum-exp of the prefill attention, the one quantity the fused importance
// mode (K1', qk_importance.hip) needs besides Q and the prompt keys:
//
//   lse[b,h,i] = log Σ_{j ≤ i (causal), j < S} exp(q[b,h,i]·k[b,h/g,j]·scale)
//
// i.e. the normaliser of the reference's softmax(Q·Kᵀ/√d + mask) (modified_llama.py:88-94) without
// materialising the [B,H,S,S] matrix.  fp32 accumulation; parity with a torch fp32 logsumexp is a
// tolerance (tests/test_gpu_lse.py).
//
// Work decomposition (gfx950, wave64): a workgroup owns 64·RG query rows of one (b, h), RG groups
// of 16 rows per wave (RG = 1 by default); it walks the key tiles of 64 rows up to the causal
// diagonal, each tile staged in LDS by LDS-DMA (double-buffered, swizzled as in qk_importance.hip)
// and shared by the 4 waves.  Each wave computes its 16·RG × 64 logits with
// v_mfma_f32_16x16x32_{f16,bf16} (RG row groups × 4 column tiles × D/32 k-steps; each key fragment
// read from LDS feeds every row group);
// every lane keeps a running (max, sum) per accumulator row over the key columns it holds, in the
// exp2 domain with a lazily raised max (rescale only when a logit passes it by 8: one wave-uniform
// branch per tile).  The 16 lanes of a row combine at the end.  Workgroups are issued longest-first
// (the last query blocks carry the most key tiles).
#include "common.h"

#include <cstdlib>

namespace rtkv {

int launch_attention_lse32(const rtkv_qk_desc& q, float* lse, hipStream_t st);  // attn_lse32.hip

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int DT> struct LFrag;
template <> struct LFrag<RTKV_F16> {
  using T = f16x8;
  __device__ __forceinline__ static f32x4 mfma(T a, T b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
template <> struct LFrag<RTKV_BF16> {
  using T = bf16x8;
  __device__ __forceinline__ static f32x4 mfma(T a, T b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};

constexpr int kLKeys = 64;   // key rows per tile
constexpr float kLSlack = 8.f;
constexpr float kLFloor = -1e30f;  // initial running max

struct LseArgs {
  rtkv_qk_desc q;
  float* lse;
  int nblk;       // query blocks per (b, h)
  int fixup = 0;  // recompute only the row blocks whose lse is +inf / NaN (after attn_lse32_kernel)
};

__device__ __forceinline__ void lds_dma16(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// One row group per wave fits 96 registers: 5 waves per SIMD (4 without the bound, at 98).
#ifndef LSE_WPE
#define LSE_WPE 5
#endif
template <int DT, int KS, int RG>
__global__ __launch_bounds__(256, RG == 1 ? LSE_WPE : 1) void attn_lse_kernel(LseArgs g) {
  constexpr int kLRows = 64 * RG;            // query rows per workgroup (4 waves × RG groups of 16)
  using FT = typename LFrag<DT>::T;
  using S_ = typename Dt<DT>::S;
  constexpr int D = 32 * KS;
  constexpr int RB = 2 * D;                  // bytes per key row
  constexpr int CH = RB / 16;                // 16-byte chunks per row
  constexpr int RPI = 1024 / RB;             // rows per DMA wave-instruction
  constexpr int TILE = kLKeys * RB;          // bytes per key tile
  constexpr int KI = TILE / 1024 / 4;        // DMA instructions per wave per tile
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];  // 2 × TILE
  const rtkv_qk_desc& q = g.q;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, kg = lane >> 4;
  // XCD-aware order (as attn_lse32.hip): each XCD runs whole heads, longest query block first
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
  const int i0 = qb * kLRows;
  const int wrow0 = i0 + wave * 16 * RG;     // the wave's rows: RG groups of 16 from here
  if (g.fixup) {  // the fix-up pass of attn_lse32.hip: blocks whose every lse is valid end here
    int bad = 0;
    if ((int)threadIdx.x < kLRows && i0 + (int)threadIdx.x < S) {
      const float v = g.lse[b * q.lse_stride_b + (int64_t)h * q.lse_stride_h + i0 + threadIdx.x];
      bad = v != v || v == INFINITY;
    }
    if (!__syncthreads_or(bad)) return;
  }
  const float sc = q.scale * 1.4426950408889634f, inv_scale = 1.f / q.scale;
  const S_* Kh = static_cast<const S_*>(q.k_dev) + b * q.k_stride_b + (int64_t)(h / grp) * q.k_stride_h;
  // key rows this block needs: causal → up to its last query row (global position row0 + i)
  int64_t kend = q.causal ? q.row0 + i0 + kLRows : S;
  if (kend > S) kend = S;
  const int ntiles = (int)((kend + kLKeys - 1) / kLKeys);
  const int lrow = lane / CH, lpc = lane % CH;
  auto issue = [&](int kt) {
    uint8_t* st = lds + (kt & 1) * TILE;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      const int r = (wave * KI + k) * RPI + lrow;
      const int c = lpc ^ (r & (CH - 1));
      int kr = kt * kLKeys + r;
      kr = kr < S ? kr : S - 1;              // rows past S: any valid row (masked)
      lds_dma16(Kh + (int64_t)kr * q.k_stride_s + c * 8, st + (wave * KI + k) * 1024);
    }
  };
  // the wave's 32 query rows, A fragments straight from global (once); each key fragment read from
  // LDS feeds both row groups (half the LDS traffic per flop of one group per wave)
  FT a[RG][KS];
#pragma unroll
  for (int rg = 0; rg < RG; ++rg) {
    const int qr = wrow0 + 16 * rg + c16 < S ? wrow0 + 16 * rg + c16 : S - 1;
    const S_* qrow = static_cast<const S_*>(q.q_dev) + b * q.q_stride_b + (int64_t)h * q.q_stride_h +
                     (int64_t)qr * q.q_stride_s;
#pragma unroll
    for (int s_ = 0; s_ < KS; ++s_) a[rg][s_] = *reinterpret_cast<const FT*>(qrow + (4 * s_ + kg) * 8);
  }
  float m[RG][4], l[RG][4];
#pragma unroll
  for (int rg = 0; rg < RG; ++rg)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      m[rg][r] = kLFloor;  // finite: exp2(-inf − m) = 0 and no −inf − (−inf)
      l[rg][r] = 0.f;
    }
  // Software pipeline: the MFMAs of key tile kt+1 are issued in the same basic block as tile kt's
  // exp2 sums (independent registers), and sched_group_barrier interleaves them — 1 LDS read, 1 MFMA,
  // 4 VALU — so the matrix core and the VALU work at once inside each wave.
  auto mfma_tile = [&](int kt, f32x4 (&acc)[RG][4]) {
    const uint8_t* st = lds + (kt & 1) * TILE;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) acc[rg][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int kr = 16 * t + c16;
      const uint8_t* krow = st + kr * RB;
#pragma unroll
      for (int s_ = 0; s_ < KS; ++s_) {
        const FT bf = *reinterpret_cast<const FT*>(krow + (((4 * s_ + kg) ^ (kr & (CH - 1))) * 16));
#pragma unroll
        for (int rg = 0; rg < RG; ++rg) acc[rg][t] = LFrag<DT>::mfma(a[rg][s_], bf, acc[rg][t]);
      }
    }
  };
  // tile kt's logits: mask keys past S and (causal) past the query position (edge tiles only), raise
  // the running max when a logit passes it by 8 (one wave-uniform branch)
  auto prepare = [&](f32x4 (&acc)[RG][4], int kt) {
    bool up = false;
    float mt[RG][4];
    if (q.kbias_dev) {  // key padding: the bias of this tile's columns (raw units), -inf for a padding key
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int j = kt * kLKeys + 16 * t + c16;
        const float kb = j < S ? key_bias_raw(q, b, j, inv_scale) : 0.f;
#pragma unroll
        for (int rg = 0; rg < RG; ++rg)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[rg][t][r] += kb;
      }
    }
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {
      const int grow0 = wrow0 + 16 * rg;      // first row of the group
      const int crow0 = grow0 + 4 * kg;       // accumulator rows crow0 + r
      const bool edge = (int64_t)(kt + 1) * kLKeys > (q.causal ? q.row0 + grow0 : (int64_t)S) || (kt + 1) * kLKeys > S;
      if (edge) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int j = kt * kLKeys + 16 * t + c16;
            const bool ok = j < S && (!q.causal || (int64_t)j <= q.row0 + crow0 + r);
            acc[rg][t][r] = ok ? acc[rg][t][r] : -INFINITY;
          }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        mt[rg][r] = fmaxf(fmaxf(acc[rg][0][r], acc[rg][1][r]), fmaxf(acc[rg][2][r], acc[rg][3][r])) * sc;
        up |= mt[rg][r] > m[rg][r] + kLSlack;
      }
    }
    if (__ballot(up)) {
#pragma unroll
      for (int rg = 0; rg < RG; ++rg)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float mn = mt[rg][r] > m[rg][r] + kLSlack ? mt[rg][r] : m[rg][r];
          l[rg][r] *= __builtin_amdgcn_exp2f(m[rg][r] - mn);
          m[rg][r] = mn;
        }
    }
  };
  auto exp_sum = [&](const f32x4 (&acc)[RG][4]) {
#pragma unroll
    for (int rg = 0; rg < RG; ++rg)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float nm = -m[rg][r];
#pragma unroll
        for (int t = 0; t < 4; ++t) l[rg][r] += __builtin_amdgcn_exp2f(__builtin_fmaf(acc[rg][t][r], sc, nm));
      }
  };
  f32x4 acc[RG][4], accn[RG][4];
  issue(0);
  if (ntiles > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KI) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();  // every wave's pieces of tile 0
  mfma_tile(0, acc);
  for (int kt = 0; kt < ntiles; ++kt) {
    prepare(acc, kt);
    if (kt + 1 < ntiles) {
      __builtin_amdgcn_s_barrier();  // every wave has read tile kt (its MFMAs are issued): slot kt&1 is free
      if (kt + 2 < ntiles) {
        issue(kt + 2);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KI) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();  // ... and every wave's pieces of tile kt+1 landed
      mfma_tile(kt + 1, accn);
      exp_sum(acc);
#pragma unroll
      for (int i = 0; i < 4 * KS * RG; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 LDS read
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // 4 VALU
      }
#pragma unroll
      for (int rg = 0; rg < RG; ++rg)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[rg][t] = accn[rg][t];
    } else {
      exp_sum(acc);
    }
  }
  // combine the 16 lanes holding each row: M = max m, L = Σ l·2^(m − M); lse = (M + log2 L)·ln 2
#pragma unroll
  for (int rg = 0; rg < RG; ++rg)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float M = m[rg][r];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) M = fmaxf(M, __shfl_xor(M, o, 64));
    float L = l[rg][r] * __builtin_amdgcn_exp2f(m[rg][r] - M);
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) L += __shfl_xor(L, o, 64);
    const int i = wrow0 + 16 * rg + 4 * kg + r;
    if (c16 == 0 && i < S)
      g.lse[b * q.lse_stride_b + (int64_t)h * q.lse_stride_h + i] =
          L > 0.f ? (M + __log2f(L)) * 0.6931471805599453f : -INFINITY;
  }
}

template <int DT, int KS, int RG>
int launch_lse_tpl(LseArgs a, const rtkv_qk_desc& q, hipStream_t st) {
  constexpr size_t lds = 2 * (size_t)kLKeys * (64 * KS);
  a.nblk = (int)((q.S + 64 * RG - 1) / (64 * RG));
  const dim3 grid((unsigned)a.nblk, (unsigned)q.H, (unsigned)q.B);
  hipLaunchKernelGGL((attn_lse_kernel<DT, KS, RG>), grid, dim3(256), lds, st, a);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

int lse_row_groups() {
  static const int v = [] {  // tuning knob RTKV_LSE_RG (1 or 2 row groups of 16 per wave)
    const char* e = std::getenv("RTKV_LSE_RG");
    return e && std::atoi(e) == 2 ? 2 : 1;
  }();
  return v;
}

}  // namespace

int launch_attention_lse(const rtkv_qk_desc& q, float* lse, hipStream_t st) {
  RTKV_REQUIRE(q.q_dev && q.k_dev && lse, "attention_lse: null pointer");
  RTKV_REQUIRE(q.B >= 1 && q.B <= 65535 && q.H >= 1 && q.H <= 65535 && q.S >= 1 && q.Hkv >= 1,
               "attention_lse: bad shape");
  RTKV_REQUIRE(q.H % q.Hkv == 0, "attention_lse: H must be a multiple of Hkv");
  RTKV_REQUIRE(q.D == 64 || q.D == 128, "attention_lse: head_dim must be 64 or 128");
  RTKV_REQUIRE(q.scale > 0.f, "attention_lse: scale must be positive");
  RTKV_REQUIRE(q.S < ((int64_t)1 << 31) && q.row0 == 0, "attention_lse: bad row range (row0 must be 0)");
  RTKV_REQUIRE(q.dtype == RTKV_F16 || q.dtype == RTKV_BF16 || q.dtype == RTKV_F32,
               "attention_lse: Q/K must be float16, bfloat16 or float32");
  if (q.dtype == RTKV_F32) return launch_attention_lse_f32(q, lse, st);
  RTKV_REQUIRE(q.q_stride_s % 8 == 0 && q.q_stride_h % 8 == 0 && q.q_stride_b % 8 == 0 && q.k_stride_s % 8 == 0 &&
                   q.k_stride_h % 8 == 0 && q.k_stride_b % 8 == 0 && ((uintptr_t)q.q_dev % 16) == 0 &&
                   ((uintptr_t)q.k_dev % 16) == 0,
               "attention_lse: Q/K rows must be 16-byte aligned");
  // head_dim 128: the 32x32x16 tiling (attn_lse32.hip); RTKV_LSE_KERNEL=16 keeps the 16x16x32 one
  // (measurement knob)
  static const bool t16 = [] {
    const char* e = std::getenv("RTKV_LSE_KERNEL");
    return e && std::atoi(e) == 16;
  }();
  LseArgs a;
  a.q = q;
  a.lse = lse;
  if (q.D == 128 && !t16) {
    const int rc = launch_attention_lse32(q, lse, st);
    if (rc) return rc;
    a.fixup = 1;  // rows whose unchecked sum overflowed: recomputed by the checked kernel
    if (q.dtype == RTKV_F16) return launch_lse_tpl<RTKV_F16, 4, 1>(a, q, st);
    return launch_lse_tpl<RTKV_BF16, 4, 1>(a, q, st);
  }
  const int ks = (int)(q.D / 32), rg = lse_row_groups();
#define RTKV_L(DT, K, R) \
  if (q.dtype == DT && ks == K && rg == R) return launch_lse_tpl<DT, K, R>(a, q, st);
  RTKV_L(RTKV_F16, 4, 1) RTKV_L(RTKV_F16, 2, 1) RTKV_L(RTKV_BF16, 4, 1) RTKV_L(RTKV_BF16, 2, 1)
  RTKV_L(RTKV_F16, 4, 2) RTKV_L(RTKV_F16, 2, 2) RTKV_L(RTKV_BF16, 4, 2) RTKV_L(RTKV_BF16, 2, 2)
#undef RTKV_L
  RTKV_REQUIRE(false, "attention_lse: unsupported configuration");
}

}  // namespace rtkv
