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
// The Q·K_Pᵀ contraction runs on MFMA (v_mfma_f32_32x32x16_{f16,bf16}): a workgroup owns 32 query
// rows; its 4 waves split the heads (h ≡ wave mod 4) and each wave computes the full 32 × P tile
// (P ≤ 128: up to four 32×32 accumulators) per head, k-stepping over D in 16s.  Fragment maps
// (cdna_hip_programming.md §3): lane l, r = l & 31, hh = l >> 5 holds A[row r][k 8hh..8hh+7] and
// B[k 8hh..8hh+7][col r]; the accumulator holds col r, rows (reg & 3) + 8(reg >> 2) + 4hh.  The
// exp and the head sum stay in registers; one LDS reduction over the 4 waves ends the block.
#include "common.h"

namespace rtkv {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct QKArgs {
  rtkv_qk_desc q;
  int P;
  float* A;
  AggExtras ex;
};

template <int DT> struct Frag;
template <> struct Frag<RTKV_F16> {
  using T = f16x8;
  __device__ __forceinline__ static f32x16 mfma(T a, T b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};
template <> struct Frag<RTKV_BF16> {
  using T = bf16x8;
  __device__ __forceinline__ static f32x16 mfma(T a, T b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};

constexpr int kQKRows = 32;   // query rows per workgroup
constexpr int kQKWaves = 4;   // head split

template <int DT, int NT>
__global__ __launch_bounds__(256) void qk_importance_kernel(QKArgs g) {
  using FT = typename Frag<DT>::T;
  using S_ = typename Dt<DT>::S;
  const rtkv_qk_desc& q = g.q;
  __shared__ float red[kQKWaves][kQKRows];
  __shared__ float tokA[kQKRows];
  zero_regions(g.ex);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int b = blockIdx.y;
  const int64_t i0 = (int64_t)blockIdx.x * kQKRows;
  const int H = (int)q.H, grp = (int)(q.H / q.Hkv), P = g.P, D = (int)q.D;
  const int64_t S = q.S;
  // this lane's A-operand row and its 16 accumulator rows
  const int64_t arow = i0 + r < S ? i0 + r : S - 1;
  int64_t crow[16];
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) crow[reg] = i0 + (reg & 3) + 8 * (reg >> 2) + 4 * hh;
  const float l2e = 1.4426950408889634f;
  const float sc = q.scale * l2e;
  float hs[NT][16];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) hs[t][reg] = 0.f;

  const S_* Qb = static_cast<const S_*>(q.q_dev) + b * q.q_stride_b + arow * q.q_stride_s + 8 * hh;
  const S_* Kb = static_cast<const S_*>(q.k_dev) + b * q.k_stride_b + 8 * hh;
  for (int h = wave; h < H; h += kQKWaves) {
    const S_* qrow = Qb + (int64_t)h * q.q_stride_h;
    const S_* kbase = Kb + (int64_t)(h / grp) * q.k_stride_h;
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
    for (int s = 0; s < D; s += 16) {
      const FT a = *reinterpret_cast<const FT*>(qrow + s);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int p = t * 32 + r;
        const FT bf = p < P ? *reinterpret_cast<const FT*>(kbase + (int64_t)p * q.k_stride_s + s) : FT{};
        acc[t] = Frag<DT>::mfma(a, bf, acc[t]);
      }
    }
    // W = exp(x·scale − lse) = exp2(x·scale·log2e − lse·log2e); masked columns / rows contribute 0
    const float* lrow = q.lse_dev + b * q.lse_stride_b + (int64_t)h * q.lse_stride_h;
    float lse2[16];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) lse2[reg] = crow[reg] < S ? lrow[crow[reg]] * l2e : 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int p = t * 32 + r;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const bool ok = p < P && crow[reg] < S && (!q.causal || p <= q.row0 + crow[reg]);
        const float w = __builtin_amdgcn_exp2f(acc[t][reg] * sc - lse2[reg]);
        hs[t][reg] += ok ? w : 0.f;
      }
    }
  }
  // Σ over the P columns: the tiles in-lane, then the 32 lanes of each half (one column each)
  float rs[16];
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    float v = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) v += hs[t][reg];
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);
    rs[reg] = v;
  }
  if (r == 0) {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) red[wave][(reg & 3) + 8 * (reg >> 2) + 4 * hh] = rs[reg];
  }
  __syncthreads();
  if (threadIdx.x < kQKRows) {
    const int64_t i = i0 + threadIdx.x;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < kQKWaves; ++w) v += red[w][threadIdx.x];
    v = v / (float)H;
    tokA[threadIdx.x] = v;
    if (i < S) {
      g.A[(int64_t)b * S + i] = v;
      if (g.ex.t2 && b == 0) {
        const int64_t n = g.ex.row0 + i + 1;  // global position (sequence shards)
        g.ex.t2[i] = g.ex.beta * ((g.ex.S_total > 1) ? torch_logf((uint32_t)n) / g.ex.logS : 0.f);
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

template <int DT>
static int launch_qk_dt(const QKArgs& a, dim3 grid, hipStream_t st) {
  const int nt = (a.P + 31) / 32;
  switch (nt) {
    case 1: hipLaunchKernelGGL((qk_importance_kernel<DT, 1>), grid, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((qk_importance_kernel<DT, 2>), grid, dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL((qk_importance_kernel<DT, 3>), grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((qk_importance_kernel<DT, 4>), grid, dim3(256), 0, st, a); break;
  }
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

int launch_qk_importance(const rtkv_qk_desc& q, int P, float* A, hipStream_t st, const AggExtras& x, int* nparts) {
  RTKV_REQUIRE(q.q_dev && q.k_dev && q.lse_dev && A, "importance_qk_lse: null pointer");
  RTKV_REQUIRE(q.B >= 1 && q.B <= 65535 && q.H >= 1 && q.S >= 1 && q.Hkv >= 1, "importance_qk_lse: bad shape");
  RTKV_REQUIRE(q.H % q.Hkv == 0, "importance_qk_lse: H must be a multiple of Hkv");
  RTKV_REQUIRE(q.D >= 16 && q.D % 16 == 0 && q.D <= 512, "importance_qk_lse: head_dim must be a multiple of 16 (<= 512)");
  RTKV_REQUIRE(P >= 1 && P <= 128, "importance_qk_lse: prompt_len must be in [1, 128]");
  RTKV_REQUIRE(q.dtype == RTKV_F16 || q.dtype == RTKV_BF16, "importance_qk_lse: Q/K must be float16 or bfloat16");
  RTKV_REQUIRE(q.q_stride_s % 8 == 0 && q.q_stride_h % 8 == 0 && q.q_stride_b % 8 == 0 && q.k_stride_s % 8 == 0 &&
                   q.k_stride_h % 8 == 0 && q.k_stride_b % 8 == 0 && ((uintptr_t)q.q_dev % 16) == 0 &&
                   ((uintptr_t)q.k_dev % 16) == 0,
               "importance_qk_lse: Q/K rows must be 16-byte aligned");
  RTKV_REQUIRE(q.S < ((int64_t)1 << 31) && q.row0 >= 0, "importance_qk_lse: bad row range");
  QKArgs a;
  a.q = q;
  a.P = P;
  a.A = A;
  a.ex = x;
  const dim3 grid((unsigned)((q.S + kQKRows - 1) / kQKRows), (unsigned)q.B);
  if (nparts) *nparts = (int)grid.x;
  if (q.dtype == RTKV_F16) return launch_qk_dt<RTKV_F16>(a, grid, st);
  return launch_qk_dt<RTKV_BF16>(a, grid, st);
}

}  // namespace rtkv
