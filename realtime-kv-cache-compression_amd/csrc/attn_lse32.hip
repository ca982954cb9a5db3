// attn_lse32.hip — the row log-sum-exp of attn_lse.hip (same result, same contract) for head_dim 128
// on the 32x32x16 MFMA (v_mfma_f32_32x32x16_{f16,bf16}).
//
// Why a second tiling: the LSE is QKᵀ followed by one exp2 + add per logit, so its VALU work per
// MFMA flop is high and the 16x16x32 tiling of attn_lse.hip is issue-bound: a 16x16x32 MFMA holds
// the SIMD's vector issue for 8 of its 16 cycles, a 32x32x16 for 8 of 32 (MI355X_MICROARCH.md,
// constants table), and a 32-row wave tile reads each key fragment from LDS once for twice the rows.
//
// Work decomposition: a workgroup owns 128 query rows of one (b, h) — 4 waves × 32 rows — and walks
// key tiles of 64 rows (2 column blocks of 32) up to its causal diagonal, each tile staged in LDS by
// LDS-DMA (a 3-slot ring, one barrier per tile; 16-byte chunks XOR-swizzled by row, conflict-free for the B reads).  A
// wave skips the MFMAs of tiles past its own last row.  Fragments (cdna_hip_programming.md): lane l
// (r = l&31, h = l>>5) holds A[row r][k = 8h + j] and B[k = 8h + j][col r]; k-step s covers the head
// dims of chunk 2s + h (a permutation of the dot product's terms, as in attn_lse.hip); the 16
// accumulator registers of a lane hold column r, rows (reg&3) + 8(reg>>2) + 4h.
//
// Softmax bookkeeping with no per-logit check: each (lane, row) takes its first finite logit as its
// reference max and sums exp2(x − m) against it unchecked from then on (fma + exp2 + add per logit;
// the lazy max raise of attn_lse.hip runs only while some row of the wave still has no reference,
// e.g. rows before their first unmasked key).  The reference is a real logit of the row, so the sum
// cannot underflow to 0; it overflows only when a later logit exceeds the first one by ~100 in log2
// units (x − m > 128 for one exp2, or a sum past 2^128).  Such a row gets a non-finite lse (+inf or
// NaN), and the fix-up launch after this kernel (attn_lse_kernel with `fixup`, attn_lse.hip)
// recomputes every 64-row block holding one with the checked algorithm.  The 32 lanes of a row combine
// at the end.
#include "common.h"

namespace rtkv {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int DT> struct L32;
template <> struct L32<RTKV_F16> {
  using T = f16x8;
  __device__ __forceinline__ static f32x16 mfma(T a, T b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};
template <> struct L32<RTKV_BF16> {
  using T = bf16x8;
  __device__ __forceinline__ static f32x16 mfma(T a, T b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};

constexpr int kD = 128;
constexpr int kRB = kD * 2;           // bytes per key row
constexpr int kCH = kRB / 16;         // 16-byte chunks per row
constexpr int kKeys = 64;             // key rows per LDS tile
constexpr int kTile = kKeys * kRB;    // 16 KiB
constexpr int kKI = kTile / 1024 / 4; // DMA instructions per wave per tile
constexpr int kRPI = 1024 / kRB;      // key rows per DMA instruction
constexpr int kRows = 128;            // query rows per workgroup
constexpr float kSlack = 8.f;
constexpr float kFloor = -1e30f;

struct Lse32Args {
  rtkv_qk_desc q;
  float* lse;
  int nblk;
};

__device__ __forceinline__ void dma16(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

template <int DT>
__global__ __launch_bounds__(256, 3) void attn_lse32_kernel(Lse32Args g) {
  using FT = typename L32<DT>::T;
  using S_ = typename Dt<DT>::S;
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];  // 3 × kTile
  const rtkv_qk_desc& q = g.q;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  // XCD-aware order (cdna_hip_programming.md T1): workgroups are dealt round-robin over the 8 XCDs, so
  // the default order spreads every head's query blocks over all 8 L2s and each L2 cycles through the
  // keys of many heads.  Remapped, XCD x runs a contiguous range of (head, query block) units — whole
  // heads, longest query block first — and a head's keys (S·256 B) stay in its XCD's L2.
  int qb, hd, b;
  {
    const int nwg = (int)(gridDim.x * gridDim.y * gridDim.z);
    int bid = (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
    if ((nwg & 7) == 0) bid = (bid & 7) * (nwg >> 3) + (bid >> 3);
    const int unit = bid / g.nblk;  // (b, h) pair
    qb = g.nblk - 1 - (bid - unit * g.nblk);  // longest-first within the head
    hd = unit % (int)gridDim.y;
    b = unit / (int)gridDim.y;
  }
  const int S = (int)q.S, grp = (int)(q.H / q.Hkv);
  const int i0 = qb * kRows, wrow0 = i0 + 32 * wave;
  const float sc = q.scale * 1.4426950408889634f, inv_scale = 1.f / q.scale;
  const S_* Kh = static_cast<const S_*>(q.k_dev) + b * q.k_stride_b + (int64_t)(hd / grp) * q.k_stride_h;
  // (row0 == 0: launch_attention_lse requires it)
  const int kend = q.causal ? min(S, i0 + kRows) : S;
  const int ntiles = (kend + kKeys - 1) / kKeys;
  // keys past this wave's last row are masked for all its rows (causal): their tiles are skipped
  const int wave_last = q.causal ? wrow0 + 31 : S;
  const int lrow = lane / kCH, lpc = lane % kCH;
  auto issue = [&](int kt) {
    uint8_t* st = lds + (kt % 3) * kTile;
#pragma unroll
    for (int k = 0; k < kKI; ++k) {
      const int r = (wave * kKI + k) * kRPI + lrow;
      const int c = lpc ^ (r & (kCH - 1));
      int kr = kt * kKeys + r;
      kr = kr < S ? kr : S - 1;
      dma16(Kh + (int64_t)kr * q.k_stride_s + c * 8, st + (wave * kKI + k) * 1024);
    }
  };
  FT a[8];
  {
    const int qr = wrow0 + r32 < S ? wrow0 + r32 : S - 1;
    const S_* qrow = static_cast<const S_*>(q.q_dev) + b * q.q_stride_b + (int64_t)hd * q.q_stride_h +
                     (int64_t)qr * q.q_stride_s;
#pragma unroll
    for (int s_ = 0; s_ < 8; ++s_) a[s_] = *reinterpret_cast<const FT*>(qrow + (2 * s_ + hh) * 8);
  }
  float m[16], l[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    m[r] = kFloor;  // finite: exp2(-inf − m) = 0 and no −inf − (−inf)
    l[r] = 0.f;
  }
  bool pending = true;  // wave-uniform: some (lane, row) has no reference max yet
  // 3-slot LDS ring: tile kt+2 goes into the slot of tile kt-1, which every wave finished reading
  // before the barrier of iteration kt — one barrier per tile.  (A software-pipelined variant — the
  // MFMAs of tile kt+1 interleaved with tile kt's exp2 sums at 2 waves/SIMD — measured 7 % slower than
  // this loop at 3 waves/SIMD: 1.91 against 1.77 ms at S = 16384, 32 heads.)
  issue(0);
  if (ntiles > 1) issue(1);
  for (int kt = 0; kt < ntiles; ++kt) {
    if (kt + 1 < ntiles) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kKI) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // every wave's pieces of tile kt landed; slot (kt+2)%3 is free
    if (kt + 2 < ntiles) issue(kt + 2);
    if (kt * kKeys > wave_last) continue;  // causal: every key of the tile is past the wave's rows
    f32x16 acc0, acc1;
    {
      const uint8_t* st = lds + (kt % 3) * kTile;
      const uint8_t* k0 = st + r32 * kRB;
      const uint8_t* k1 = st + (32 + r32) * kRB;
      const int sw = r32 & (kCH - 1);  // (32 + r32) & 15 == r32 & 15
      FT b0[8], b1[8];
#pragma unroll
      for (int s_ = 0; s_ < 8; ++s_) {  // every fragment in flight before the first MFMA
        const int c = ((2 * s_ + hh) ^ sw) * 16;
        b0[s_] = *reinterpret_cast<const FT*>(k0 + c);
        b1[s_] = *reinterpret_cast<const FT*>(k1 + c);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) { acc0[r] = 0.f; acc1[r] = 0.f; }
#pragma unroll
      for (int s_ = 0; s_ < 8; ++s_) {
        acc0 = L32<DT>::mfma(a[s_], b0[s_], acc0);
        acc1 = L32<DT>::mfma(a[s_], b1[s_], acc1);
      }
    }
    const int j0 = kt * kKeys + r32, j1 = j0 + 32;
    if (q.kbias_dev) {  // key padding (raw units, -inf for a padding key)
      const float kb0 = j0 < S ? key_bias_raw(q, b, j0, inv_scale) : 0.f;
      const float kb1 = j1 < S ? key_bias_raw(q, b, j1, inv_scale) : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) { acc0[r] += kb0; acc1[r] += kb1; }
    }
    const bool edge = (kt + 1) * kKeys > (q.causal ? wrow0 : S) || (kt + 1) * kKeys > S;
    if (edge) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wrow0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        acc0[r] = (j0 < S && (!q.causal || j0 <= row)) ? acc0[r] : -INFINITY;
        acc1[r] = (j1 < S && (!q.causal || j1 <= row)) ? acc1[r] : -INFINITY;
      }
    }
    if (pending) {
      // a (lane, row) without a reference max yet takes its first finite logit (+ the lazy raise of
      // attn_lse.hip while any row of the wave is still without one)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float mt = fmaxf(acc0[r], acc1[r]) * sc;
        if (mt > m[r] + kSlack) {
          l[r] *= __builtin_amdgcn_exp2f(m[r] - mt);
          m[r] = mt;
        }
      }
      bool none = false;
#pragma unroll
      for (int r = 0; r < 16; ++r) none |= m[r] == kFloor;
      pending = __ballot(none) != 0;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float nm = -m[r];
      l[r] += __builtin_amdgcn_exp2f(__builtin_fmaf(acc0[r], sc, nm)) + __builtin_amdgcn_exp2f(__builtin_fmaf(acc1[r], sc, nm));
    }
  }
  // combine the 32 lanes holding each row: M = max m, L = Σ l·2^(m − M); lse = (M + log2 L)·ln 2
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float M = m[r];
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) M = fmaxf(M, __shfl_xor(M, o, 64));
    float L = l[r] * __builtin_amdgcn_exp2f(m[r] - M);
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) L += __shfl_xor(L, o, 64);
    const int i = wrow0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
    // L = +inf or NaN: an exp2 overflowed against the reference max → a non-finite (+inf / NaN) lse
    // that the fix-up pass recomputes; L = 0: the row sees no key → -inf
    if (r32 == 0 && i < S)
      g.lse[b * q.lse_stride_b + (int64_t)hd * q.lse_stride_h + i] =
          L > 0.f ? (M + __log2f(L)) * 0.6931471805599453f : (L == 0.f ? -INFINITY : __builtin_nanf(""));
  }
}

template <int DT> int launch_inst(const rtkv_qk_desc& q, float* lse, hipStream_t st) {
  constexpr size_t lds = 3 * (size_t)kTile;
  Lse32Args a;
  a.q = q;
  a.lse = lse;
  a.nblk = (int)((q.S + kRows - 1) / kRows);
  hipLaunchKernelGGL((attn_lse32_kernel<DT>), dim3((unsigned)a.nblk, (unsigned)q.H, (unsigned)q.B), dim3(256), lds, st, a);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

}  // namespace

// head_dim 128, f16/bf16, shapes and alignment checked by launch_attention_lse
int launch_attention_lse32(const rtkv_qk_desc& q, float* lse, hipStream_t st) {
  if (q.dtype == RTKV_F16) return launch_inst<RTKV_F16>(q, lse, st);
  return launch_inst<RTKV_BF16>(q, lse, st);
}

}  // namespace rtkv
