// importance.hip — K1: prompt-attention aggregation (token_importance.py:21-47), plus the small
// score helpers (position bias :87-110, min-max normalisation :49-85).
//
// K1 reads the [B,H,S,P] prompt columns of W exactly once (the dominant input of the importance
// stage, B·H·S·P·e bytes) and reproduces PyTorch's CPU reduction order bit for bit:
//   mean over heads  = multi_row_sum cascade (16-element blocks, 4 levels) / H   (vectorized_outer_sum)
//   sum over prompt  = vectorized_inner_sum with 8 fp32 lanes, ilp-4 partials, lanes added last
// Work decomposition: a 256-thread workgroup owns TT consecutive tokens of one batch row.  For each
// head the TT×P slab is contiguous in a [B,H,S,P] slice, so the workgroup streams H slabs with one
// 16-byte load per thread per head (16 heads in flight per thread).  Means go to LDS; 8 threads per
// token then form the 8 vector lanes of the inner sum and one thread folds them.
#include "common.h"

namespace rtkv {

// ----------------------------------------------------------------------------- reduction order
// PyTorch multi_row_sum for one column, n < 2^20 (level_power = 4, level_step = 16).
template <typename Get> __device__ __forceinline__ float cascade_seq(Get get, int n) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int i = 0;
  while (i + 16 <= n) {
    for (int j = 0; j < 16; ++j, ++i) a0 += get(i);
    a1 += a0;
    a0 = 0.f;
    if ((i & (15 << 4)) == 0) {
      a2 += a1;
      a1 = 0.f;
      if ((i & (15 << 8)) == 0) {
        a3 += a2;
        a2 = 0.f;
      }
    }
  }
  for (; i < n; ++i) a0 += get(i);
  a0 += a1;
  a0 += a2;
  a0 += a3;
  return a0;
}

// PyTorch row_sum<.., ilp_factor = 4>: part k = cascade over elements 4j+k, tail into part 0.
template <typename Get> __device__ __forceinline__ float row_sum_ilp4(Get get, int n) {
  const int nq = n >> 2;
  float part[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) part[k] = cascade_seq([&](int j) { return get(4 * j + k); }, nq);
  for (int i = nq * 4; i < n; ++i) part[0] += get(i);
  part[0] += part[1];
  part[0] += part[2];
  part[0] += part[3];
  return part[0];
}

// ----------------------------------------------------------------------------- K1 aggregation
template <int DT, int VEC> struct VecT;
template <> struct VecT<RTKV_F32, 4> { using T = float4; };
template <> struct VecT<RTKV_F16, 8> { using T = uint4; };
template <> struct VecT<RTKV_BF16, 8> { using T = uint4; };

template <int DT, int VEC>
__device__ __forceinline__ void unpack_vec(const typename VecT<DT, VEC>::T& v, float (&x)[VEC]) {
  if constexpr (DT == RTKV_F32) {
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  } else {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x[2 * k] = Dt<DT>::load((uint16_t)(w[k] & 0xffffu));
      x[2 * k + 1] = Dt<DT>::load((uint16_t)(w[k] >> 16));
    }
  }
}

// Fast path: P % VEC == 0, 16-byte aligned rows.  Thread → one VEC-wide chunk of one token row.
template <int DT, int VEC>
__global__ __launch_bounds__(256) void aggregation_vec_kernel(const typename Dt<DT>::S* __restrict__ W,
                                                              int H, int64_t S, int P, int64_t sb,
                                                              int64_t sh, int64_t ss, int TT, int64_t lim,
                                                              float* __restrict__ A, AggExtras ex) {
  using S_ = typename Dt<DT>::S;
  using V = typename VecT<DT, VEC>::T;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* means = smem;                 // [TT][P]
  float* lanes = smem + TT * P;        // [TT][8]
  float* tokA = lanes + TT * 8;        // [TT]
  zero_regions(ex);
  const int b = blockIdx.y;
  const int64_t i0 = (int64_t)blockIdx.x * TT;
  const int cpr = P / VEC;
  const S_* Wb = W + b * sb;
  for (int e = threadIdx.x; e < TT * cpr; e += blockDim.x) {
    const int tok = e / cpr, ch = e - tok * cpr;
    const int64_t i = i0 + tok;
    if (i >= S) continue;
    const S_* base = Wb + i * ss + (int64_t)ch * VEC;
    float a0[VEC], a1[VEC], a2[VEC], a3[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) a0[k] = a1[k] = a2[k] = a3[k] = 0.f;
    int h = 0;
    while (h + 16 <= H) {
      V v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = *reinterpret_cast<const V*>(base + (int64_t)(h + j) * sh);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        float x[VEC];
        unpack_vec<DT, VEC>(v[j], x);
#pragma unroll
        for (int k = 0; k < VEC; ++k) a0[k] += x[k];
      }
      h += 16;
#pragma unroll
      for (int k = 0; k < VEC; ++k) { a1[k] += a0[k]; a0[k] = 0.f; }
      if ((h & (15 << 4)) == 0) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) { a2[k] += a1[k]; a1[k] = 0.f; }
        if ((h & (15 << 8)) == 0) {
#pragma unroll
          for (int k = 0; k < VEC; ++k) { a3[k] += a2[k]; a2[k] = 0.f; }
        }
      }
    }
    for (; h < H; ++h) {
      float x[VEC];
      unpack_vec<DT, VEC>(*reinterpret_cast<const V*>(base + (int64_t)h * sh), x);
#pragma unroll
      for (int k = 0; k < VEC; ++k) a0[k] += x[k];
    }
    const float fH = (float)H;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      float s = a0[k];
      s += a1[k];
      s += a2[k];
      s += a3[k];
      const int p = ch * VEC + k;
      const int64_t col = i * P + p;
      if (col >= lim) {  // columns past the 32-aligned block: row_sum (ilp 4) order
        const S_* colp = Wb + i * ss + p;
        s = row_sum_ilp4([&](int hh) { return Dt<DT>::load(colp[(int64_t)hh * sh]); }, H);
      }
      means[tok * P + p] = Dt<DT>::rnd(s / fH);
    }
  }
  __syncthreads();
  // inner sum over the prompt columns: 8 fp32 vector lanes per token
  constexpr int VN = (DT == RTKV_F32) ? 8 : 16;
  if (P >= VN) {
    const int nv = P / VN;
    for (int e = threadIdx.x; e < TT * 8; e += blockDim.x) {
      const int tok = e >> 3, l = e & 7;
      if (i0 + tok >= S) continue;
      const float* x = means + tok * P;
      lanes[tok * 8 + l] = row_sum_ilp4(
          [&](int m) { return VN == 8 ? x[8 * m + l] : (x[16 * m + l] + x[16 * m + 8 + l]); }, nv);
    }
  }
  __syncthreads();
  for (int tok = threadIdx.x; tok < TT; tok += blockDim.x) {
    const int64_t i = i0 + tok;
    if (i >= S) continue;
    const float* x = means + tok * P;
    float fin;
    if (P >= VN) {
      const int nv = P / VN;
      fin = 0.f;
      for (int k = nv * VN; k < P; ++k) fin += x[k];
#pragma unroll
      for (int l = 0; l < 8; ++l) fin += lanes[tok * 8 + l];
    } else {
      fin = row_sum_ilp4([&](int k) { return x[k]; }, P);
    }
    const float Ai = Dt<DT>::rnd(fin);
    A[(int64_t)b * S + i] = Ai;
    tokA[tok] = Ai;
    if (ex.t2 && b == 0) ex.t2[i] = ex.beta * ((S > 1) ? torch_logf((uint32_t)(i + 1)) / ex.logS : 0.f);
  }
  if (ex.part) {  // block (min, max) of A for the score normalisation (token_importance.py:71-83)
    __syncthreads();
    if (threadIdx.x == 0) {
      float mn = INFINITY, mx = -INFINITY;
      for (int t = 0; t < TT && i0 + t < S; ++t) { mn = fminf(mn, tokA[t]); mx = fmaxf(mx, tokA[t]); }
      ex.part[((int64_t)b * gridDim.x + blockIdx.x) * 2] = mn;
      ex.part[((int64_t)b * gridDim.x + blockIdx.x) * 2 + 1] = mx;
    }
  }
}

// Register path for fp16/bf16 with P = 8·CPR (CPR = 16 for P = 128): thread (token, chunk) holds the
// 8 head means of its 16-byte chunk, and the inner sum over the prompt columns runs across the CPR
// lanes of the token with wave shuffles in exactly PyTorch's order (no LDS, no barrier):
//   y_m[l]   = x[16m + l] + x[16m + 8 + l]          (chunks 2m, 2m+1: one 16-wide Vectorized<Half>)
//   part_k   = Σ_j y_{4j+k} (sequential), tail m >= 4·nq into part 0, then part0+part1+part2+part3
//   A        = Σ_l lanes[l] (l = 0..7, sequential)                       (vectorized_inner_sum, ILP 4)
// HB heads per load batch; PF: the next batch's loads are issued before the current batch is
// summed (two batches in flight, so every wave keeps streaming).  The per-element addition order is
// the same for every (HB, PF): heads in order, the cascade step after every 16th head.
//
// SPLIT (32 <= H <= 64): the workgroup's two halves stream the head range in two parts at once —
// half 0 the first ceil(nb/2) 16-head blocks, half 1 the other full blocks (each summed from zero, as
// multi_row_sum sums a block before adding it into the level-1 accumulator) and the tail — so a
// 16-byte chunk per thread gives twice the threads (waves per CU) of the unsplit kernel, and every
// thread's loads are in flight at once.  Half 1 hands its block sums over through LDS; half 0 adds
// them in block order (a1 += block, the cascade step) and takes the tail as a0: the same additions
// in the same order as the sequential loop.
template <int DT, int CPR, int HB = 16, bool PF = false, int BT = 256, bool SPLIT = false, int HC = 0>
__global__ __launch_bounds__(BT, SPLIT ? 2 * BT / 256 : 1) void aggregation_shfl_kernel(const typename Dt<DT>::S* __restrict__ W, int H,
                                                               int64_t S, int64_t sb, int64_t sh, int64_t ss,
                                                               int64_t lim, float* __restrict__ A, AggExtras ex) {
  using S_ = typename Dt<DT>::S;
  using V = uint4;
  constexpr int P = 8 * CPR;
  constexpr int HALF = SPLIT ? BT / 2 : BT;
  constexpr int TT = HALF / CPR; // tokens per block
  constexpr int NV = CPR / 2;    // 16-column groups
  constexpr int NQ = NV / 4;
  constexpr int NW = BT / 64;
  __shared__ float red[2][NW];
  zero_regions(ex);
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int half = SPLIT ? (int)(threadIdx.x >= HALF) : 0;
  const int tid = threadIdx.x - half * HALF;
  const int tok = tid / CPR, ch = tid % CPR;
  const int64_t i = (int64_t)blockIdx.x * TT + tok;
  const bool valid = i < S;
  const int64_t ic = valid ? i : S - 1;  // clamped row (its loads are discarded)
  const S_* base = W + b * sb + ic * ss + ch * 8;
  float a0[8], a1[8], a2[8], a3[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a0[k] = a1[k] = a2[k] = a3[k] = 0.f;
  // multi_row_sum's cascade: after every 16th head a1 += a0, every 256th a2 += a1, every 4096th a3 += a2
  auto cascade = [&](int hh) {
    if ((hh & 15) == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) { a1[k] += a0[k]; a0[k] = 0.f; }
      if ((hh & (15 << 4)) == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) { a2[k] += a1[k]; a1[k] = 0.f; }
        if ((hh & (15 << 8)) == 0) {
#pragma unroll
          for (int k = 0; k < 8; ++k) { a3[k] += a2[k]; a2[k] = 0.f; }
        }
      }
    }
  };
  auto load_batch = [&](V (&v)[HB], int h0) {
#pragma unroll
    for (int j = 0; j < HB; ++j) v[j] = load16_nt(base + (int64_t)(h0 + j) * sh);
  };
  auto consume = [&](const V (&v)[HB], int h0) {
#pragma unroll
    for (int j = 0; j < HB; ++j) {
      float x[8];
      unpack_vec<DT, 8>(v[j], x);
#pragma unroll
      for (int k = 0; k < 8; ++k) a0[k] += x[k];
      if (((h0 + j + 1) & 15) == 0) cascade(h0 + j + 1);
    }
  };
  int h = 0;
  if constexpr (SPLIT) {
    static_assert(!PF && HC >= 32 && HC <= 64, "split: a compile-time head count in [32, 64]");
    __shared__ float4 xfer[3][HALF][2];  // half 1's full-block sums (<= 2) and tail sum, 8 floats per thread
    constexpr int nfull = HC >> 4, nb0 = (nfull + 1) >> 1;
    // 4-head load batches (as the fp32 kernel): <= 64 VGPRs, so two 1024-thread workgroups (32 waves,
    // 128 KB of loads in flight) fit a CU
    auto add4 = [&](int h0) {
      V v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = load16_nt(base + (int64_t)(h0 + j) * sh);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x[8];
        unpack_vec<DT, 8>(v[j], x);
#pragma unroll
        for (int e = 0; e < 8; ++e) a0[e] += x[e];
      }
      // the next batch's loads stay behind this one's adds (the sums are pinned here, then no memory
      // op crosses): 4 loads in flight per thread, 32 waves per CU
      asm volatile("" : "+v"(a0[0]), "+v"(a0[1]), "+v"(a0[2]), "+v"(a0[3]), "+v"(a0[4]), "+v"(a0[5]), "+v"(a0[6]),
                   "+v"(a0[7])::"memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    if (half == 0) {
#pragma unroll
      for (; h < 16 * nb0; h += 16) {
        add4(h);
        add4(h + 4);
        add4(h + 8);
        add4(h + 12);
#pragma unroll
        for (int e = 0; e < 8; ++e) {  // the cascade step (H <= 64: a2, a3 stay zero)
          a1[e] += a0[e];
          a0[e] = 0.f;
        }
      }
    } else {
      int k = 0;
#pragma unroll
      for (h = 16 * nb0; h + 16 <= HC; h += 16, ++k) {
        add4(h);
        add4(h + 4);
        add4(h + 8);
        add4(h + 12);
        xfer[k][tid][0] = make_float4(a0[0], a0[1], a0[2], a0[3]);
        xfer[k][tid][1] = make_float4(a0[4], a0[5], a0[6], a0[7]);
#pragma unroll
        for (int e = 0; e < 8; ++e) a0[e] = 0.f;
      }
#pragma unroll
      for (; h < HC; ++h) {  // the tail (H % 16 heads), sequential from zero
        float x[8];
        unpack_vec<DT, 8>(*reinterpret_cast<const V*>(base + (int64_t)h * sh), x);
#pragma unroll
        for (int e = 0; e < 8; ++e) a0[e] += x[e];
      }
      xfer[2][tid][0] = make_float4(a0[0], a0[1], a0[2], a0[3]);
      xfer[2][tid][1] = make_float4(a0[4], a0[5], a0[6], a0[7]);
    }
    __syncthreads();
    if (half == 0) {
      for (int k = 0; k < nfull - nb0; ++k) {  // blocks nb0.. in order: the cascade step of each
        const float4 u = xfer[k][tid][0], w = xfer[k][tid][1];
        const float blk[8] = {u.x, u.y, u.z, u.w, w.x, w.y, w.z, w.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) a1[e] += blk[e];
      }
      const float4 u = xfer[2][tid][0], w = xfer[2][tid][1];
      a0[0] = u.x; a0[1] = u.y; a0[2] = u.z; a0[3] = u.w; a0[4] = w.x; a0[5] = w.y; a0[6] = w.z; a0[7] = w.w;
    }
    h = HC;
  } else if constexpr (!PF) {
    while (h + HB <= H) {
      V v[HB];
      load_batch(v, h);
      consume(v, h);
      h += HB;
    }
  } else if (H >= HB) {
    V v0[HB], v1[HB];
    load_batch(v0, 0);
    while (true) {
      if (h + 2 * HB <= H) load_batch(v1, h + HB);
      consume(v0, h);
      h += HB;
      if (h + HB > H) break;
      if (h + 2 * HB <= H) load_batch(v0, h + HB);
      consume(v1, h);
      h += HB;
      if (h + HB > H) break;
    }
  }
  for (; h < H; ++h) {
    float x[8];
    unpack_vec<DT, 8>(*reinterpret_cast<const V*>(base + (int64_t)h * sh), x);
#pragma unroll
    for (int k = 0; k < 8; ++k) a0[k] += x[k];
    if (((h + 1) & 15) == 0) cascade(h + 1);
  }
  const float fH = (float)H;
  float m[8];  // head means of columns ch*8 .. ch*8+7, rounded to the dtype
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float s = a0[k];
    s += a1[k];
    s += a2[k];
    s += a3[k];
    const int64_t col = ic * P + ch * 8 + k;
    // columns past the 32-aligned block of the flattened [S*P] take row_sum's (ilp 4) order; with P a
    // multiple of 32 every column is inside it (lim = S*P), and the branch compiles away
    if (P % 32 != 0 && col >= lim && half == 0) {
      const S_* colp = W + b * sb + ic * ss + ch * 8 + k;
      s = row_sum_ilp4([&](int hh) { return Dt<DT>::load(colp[(int64_t)hh * sh]); }, H);
    }
    m[k] = Dt<DT>::rnd(s / fH);
  }
  // y_m on even chunks (m = ch / 2): this chunk + the next one
  float y[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) y[k] = m[k] + __shfl_xor(m[k], 1, 64);
  // part_k (k = 0..3) on chunk 2k: Σ_{j < NQ} y_{4j+k} in order, then the tail groups into part 0
  const int tl = lane - ch;  // lane of this token's chunk 0
  float part[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < NQ; ++j) acc += __shfl(y[k], tl + 2 * (4 * j + (ch >> 1 & 3)), 64);
    part[k] = acc;
    if constexpr (SPLIT) __builtin_amdgcn_sched_barrier(0);  // one k at a time: fits 64 VGPRs
  }
  // chunk 0 folds: part0 (+ tail groups) + part1 + part2 + part3, then the 8 vector lanes
  float fin = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if constexpr (SPLIT) __builtin_amdgcn_sched_barrier(0);
    float p0 = part[k];
#pragma unroll
    for (int mm = 4 * NQ; mm < NV; ++mm) p0 += __shfl(y[k], tl + 2 * mm, 64);
    const float p1 = __shfl(part[k], tl + 2, 64), p2 = __shfl(part[k], tl + 4, 64), p3 = __shfl(part[k], tl + 6, 64);
    p0 += p1;
    p0 += p2;
    p0 += p3;
    fin += p0;
  }
  const float Ai = Dt<DT>::rnd(fin);
  float mn = INFINITY, mx = -INFINITY;
  if (ch == 0 && valid && half == 0) {  // (SPLIT: half 1's waves only streamed heads)
    A[(int64_t)b * S + i] = Ai;
    if (ex.t2 && b == 0) ex.t2[i] = ex.beta * ((S > 1) ? torch_logf((uint32_t)(i + 1)) / ex.logS : 0.f);
    mn = mx = Ai;
  }
  if (ex.part) {  // block (min, max) of A for the score normalisation (token_importance.py:71-83)
    mn = wave_min(mn);
    mx = wave_max(mx);
    if (lane == 0) { red[0][wave] = mn; red[1][wave] = mx; }
    __syncthreads();
    if (threadIdx.x == 0) {
      float lo = red[0][0], hi = red[1][0];
#pragma unroll
      for (int w2 = 1; w2 < NW; ++w2) { lo = fminf(lo, red[0][w2]); hi = fmaxf(hi, red[1][w2]); }
      ex.part[((int64_t)b * gridDim.x + blockIdx.x) * 2] = lo;
      ex.part[((int64_t)b * gridDim.x + blockIdx.x) * 2 + 1] = hi;
    }
  }
}

// Register path for fp32 with P = 4·CPR (CPR = 32 for P = 128): thread (token, chunk) streams one
// 16-byte chunk (4 columns) of its token's prompt row for every head, as the 16-bit kernel above,
// and the inner sum runs across the token's CPR lanes with shuffles in PyTorch's fp32 order
// (Vectorized<float> = 8 lanes, so chunks 2m and 2m+1 form vector m):
//   part_k[l] = Σ_j x[8(4j+k) + l]   (j = 0..NV/4-1 sequential from 0, k = 0..3)   row_sum ilp 4
//   lane[l]   = part_0 + part_1 + part_2 + part_3, A = Σ_l lane[l] (l = 0..7)      vectorized_inner_sum
// Chunk ch < 8 holds part_{ch/2}[(ch%2)*4 + e] after the first step; chunk 0 folds.
template <int CPR, int HB = 16, int BT = 256>
__global__ __launch_bounds__(BT) void aggregation_shfl32_kernel(const float* __restrict__ W, int H, int64_t S,
                                                                 int64_t sb, int64_t sh, int64_t ss, int64_t lim,
                                                                 float* __restrict__ A, AggExtras ex) {
  constexpr int P = 4 * CPR;
  constexpr int TT = BT / CPR;   // tokens per block
  constexpr int NV = CPR / 2;    // 8-column vectors
  constexpr int NQ = NV / 4;
  constexpr int NW = BT / 64;
  static_assert(NV % 4 == 0 && CPR <= 64, "aggregation_shfl32: CPR must be a multiple of 8, at most 64");
  __shared__ float red[2][NW];
  zero_regions(ex);
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tok = threadIdx.x / CPR, ch = threadIdx.x % CPR;
  const int64_t i = (int64_t)blockIdx.x * TT + tok;
  const bool valid = i < S;
  const int64_t ic = valid ? i : S - 1;  // clamped row (its loads are discarded)
  const float* base = W + b * sb + ic * ss + ch * 4;
  float a0[4], a1[4], a2[4], a3[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) a0[k] = a1[k] = a2[k] = a3[k] = 0.f;
  auto cascade = [&](int hh) {  // multi_row_sum: after every 16th head a1 += a0, every 256th a2 += a1, ...
    if ((hh & 15) == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) { a1[k] += a0[k]; a0[k] = 0.f; }
      if ((hh & (15 << 4)) == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) { a2[k] += a1[k]; a1[k] = 0.f; }
        if ((hh & (15 << 8)) == 0) {
#pragma unroll
          for (int k = 0; k < 4; ++k) { a3[k] += a2[k]; a2[k] = 0.f; }
        }
      }
    }
  };
  int h = 0;
  while (h + HB <= H) {
    uint4 v[HB];
#pragma unroll
    for (int j = 0; j < HB; ++j) v[j] = load16_nt(base + (int64_t)(h + j) * sh);
#pragma unroll
    for (int j = 0; j < HB; ++j) {
      a0[0] += __uint_as_float(v[j].x);
      a0[1] += __uint_as_float(v[j].y);
      a0[2] += __uint_as_float(v[j].z);
      a0[3] += __uint_as_float(v[j].w);
      if (((h + j + 1) & 15) == 0) cascade(h + j + 1);
    }
    h += HB;
  }
  for (; h < H; ++h) {
    const uint4 v = load16_nt(base + (int64_t)h * sh);
    a0[0] += __uint_as_float(v.x);
    a0[1] += __uint_as_float(v.y);
    a0[2] += __uint_as_float(v.z);
    a0[3] += __uint_as_float(v.w);
    if (((h + 1) & 15) == 0) cascade(h + 1);
  }
  const float fH = (float)H;
  float m[4];  // head means of columns ch*4 .. ch*4+3
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float s = a0[k];
    s += a1[k];
    s += a2[k];
    s += a3[k];
    const int64_t col = ic * P + ch * 4 + k;
    if (P % 32 != 0 && col >= lim) {  // columns past the 32-aligned block: row_sum (ilp 4) order
      const float* colp = W + b * sb + ic * ss + ch * 4 + k;
      s = row_sum_ilp4([&](int hh) { return colp[(int64_t)hh * sh]; }, H);
    }
    m[k] = s / fH;
  }
  const int tl = lane - ch;  // lane of this token's chunk 0
  // part_{ch/2}[(ch%2)*4 + e] on chunks ch < 8: vectors m' = 4j + ch/2 live on chunks 8j + ch
  float part[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < NQ; ++j) acc += __shfl(m[e], tl + 8 * j + (ch & 7), 64);
    part[e] = acc;
  }
  float fin = 0.f;
#pragma unroll
  for (int l = 0; l < 8; ++l) {
    const int hi = l >> 2, e = l & 3;
    float p0 = __shfl(part[e], tl + hi, 64);
    const float p1 = __shfl(part[e], tl + 2 + hi, 64), p2 = __shfl(part[e], tl + 4 + hi, 64),
                p3 = __shfl(part[e], tl + 6 + hi, 64);
    p0 += p1;
    p0 += p2;
    p0 += p3;
    fin += p0;
  }
  const float Ai = fin;
  float mn = INFINITY, mx = -INFINITY;
  if (ch == 0 && valid) {
    A[(int64_t)b * S + i] = Ai;
    if (ex.t2 && b == 0) ex.t2[i] = ex.beta * ((S > 1) ? torch_logf((uint32_t)(i + 1)) / ex.logS : 0.f);
    mn = mx = Ai;
  }
  if (ex.part) {  // block (min, max) of A for the score normalisation (token_importance.py:71-83)
    mn = wave_min(mn);
    mx = wave_max(mx);
    if (lane == 0) { red[0][wave] = mn; red[1][wave] = mx; }
    __syncthreads();
    if (threadIdx.x == 0) {
      float lo = red[0][0], hi = red[1][0];
#pragma unroll
      for (int w2 = 1; w2 < NW; ++w2) { lo = fminf(lo, red[0][w2]); hi = fmaxf(hi, red[1][w2]); }
      ex.part[((int64_t)b * gridDim.x + blockIdx.x) * 2] = lo;
      ex.part[((int64_t)b * gridDim.x + blockIdx.x) * 2 + 1] = hi;
    }
  }
}

// Generic path: any P / strides / alignment (scalar loads; the cfg1 P = 102 case lands here).
template <int DT>
__global__ __launch_bounds__(256) void aggregation_scalar_kernel(const typename Dt<DT>::S* __restrict__ W,
                                                                 int H, int64_t S, int P, int64_t sb,
                                                                 int64_t sh, int64_t ss, int TT, int64_t lim,
                                                                 float* __restrict__ A, AggExtras ex) {
  using S_ = typename Dt<DT>::S;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* means = smem;
  float* lanes = smem + TT * P;
  float* tokA = lanes + TT * 8;
  zero_regions(ex);
  const int b = blockIdx.y;
  const int64_t i0 = (int64_t)blockIdx.x * TT;
  const S_* Wb = W + b * sb;
  for (int e = threadIdx.x; e < TT * P; e += blockDim.x) {
    const int tok = e / P, p = e - tok * P;
    const int64_t i = i0 + tok;
    if (i >= S) continue;
    const S_* colp = Wb + i * ss + p;
    auto get = [&](int hh) { return Dt<DT>::load(colp[(int64_t)hh * sh]); };
    const int64_t col = i * P + p;
    const float s = (col < lim) ? cascade_seq(get, H) : row_sum_ilp4(get, H);
    means[tok * P + p] = Dt<DT>::rnd(s / (float)H);
  }
  __syncthreads();
  constexpr int VN = (DT == RTKV_F32) ? 8 : 16;
  if (P >= VN) {
    const int nv = P / VN;
    for (int e = threadIdx.x; e < TT * 8; e += blockDim.x) {
      const int tok = e >> 3, l = e & 7;
      if (i0 + tok >= S) continue;
      const float* x = means + tok * P;
      lanes[tok * 8 + l] = row_sum_ilp4(
          [&](int m) { return VN == 8 ? x[8 * m + l] : (x[16 * m + l] + x[16 * m + 8 + l]); }, nv);
    }
  }
  __syncthreads();
  for (int tok = threadIdx.x; tok < TT; tok += blockDim.x) {
    const int64_t i = i0 + tok;
    if (i >= S) continue;
    const float* x = means + tok * P;
    float fin;
    if (P >= VN) {
      const int nv = P / VN;
      fin = 0.f;
      for (int k = nv * VN; k < P; ++k) fin += x[k];
      for (int l = 0; l < 8; ++l) fin += lanes[tok * 8 + l];
    } else {
      fin = row_sum_ilp4([&](int k) { return x[k]; }, P);
    }
    const float Ai = Dt<DT>::rnd(fin);
    A[(int64_t)b * S + i] = Ai;
    tokA[tok] = Ai;
    if (ex.t2 && b == 0) ex.t2[i] = ex.beta * ((S > 1) ? torch_logf((uint32_t)(i + 1)) / ex.logS : 0.f);
  }
  if (ex.part) {  // block (min, max) of A for the score normalisation (token_importance.py:71-83)
    __syncthreads();
    if (threadIdx.x == 0) {
      float mn = INFINITY, mx = -INFINITY;
      for (int t = 0; t < TT && i0 + t < S; ++t) { mn = fminf(mn, tokA[t]); mx = fmaxf(mx, tokA[t]); }
      ex.part[((int64_t)b * gridDim.x + blockIdx.x) * 2] = mn;
      ex.part[((int64_t)b * gridDim.x + blockIdx.x) * 2 + 1] = mx;
    }
  }
}

// Columns of the flattened [S*P] head-mean below this limit take the cascade order (see
// oracle/rtkv_oracle.c outer_cascade_limit).
static int64_t cascade_limit(int dt, int64_t M) {
  const int64_t vec = (dt == RTKV_F32) ? 8 : 16;
  if (M >= vec) return (M / 32) * 32;
  return (M / 4) * 4;
}

// Register-path workgroup size: 1024 threads (16 KB contiguous per head per workgroup, the fastest at
// cfg3) as long as that still gives every CU a workgroup; smaller workgroups below, so that short
// prompts (S = 4096: 128 workgroups of 1024 threads would leave half the CUs idle) fill the chip.
// chunks = 16-byte chunks per token row (16 fp16/bf16, 32 fp32 at P = 128).
static int k1_block_threads(int64_t tokens, int chunks) {
  const int64_t want = 256;  // one per CU
  for (int bt = 1024; bt > 256; bt >>= 1)
    if (tokens / (bt / chunks) >= want) return bt;
  return 256;
}

template <int DT>
static int launch_agg_dt(const rtkv_attn_desc& w, int P, float* A, hipStream_t st, const AggExtras& x) {
  using S_ = typename Dt<DT>::S;
  constexpr int VEC = 16 / Dt<DT>::kBytes;
  const S_* W = static_cast<const S_*>(w.w_dev);
  // flattened [S*P] column index of local row i is (row0 + i)*P + p: shift the global boundary
  const int64_t lim = x.S_total ? cascade_limit(DT, x.S_total * (int64_t)P) - x.row0 * (int64_t)P
                                : cascade_limit(DT, w.S * (int64_t)P);
  const bool aligned = ((uintptr_t)W % 16 == 0) && (P % VEC == 0) && (w.stride_s % VEC == 0) &&
                       (w.stride_h % VEC == 0) && (w.stride_b % VEC == 0);
  const int H = (int)w.H;
  if constexpr (DT != RTKV_F32) {
    if (aligned && P == 128) {  // register path (Llama prompts: P = 128)
      // 16-head load batches: in the pipeline (after K4's write-back) 29.9 us, against 30.9 us for
      // 4-head batches with the next one in flight (isolated, tools/k1_grid_probe.hip: 28.7 vs 24.9).
      // 1024-thread workgroups: 64 tokens, 16 KB contiguous per head per workgroup (cfg3 fp16 in the
      // pipeline: 27.8 us against 30.0 for 512 threads and 30.1 for 256).  RTKV_K1_BT16: 256/512/1024.
      static const int bt_env = [] {
        const char* e = getenv("RTKV_K1_BT16");
        const int v = e ? atoi(e) : 0;
        return v == 256 || v == 512 || v == 1024 ? v : 0;
      }();
      if ((H == 32 || H == 40) && w.S * w.B < 16384 && !getenv("RTKV_K1_NOSPLIT")) {
        // Llama-2-7B / 13B heads, short prompts: the head range in two halves per workgroup, twice the
        // waves per CU (S = 4096 f16: 14.3 against 17.6 us; at S = 16384, where the unsplit grid already
        // gives every CU a workgroup, the split measured slower: 31.0 against 27.8 us, r04b).
        // RTKV_K1_NOSPLIT: the unsplit kernel, for cross-checks.
        dim3 grid((unsigned)((w.S + 31) / 32), (unsigned)w.B);
        if (x.nparts) *x.nparts = (int)grid.x;
        if (H == 32)
          hipLaunchKernelGGL((aggregation_shfl_kernel<DT, 16, 16, false, 1024, true, 32>), grid, dim3(1024), 0, st,
                             W, H, w.S, w.stride_b, w.stride_h, w.stride_s, lim, A, x);
        else
          hipLaunchKernelGGL((aggregation_shfl_kernel<DT, 16, 16, false, 1024, true, 40>), grid, dim3(1024), 0, st,
                             W, H, w.S, w.stride_b, w.stride_h, w.stride_s, lim, A, x);
        RTKV_HIP_CHECK(hipGetLastError());
        return RTKV_OK;
      }
      const int bt = bt_env ? bt_env : k1_block_threads(w.S * w.B, 16);
      const int tt = bt / 16;
      dim3 grid((unsigned)((w.S + tt - 1) / tt), (unsigned)w.B);
      if (x.nparts) *x.nparts = (int)grid.x;
      if (bt == 1024)
        hipLaunchKernelGGL((aggregation_shfl_kernel<DT, 16, 16, false, 1024>), grid, dim3(1024), 0, st, W, H, w.S,
                           w.stride_b, w.stride_h, w.stride_s, lim, A, x);
      else if (bt == 512)
        hipLaunchKernelGGL((aggregation_shfl_kernel<DT, 16, 16, false, 512>), grid, dim3(512), 0, st, W, H, w.S,
                           w.stride_b, w.stride_h, w.stride_s, lim, A, x);
      else
        hipLaunchKernelGGL((aggregation_shfl_kernel<DT, 16>), grid, dim3(256), 0, st, W, H, w.S, w.stride_b,
                           w.stride_h, w.stride_s, lim, A, x);
      RTKV_HIP_CHECK(hipGetLastError());
      return RTKV_OK;
    }
  } else {
    if (aligned && P == 128 && !getenv("RTKV_K1_LDS")) {  // register path; RTKV_K1_LDS: cross-check knob
      // 4 heads per load batch (tools/k1_grid_probe.hip: 46.5 us vs 56 us for 16-head batches at cfg3);
      // 1024-thread workgroups: 32 tokens, i.e. 16 KB contiguous per head per workgroup (cfg3 in the
      // pipeline: 47.1 us against 48.6 for 512 threads and 52.8 for 256).  RTKV_K1_BT: 256/512/1024.
      static const int bt_env = [] {
        const char* e = getenv("RTKV_K1_BT");
        const int v = e ? atoi(e) : 0;
        return v == 256 || v == 512 || v == 1024 ? v : 0;
      }();
      const int bt = bt_env ? bt_env : k1_block_threads(w.S * w.B, 32);
      const int tt = bt / 32;
      dim3 grid((unsigned)((w.S + tt - 1) / tt), (unsigned)w.B);
      if (x.nparts) *x.nparts = (int)grid.x;
      if (bt == 1024)
        hipLaunchKernelGGL((aggregation_shfl32_kernel<32, 4, 1024>), grid, dim3(1024), 0, st, W, H, w.S, w.stride_b,
                           w.stride_h, w.stride_s, lim, A, x);
      else if (bt == 512)
        hipLaunchKernelGGL((aggregation_shfl32_kernel<32, 4, 512>), grid, dim3(512), 0, st, W, H, w.S, w.stride_b,
                           w.stride_h, w.stride_s, lim, A, x);
      else
        hipLaunchKernelGGL((aggregation_shfl32_kernel<32, 4, 256>), grid, dim3(256), 0, st, W, H, w.S, w.stride_b,
                           w.stride_h, w.stride_s, lim, A, x);
      RTKV_HIP_CHECK(hipGetLastError());
      return RTKV_OK;
    }
  }
  if (aligned) {
    const int cpr = P / VEC;
    int TT = 256 / cpr;
    if (TT < 1) TT = 1;
    if (TT > 64) TT = 64;
    const size_t lds = sizeof(float) * (size_t)TT * (P + 9);
    dim3 grid((unsigned)((w.S + TT - 1) / TT), (unsigned)w.B);
    if (x.nparts) *x.nparts = (int)grid.x;
    hipLaunchKernelGGL((aggregation_vec_kernel<DT, VEC>), grid, dim3(256), lds, st, W, H, w.S, P,
                       w.stride_b, w.stride_h, w.stride_s, TT, lim, A, x);
  } else {
    int TT = 256 / P;
    if (TT < 1) TT = 1;
    const size_t lds = sizeof(float) * (size_t)TT * (P + 9);
    dim3 grid((unsigned)((w.S + TT - 1) / TT), (unsigned)w.B);
    if (x.nparts) *x.nparts = (int)grid.x;
    hipLaunchKernelGGL((aggregation_scalar_kernel<DT>), grid, dim3(256), lds, st, W, H, w.S, P,
                       w.stride_b, w.stride_h, w.stride_s, TT, lim, A, x);
  }
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

int launch_aggregation(const rtkv_attn_desc& w, int P, float* A, hipStream_t st, const AggExtras& x) {
  RTKV_REQUIRE(w.w_dev && A, "aggregation: null pointer");
  RTKV_REQUIRE(w.B >= 1 && w.H >= 1 && w.S >= 1, "aggregation: empty shape");
  RTKV_REQUIRE(w.H < (1 << 20), "aggregation: H must be < 2^20");
  RTKV_REQUIRE(P >= 1 && P <= w.cols, "aggregation: prompt_len must be in [1, cols]");
  RTKV_REQUIRE(P <= 8192, "aggregation: prompt_len > 8192 unsupported");
  RTKV_REQUIRE(w.B <= 65535, "aggregation: B > 65535 unsupported");
  switch (w.dtype) {
    case RTKV_F32: return launch_agg_dt<RTKV_F32>(w, P, A, st, x);
    case RTKV_F16: return launch_agg_dt<RTKV_F16>(w, P, A, st, x);
    case RTKV_BF16: return launch_agg_dt<RTKV_BF16>(w, P, A, st, x);
  }
  RTKV_REQUIRE(false, "aggregation: bad dtype");
}

// ----------------------------------------------------------------------------- position bias
__global__ void position_bias_kernel(int64_t S, float logS, float* pos) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S) return;
  pos[i] = (S <= 1) ? 0.f : torch_logf((uint32_t)(i + 1)) / logS;
}

int launch_position_bias(int64_t S, float* pos, hipStream_t st) {
  RTKV_REQUIRE(pos != nullptr || S == 0, "position_bias: null output");
  RTKV_REQUIRE(S < (int64_t)1 << 31, "position_bias: S too large");
  if (S == 0) return RTKV_OK;
  const float logS = (float)std::log((double)S);
  hipLaunchKernelGGL(position_bias_kernel, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st, S, logS, pos);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

// ----------------------------------------------------------------------------- min-max normalise
template <int DT>
__global__ __launch_bounds__(1024) void minmax_normalize_kernel(const typename Dt<DT>::S* __restrict__ x,
                                                                int64_t S, typename Dt<DT>::S* __restrict__ out) {
  __shared__ float red[2][16];
  const int b = blockIdx.x;
  const typename Dt<DT>::S* xb = x + (int64_t)b * S;
  float mn = INFINITY, mx = -INFINITY;
  for (int64_t i = threadIdx.x; i < S; i += blockDim.x) {
    const float v = Dt<DT>::load(xb[i]);
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { red[0][wid] = mn; red[1][wid] = mx; }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int nw = blockDim.x >> 6;
    mn = lane < nw ? red[0][lane] : INFINITY;
    mx = lane < nw ? red[1][lane] : -INFINITY;
    mn = wave_min(mn);
    mx = wave_max(mx);
    if (lane == 0) { red[0][0] = mn; red[1][0] = mx; }
  }
  __syncthreads();
  mn = red[0][0];
  mx = red[1][0];
  const float den = Dt<DT>::rnd(mx - mn);
  const float eps = Dt<DT>::rnd(1e-8f);
  for (int64_t i = threadIdx.x; i < S; i += blockDim.x) {
    const float v = Dt<DT>::load(xb[i]);
    float qn = Dt<DT>::rnd(v - mn) / den;
    asm volatile("" : "+v"(qn));  // keep the fp32 IEEE division (LLVM would narrow it to an inexact f16 one)
    const float n = (den > eps) ? Dt<DT>::rnd(qn) : 0.f;
    out[(int64_t)b * S + i] = Dt<DT>::store(n);
  }
}

int launch_minmax_normalize(const void* x, int dt, int64_t B, int64_t S, void* out, hipStream_t st) {
  RTKV_REQUIRE(x && out, "minmax_normalize: null pointer");
  RTKV_REQUIRE(B >= 1 && S >= 1 && B <= 65535, "minmax_normalize: bad shape");
  switch (dt) {
    case RTKV_F32:
      hipLaunchKernelGGL(minmax_normalize_kernel<RTKV_F32>, dim3((unsigned)B), dim3(1024), 0, st,
                         (const float*)x, S, (float*)out);
      break;
    case RTKV_F16:
      hipLaunchKernelGGL(minmax_normalize_kernel<RTKV_F16>, dim3((unsigned)B), dim3(1024), 0, st,
                         (const uint16_t*)x, S, (uint16_t*)out);
      break;
    case RTKV_BF16:
      hipLaunchKernelGGL(minmax_normalize_kernel<RTKV_BF16>, dim3((unsigned)B), dim3(1024), 0, st,
                         (const uint16_t*)x, S, (uint16_t*)out);
      break;
    default:
      RTKV_REQUIRE(false, "minmax_normalize: bad dtype");
  }
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

}  // namespace rtkv
