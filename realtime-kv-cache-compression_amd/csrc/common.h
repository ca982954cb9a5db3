// common.h — device helpers shared by the rtkv kernels (gfx950 / CDNA4, wave64).
//
// Numerics contract (see include/rtkv.h): every elementwise op of the reference is an fp32 op
// followed by a round-to-nearest-even into the tensor dtype; the library is compiled with
// -ffp-contract=off and IEEE fp32 division so that the device ops equal PyTorch's CPU ops bit for bit.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "rtkv.h"

namespace rtkv {

constexpr int kWave = 64;

// ------------------------------------------------------------------------------------ dtypes
template <int DT> struct Dt;

template <> struct Dt<RTKV_F32> {
  using S = float;                       // storage type
  static constexpr int kBytes = 4;
  static constexpr int kPrecision = 24;  // significand bits incl. the hidden bit
  __device__ __forceinline__ static float load(S v) { return v; }
  __device__ __forceinline__ static S store(float f) { return f; }
  __device__ __forceinline__ static float rnd(float f) { return f; }
};

template <> struct Dt<RTKV_F16> {
  using S = uint16_t;
  static constexpr int kBytes = 2;
  static constexpr int kPrecision = 11;
  __device__ __forceinline__ static float load(S v) { return (float)__builtin_bit_cast(_Float16, v); }
  __device__ __forceinline__ static S store(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
  __device__ __forceinline__ static float rnd(float f) { return (float)(_Float16)f; }
};

template <> struct Dt<RTKV_BF16> {
  using S = uint16_t;
  static constexpr int kBytes = 2;
  static constexpr int kPrecision = 8;
  __device__ __forceinline__ static float load(S v) { return __builtin_bit_cast(float, (uint32_t)v << 16); }
  __device__ __forceinline__ static S store(float f) {
    uint32_t u = __builtin_bit_cast(uint32_t, f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (S)((u >> 16) | 0x40u);
    return (S)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
  }
  __device__ __forceinline__ static float rnd(float f) { return load(store(f)); }
};

__device__ __forceinline__ float rnd_dt(int dt, float x) {
  if (dt == RTKV_F16) return Dt<RTKV_F16>::rnd(x);
  if (dt == RTKV_BF16) return Dt<RTKV_BF16>::rnd(x);
  return x;
}

inline int dtype_bytes(int dt) { return dt == RTKV_F32 ? 4 : 2; }
inline int dtype_precision(int dt) { return dt == RTKV_F16 ? 11 : (dt == RTKV_BF16 ? 8 : 24); }

// Bits per packed element (include/rtkv.h rtkv_field_width).
__host__ __device__ inline int field_width(int dt, int bits) {
  if (bits < 1 || bits > 16) return 0;
  if (dt == RTKV_F16 && bits >= 16) return 0;
  const int prec = dt == RTKV_F16 ? 11 : (dt == RTKV_BF16 ? 8 : 24);
  return bits > prec ? bits + 1 : bits;
}

// ------------------------------------------------------------------------------------ streaming
// Non-temporal 16-byte load: data read exactly once (K/V rows, attention columns) does not displace
// cache lines other kernels of the layer re-read.
typedef unsigned int rtkv_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 load16_nt(const void* p) {
  const rtkv_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const rtkv_u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Cross-workgroup hand-off accesses (MI355X_MICROARCH.md "Valid forms"): relaxed agent-scope
// atomic loads/stores lower to global_load/store ... sc1 (bypass L1, write through L2).
template <typename T> __device__ __forceinline__ void st_sc1(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T> __device__ __forceinline__ T ld_sc1(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The early statistics' 128-byte host line (rtkv_early_stats, include/rtkv.h) from one wave: lane l < 16
// stores word l of `w` (the caller's 16 words, wave-uniform in LDS) with ONE system-scope store
// instruction — no ordering wait: the seq sits in words 0 and 15.  (Field-by-field stores, a wait for
// their acknowledgements and the seq last made the publishing selection kernel ~4 us longer: the wait,
// then the seq's own round trip to host memory, ran past the kernel's natural end.)
__device__ __forceinline__ void host_line_store(uint64_t* line, const uint64_t* w) {
  const int lane = threadIdx.x & 63;
  if (lane < 16) __hip_atomic_store(line + lane, w[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------------------------ keys
// Order-preserving uint32 key of an fp32 score (larger key = larger score; -0 folded onto +0 so
// that equal scores compare equal, as in the reference's `>` comparator).
__device__ __forceinline__ uint32_t score_key(float s) {
  uint32_t u = __builtin_bit_cast(uint32_t, s);
  if (u == 0x80000000u) u = 0u;
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// torch.log(float(n)) on the CPU = Sleef_logf8_u10: the correctly rounded logf except at these
// integers (measured against torch 2.10; oracle/rtkv_oracle.c carries the same table).
static __constant__ uint32_t kSleefN[14] = {73223, 109922, 127729, 183800, 212513, 415941, 495891,
                                     639580, 691150, 717811, 753016, 920019, 941358, 942898};
static __constant__ uint32_t kSleefBits[14] = {0x41333861u, 0x4139b86du, 0x413c1f67u, 0x4141f217u, 0x414444a4u,
                                        0x414f0345u, 0x4151d367u, 0x4155e5a6u, 0x41572347u, 0x4157be4fu,
                                        0x4158826du, 0x415bb6e2u, 0x415c14ceu, 0x415c1b80u};

static __device__ __forceinline__ float torch_logf(uint32_t n) {
  if (n >= 73223u) {
#pragma unroll
    for (int k = 0; k < 14; ++k)
      if (kSleefN[k] == n) return __builtin_bit_cast(float, kSleefBits[k]);
  }
  return (float)log((double)n);
}

// ------------------------------------------------------------------------------------ waves
template <typename T> __device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Inclusive prefix sum across the wave (Hillis-Steele over shuffles).
template <typename T> __device__ __forceinline__ T wave_inclusive_scan(T v) {
  const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    T n = __shfl_up(v, o, kWave);
    if (lane >= o) v += n;
  }
  return v;
}

// ------------------------------------------------------------------------------------ errors
void set_error(const std::string& msg);

#define RTKV_HIP_CHECK(expr)                                                      \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      ::rtkv::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));       \
      return RTKV_ERR_HIP;                                                        \
    }                                                                             \
  } while (0)

#define RTKV_REQUIRE(cond, msg)                                                   \
  do {                                                                            \
    if (!(cond)) {                                                                \
      ::rtkv::set_error(std::string("rtkv: ") + (msg));                           \
      return RTKV_ERR_INVALID;                                                    \
    }                                                                             \
  } while (0)

// ------------------------------------------------------------------------------------ launchers
// (implemented in the .hip translation units; all return rtkv_status)
// K1.  Optional t2 output: t2[i] = β·log(i+1)/log(S) (fp32, the position term of the score) written
// by the batch-row-0 blocks, so K2 needs no transcendental per token.
// Optional side outputs of K1 (all nullable):
//   t2[i]      = β·log(i+1)/log(S) (fp32, the position term of the score), written by batch row 0;
//   part[b][k] = (min, max) of A over K1 block k of batch row b (2 floats), *nparts = blocks per row;
//   zero0/zero1: byte regions (multiple of 4 bytes) cleared by the K1 grid for the next kernels.
struct AggExtras {
  float* t2 = nullptr;
  float beta = 0.f;
  float logS = 1.f;
  float* part = nullptr;
  int* nparts = nullptr;
  void* zero0 = nullptr;
  size_t zero0_bytes = 0;
  void* zero1 = nullptr;
  size_t zero1_bytes = 0;
  // sequence shard: W holds rows [row0, row0 + w.S) of an S_total-row matrix (S_total = 0: unsharded).
  // Only the position of the reduction-order boundary (cascade_limit) depends on it.
  int64_t row0 = 0;
  int64_t S_total = 0;
  // device time stamp of the layer's start (rtkv_layer_times.begin, s_memrealtime), written by the
  // first block of the layer's first kernel
  unsigned long long* t_begin = nullptr;
};
// rtkv_layer_times.begin: the 100 MHz real-time counter when the layer's first block starts
__device__ __forceinline__ void stamp_begin(unsigned long long* t) {
  if (t && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0)
    *t = (unsigned long long)__builtin_amdgcn_s_memrealtime();
}
// The K1 grid clears the selection scratch of the next kernels (4-byte words, grid-strided).
__device__ __forceinline__ void zero_regions(const AggExtras& x) {
  stamp_begin(x.t_begin);
  const int64_t nb = (int64_t)gridDim.x * gridDim.y;
  const int64_t id = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  for (int r = 0; r < 2; ++r) {
    uint32_t* p = static_cast<uint32_t*>(r ? x.zero1 : x.zero0);
    const int64_t words = (int64_t)((r ? x.zero1_bytes : x.zero0_bytes) / 4);
    if (!p) continue;
    for (int64_t w = id * blockDim.x + threadIdx.x; w < words; w += nb * blockDim.x) p[w] = 0u;
  }
}
int launch_aggregation(const rtkv_attn_desc& w, int P, float* A, hipStream_t st, const AggExtras& x = AggExtras());
// scratch: [B][H][S] fp32 (qk_scratch_bytes) for the head-major kernel, or null (head-walking kernel)
size_t qk_scratch_bytes(int64_t B, int64_t H, int64_t S);
// fp32 states on the f32 MFMA (attn_f32.hip): the row LSE and the head-major K1' per-head masses
int launch_attention_lse_f32(const rtkv_qk_desc& q, float* lse, hipStream_t st);
int launch_qk_head_f32(const rtkv_qk_desc& q, int P, float* part, hipStream_t st, unsigned long long* t_begin);
// an additive key bias in raw dot-product units (bias / scale), -inf for a padding key (< -1e30)
__device__ __forceinline__ float key_bias_raw(const rtkv_qk_desc& q, int64_t b, int64_t j, float inv_scale) {
  const float v = q.kbias_dev[b * q.kbias_stride_b + j];
  return v < -1e30f ? -INFINITY : v * inv_scale;
}
int launch_qk_importance(const rtkv_qk_desc& q, int P, float* A, hipStream_t st, const AggExtras& x, int* nparts,
                         float* scratch = nullptr, size_t scratch_bytes = 0);
int launch_attention_lse(const rtkv_qk_desc& q, float* lse, hipStream_t st);
int launch_position_bias(int64_t S, float* pos, hipStream_t st);
int launch_minmax_normalize(const void* x, int dt, int64_t B, int64_t S, void* out, hipStream_t st);

struct FinalizeArgs {
  const float* A;          // aggregation (mode_scores = 1)
  const float* A_part;     // K1 per-block (min, max) of A, [B][A_nparts][2] (nullable)
  int A_nparts;
  const float* T2;         // β·pos per token from K1 (nullable: computed in place)
  int a_dtype;
  float* scores;           // written when mode_scores = 1, read otherwise
  uint8_t* labels;         // written when mode_labels = 1, read otherwise
  uint8_t* mask;           // may be null when mode_select = 0
  int32_t* kept_index;     // may be null
  int64_t* row_offset;     // may be null
  int64_t row_capacity;
  int64_t B, S, F;
  int kv_dtype;
  rtkv_layer_params p;
  float logS;              // (float)log((double)S), host libm (as Python's math.log)
  float ctx;               // (float)min(1, P/S)
  rtkv_layer_stats* stats;
  int mode_scores, mode_labels, mode_select;
  int fb_group;            // 1: select the top-10% fallback group alongside (set by launch_select)
  uint8_t* row_label;      // optional [B][cap] class of each kept row, for K4 (fast path writes it)
  rtkv_early_stats* early = nullptr;  // optional host-mapped stats mirror (fast path only)
  uint64_t early_seq = 0;
  // optional (fast path, B = 1): the rtkv_shard_ranges table of a sequence-sharded layer, written by the
  // selection's compaction phase itself — rank j's first output row and packed byte at token j·shard_S_local
  int64_t* shard_ranges = nullptr;
  int64_t shard_S_local = 0;
  int shard_nranks = 0;
};
// K2 pipeline (select.hip).  sel_ws: select_workspace_bytes(B, S) bytes; `zeroed` = its first
// select_zero_bytes(B) bytes and the stats are already zero (K1 clears them in rtkv_compress_layer).
size_t select_workspace_bytes(int64_t B, int64_t S);
size_t select_zero_bytes(int64_t B);
int launch_select(const FinalizeArgs& a, void* sel_ws, bool zeroed, hipStream_t st);
// One-launch K2 (select_fast.hip) for B = 1, S <= 65536; launch_select takes it whenever it is
// eligible.  It needs select_fast_zero_bytes() of zeroed workspace (K1 clears them).
bool select_fast_shape(int64_t B, int64_t S);
bool select_fast_eligible(const FinalizeArgs& a);
size_t select_fast_zero_bytes();
size_t select_fast_workspace_bytes(int64_t S);
int launch_select_fast(const FinalizeArgs& a, void* sel_ws, bool zeroed, hipStream_t st);

struct QuantArgs {
  rtkv_kv_desc kv;
  const uint8_t* labels;          // [B,S]
  const int32_t* kept_index;      // [B,cap] or null (all tokens)
  const uint8_t* row_label;       // [B,cap] class of each kept row, or null (then labels[kept_index])
  const rtkv_layer_stats* stats;  // kept counts / max_kept (null when kept_index is null)
  int32_t bits[3];
  rtkv_layer_out out;
  // Sequence shard (rtkv_quantize_rows_shard): kv holds tokens [row0, row0 + kv.S) of an S_glob-token
  // selection; only kept rows inside that window are processed; padding rows get their zero scale/zp on
  // every rank and their zero dequantized row only from the pad owner.
  // S_glob = 0: unsharded (S_glob = kv.S, every row processed).
  int64_t S_glob;
  int64_t row0;
  int32_t pad_owner;
  // Optional rtkv_shard_ranges table: dequantized rows go to LOCAL output row r - first_row(b, rank)
  // (packed codes and scale/zero-point keep their global positions).
  int32_t shard_rank, shard_nranks;
  const int64_t* shard_ranges;
  // rtkv_compress_layer_finish: the caller's buffers were sized from the early statistics.  out_rows > 0:
  // K'/V' hold that many rows per batch row and out.packed_capacity bytes per code plane; K4 compares them
  // with the device statistics first (RTKV_FLAG_OUTPUT_OVERFLOW, nothing written).  final_host: K4's first
  // lane publishes the layer's final flags + final_seq there.
  int64_t out_rows;
  // RTKV_FINISH_EXACT: out_rows must be max(S'_max, 1) and out.packed_capacity max(packed bytes, 1) rounded up
  // to 256 — any other size (a torn or stale read of the early line on the host) is flagged as an overflow
  int32_t exact_sizes;
  rtkv_early_stats* final_host;
  uint64_t final_seq;
  // rtkv_layer_times.end of the fused driver's layer (atomic max over K4's workgroups), or null
  unsigned long long* t_end;
};
// rtkv_layer_times.end: the waves of K4 that wrote one of the layer's last rows (kStampWindow tasks,
// quant_impl.h) stamp their end into slot (wave index mod RTKV_TIME_SLOTS), the largest stays.  Per wave, no
// barrier (a workgroup-end barrier held finished waves' slots: K4 +7 %); spread over 128-byte lines (one
// address: the atomics serialised, K4 x2).  Earlier waves end before the last rows are written.
__device__ __forceinline__ void stamp_end(unsigned long long* t, bool wrote) {
  if (!t || !wrote || (threadIdx.x & 63) != 0) return;
  const unsigned slot = ((unsigned)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % RTKV_TIME_SLOTS;
  atomicMax(t + 16 * slot, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
int launch_quant(const QuantArgs& a, hipStream_t st);


int launch_shard_ranges(const int32_t* kept_index, const int64_t* row_offset, const rtkv_layer_stats* stats, int64_t B,
                        int64_t cap, int64_t S_local, int nranks, int64_t* ranges, hipStream_t st);
int launch_prefetch_rows(const rtkv_kv_desc* kv, const int32_t* kept_index, const rtkv_layer_stats* stats,
                         int64_t max_bytes, hipStream_t st);
int launch_gather(const void* src, int64_t B, int64_t S, int64_t row_bytes, const int32_t* kept_index, int64_t cap,
                  int64_t ssb, void* dst, int64_t dsb, int64_t sss, const rtkv_layer_stats* stats, hipStream_t st);
int launch_unpack(const uint8_t* packed, const int64_t* row_offset, const float* scale_zp, int which,
                  const int32_t* kept_index, const uint8_t* labels, int64_t B, int64_t S, int64_t cap,
                  const int64_t* rows, int64_t H, int64_t D, int dt, const int32_t bits[3], void* out,
                  int64_t ob, int64_t os, int64_t oh, hipStream_t st);

size_t decode_workspace_bytes(int64_t B, int64_t Hq, int64_t Hkv, int64_t D, int64_t cap);
int launch_decode(const uint8_t* codes_k, const uint8_t* codes_v, int64_t codes_bytes, const int64_t* row_offset,
                  const float* scale_zp,
                  const int32_t* kept_index, const uint8_t* labels, int64_t B, int64_t S, int64_t cap,
                  const int64_t* rows, int64_t Hkv, int64_t D, int dt, const int32_t bits[3], const void* q,
                  int64_t Hq, float scale, float* out, void* ws, size_t ws_bytes, hipStream_t st);

int launch_tensor_params(const void* x, int dt, int64_t n_rows, int64_t row_len, const uint8_t* row_labels,
                         int label_value, int bits, float* scale_zp, void* ws, size_t ws_bytes, hipStream_t st);
int launch_tensor_fake_quant(const void* x, int dt, int64_t n_rows, int64_t row_len, const uint8_t* row_labels,
                             int label_value, int bits, const float* scale_zp, void* out, hipStream_t st);
int launch_selfcheck_division(int dt, unsigned long long* counts, hipStream_t st);
int launch_selfcheck_division_f32(int64_t s_lo, int64_t s_hi, int ex, int es, int neg, unsigned long long* counts,
                                  hipStream_t st);

}  // namespace rtkv
