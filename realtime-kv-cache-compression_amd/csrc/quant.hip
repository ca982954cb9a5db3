// quant.hip — the K4 dispatcher (per-dtype instantiations live in quant_f16/bf16/f32.hip so they
// compile in parallel), the gather, unpack (consumer), whole-tensor and self-check kernels.
// Device helpers and the K4 kernel: quant_impl.h.
#include "quant_impl.h"

namespace rtkv {

extern template int launch_quant_dt<RTKV_F32>(const QuantArgs&, hipStream_t);
extern template int launch_quant_dt<RTKV_F16>(const QuantArgs&, hipStream_t);
extern template int launch_quant_dt<RTKV_BF16>(const QuantArgs&, hipStream_t);

int launch_quant(const QuantArgs& a, hipStream_t st) {
  RTKV_REQUIRE(a.kv.k_dev && a.kv.v_dev && a.labels, "quantize_rows: null K/V/labels");
  RTKV_REQUIRE(a.kv.B >= 1 && a.kv.S >= 1 && a.kv.H >= 1 && a.kv.D >= 1, "quantize_rows: empty shape");
  RTKV_REQUIRE(!a.kept_index || a.stats, "quantize_rows: kept_index requires stats");
  RTKV_REQUIRE(!a.out.k_out_dev == !a.out.v_out_dev, "quantize_rows: k_out and v_out must both be set or both null");
  RTKV_REQUIRE(!a.out.packed_k_dev == !a.out.packed_v_dev, "quantize_rows: packed_k and packed_v must match");
  RTKV_REQUIRE(!a.out.packed_k_dev || a.out.row_offset_dev, "quantize_rows: packed output needs row offsets");
  RTKV_REQUIRE(a.out.row_capacity >= 1, "quantize_rows: row_capacity must be >= 1");
  RTKV_REQUIRE(a.kept_index || a.out.row_capacity >= a.kv.S, "quantize_rows: row_capacity < S without kept_index");
  for (int g = 0; g < 3; ++g) {
    RTKV_REQUIRE(a.bits[g] >= 1 && a.bits[g] <= 16, "quantize_rows: bits must be in [1, 16]");
    if (a.out.packed_k_dev)
      RTKV_REQUIRE(field_width(a.kv.dtype, a.bits[g]) > 0, "quantize_rows: packed codes unsupported for this dtype/bits");
  }
  switch (a.kv.dtype) {
    case RTKV_F32: return launch_quant_dt<RTKV_F32>(a, st);
    case RTKV_F16: return launch_quant_dt<RTKV_F16>(a, st);
    case RTKV_BF16: return launch_quant_dt<RTKV_BF16>(a, st);
  }
  RTKV_REQUIRE(false, "quantize_rows: bad dtype");
}

// ------------------------------------------------------------------------------------ gather
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint8_t* __restrict__ src, int64_t B, int64_t row_bytes,
                                                          const int32_t* __restrict__ kept_index, int64_t cap,
                                                          int64_t ssb, int64_t sss, uint8_t* __restrict__ dst, int64_t dsb,
                                                          const rtkv_layer_stats* __restrict__ stats) {
  const int64_t R = stats->max_kept;
  const rtkv_batch_stats* bst = reinterpret_cast<const rtkv_batch_stats*>(stats + 1);
  const int64_t db = dsb >= 0 ? dsb : R * row_bytes;
  const bool vec = ((row_bytes | ssb | sss | db) & 15) == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0;
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t t = gw; t < B * R; t += nw) {
    const int64_t b = t / R, r = t - b * R;
    uint8_t* d = dst + b * db + r * row_bytes;
    const bool keep = r < bst[b].kept;
    const uint8_t* s = keep ? src + b * ssb + (int64_t)kept_index[b * cap + r] * sss : nullptr;
    if (vec) {
      for (int64_t o = (int64_t)lane * 16; o < row_bytes; o += 64 * 16)
        *reinterpret_cast<uint4*>(d + o) = keep ? *reinterpret_cast<const uint4*>(s + o) : make_uint4(0, 0, 0, 0);
    } else {
      for (int64_t o = lane; o < row_bytes; o += 64) d[o] = keep ? s[o] : (uint8_t)0;
    }
  }
}

int launch_gather(const void* src, int64_t B, int64_t S, int64_t row_bytes, const int32_t* kept_index, int64_t cap,
                  int64_t ssb, void* dst, int64_t dsb, int64_t sss, const rtkv_layer_stats* stats, hipStream_t st) {
  RTKV_REQUIRE(src && dst && kept_index && stats, "gather_rows: null pointer");
  RTKV_REQUIRE(B >= 1 && S >= 1 && row_bytes >= 1 && cap >= 1, "gather_rows: bad shape");
  int64_t blocks = (B * (cap < S ? cap : S) + 3) / 4;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, static_cast<const uint8_t*>(src), B,
                     row_bytes, kept_index, cap, ssb, sss, static_cast<uint8_t*>(dst), dsb, stats);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

// ------------------------------------------------------------------------------------ prefetch
// The first kept rows of K and V (K4's first tasks, in K4's task order) read with the default cache
// policy and discarded, so that they sit in the Infinity Cache when K4 starts.  For the drop-in path:
// between K2's early publication and the K4 launch the host allocates the outputs and the device idles
// (~15-20 us per layer); this kernel, enqueued right after K2, uses that window.  Loads only.
__global__ __launch_bounds__(256) void prefetch_rows_kernel(const uint8_t* __restrict__ k, const uint8_t* __restrict__ v,
                                                            int64_t sss, int64_t row_bytes,
                                                            const int32_t* __restrict__ kept_index, int64_t S,
                                                            int64_t max_rows, const rtkv_layer_stats* __restrict__ stats) {
  const int64_t kept = stats->max_kept < max_rows ? stats->max_kept : max_rows;
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t r = t >> 1;
  if (r >= kept) return;
  const int64_t i = kept_index[r];
  if (i < 0 || i >= S) return;
  const uint8_t* src = ((t & 1) ? v : k) + i * sss;
  uint32_t acc = 0;
  for (int64_t o = (int64_t)lane * 16; o < row_bytes; o += 64 * 16) {
    const uint4 x = *reinterpret_cast<const uint4*>(src + o);
    acc ^= x.x ^ x.w;
  }
  asm volatile("" ::"v"(acc));  // keep the loads
}

int launch_prefetch_rows(const rtkv_kv_desc* kv, const int32_t* kept_index, const rtkv_layer_stats* stats,
                         int64_t max_bytes, hipStream_t st) {
  RTKV_REQUIRE(kv && kept_index && stats, "prefetch_kept_rows: null pointer");
  const int esz = kv->dtype == RTKV_F32 ? 4 : 2;
  const int64_t F = kv->H * kv->D;
  const int64_t row_bytes = F * esz;
  // one batch row with contiguous 16-byte aligned rows (every drop-in configuration); otherwise nothing
  const bool ok = kv->B == 1 && (kv->H == 1 || kv->stride_h == kv->D) && (row_bytes % 16) == 0 &&
                  ((kv->stride_s * esz) % 16) == 0 && (((uintptr_t)kv->k_dev | (uintptr_t)kv->v_dev) & 15) == 0;
  if (!ok || max_bytes <= 0) return RTKV_OK;
  int64_t rows = max_bytes / (2 * row_bytes);
  if (rows > kv->S) rows = kv->S;
  if (rows < 1) return RTKV_OK;
  const int64_t blocks = (2 * rows + 3) / 4;
  hipLaunchKernelGGL(prefetch_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     static_cast<const uint8_t*>(kv->k_dev), static_cast<const uint8_t*>(kv->v_dev), kv->stride_s * esz,
                     row_bytes, kept_index, kv->S, rows, stats);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

// ------------------------------------------------------------------------------------ shard ranges
// ranges[b][j] = {first output row, first packed byte} of rank j's tokens [j*S_local, (j+1)*S_local)
// (j = nranks: one past the last kept row of batch row b).  kept_index is ascending per batch row.
__global__ void shard_ranges_kernel(const int32_t* __restrict__ kept_index, const int64_t* __restrict__ row_offset,
                                    const rtkv_layer_stats* __restrict__ stats, int64_t B, int64_t cap, int64_t S_local,
                                    int nranks, int64_t* __restrict__ ranges) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * (nranks + 1)) return;
  const int64_t b = t / (nranks + 1);
  const int j = (int)(t - b * (nranks + 1));
  const rtkv_batch_stats* bst = reinterpret_cast<const rtkv_batch_stats*>(stats + 1);
  int64_t base = 0;
  for (int64_t bb = 0; bb < b; ++bb) base += bst[bb].packed_bytes;
  const int64_t kept = bst[b].kept;
  const int64_t bound = (int64_t)j * S_local;
  int64_t lo = 0, hi = kept;  // first row whose token index >= bound
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)kept_index[b * cap + mid] < bound) lo = mid + 1;
    else hi = mid;
  }
  if (j == nranks) lo = kept;
  ranges[t * 2] = lo;
  ranges[t * 2 + 1] = row_offset ? (lo < kept ? row_offset[b * cap + lo] : base + bst[b].packed_bytes) : 0;
}

int launch_shard_ranges(const int32_t* kept_index, const int64_t* row_offset, const rtkv_layer_stats* stats, int64_t B,
                        int64_t cap, int64_t S_local, int nranks, int64_t* ranges, hipStream_t st) {
  RTKV_REQUIRE(kept_index && stats && ranges, "shard_ranges: null pointer");
  RTKV_REQUIRE(B >= 1 && cap >= 1 && S_local >= 1 && nranks >= 1, "shard_ranges: bad shape");
  const int64_t n = B * (nranks + 1);
  hipLaunchKernelGGL(shard_ranges_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, kept_index, row_offset,
                     stats, B, cap, S_local, nranks, ranges);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

// ------------------------------------------------------------------------------------ unpack
template <int DT>
__global__ __launch_bounds__(256) void unpack_kernel(const uint8_t* __restrict__ packed, const int64_t* __restrict__ row_offset,
                                                     const float* __restrict__ scale_zp, int which,
                                                     const int32_t* __restrict__ kept_index, const uint8_t* __restrict__ labels,
                                                     int64_t B, int64_t S, int64_t cap, const int64_t* __restrict__ rows,
                                                     int64_t H, int64_t D, int b0, int b1, int b2,
                                                     typename Dt<DT>::S* __restrict__ out, int64_t ob, int64_t os, int64_t oh) {
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t F = H * D, nch = (F + 7) >> 3;
  const int bitsv[3] = {b0, b1, b2};
  for (int64_t t = gw; t < B * cap; t += nw) {
    const int64_t b = t / cap, r = t - b * cap;
    if (r >= rows[b]) continue;
    const int64_t i = kept_index ? kept_index[b * cap + r] : r;
    const int w = field_width(DT, bitsv[labels[b * S + i]]);
    RowParams rp;
    rp.scale = scale_zp[(b * cap + r) * 4 + which * 2];
    rp.zp = scale_zp[(b * cap + r) * 4 + which * 2 + 1];
    const uint8_t* src = packed + row_offset[b * cap + r];
    for (int64_t c = lane; c < nch; c += 64) {
      const int64_t f0 = c * 8;
      const int nvalid = (F - f0) < 8 ? (int)(F - f0) : 8;
      const uint8_t* p = src + c * w;
      const int nb = (nvalid * w + 7) >> 3;
      uint64_t wd[3] = {0, 0, 0};
      for (int k = 0; k < nb; ++k) wd[k >> 3] |= (uint64_t)p[k] << ((k & 7) * 8);
      const uint64_t m = (w >= 64) ? ~0ull : ((1ull << w) - 1ull);
      for (int e = 0; e < nvalid; ++e) {
        const int bit = e * w, word = bit >> 6, sh = bit & 63;
        uint64_t v = wd[word] >> sh;
        if (sh && word < 2) v |= wd[word + 1] << (64 - sh);
        const float q = (float)(uint32_t)(v & m);
        const int64_t f = f0 + e;
        out[b * ob + r * os + (f / D) * oh + (f % D)] = Dt<DT>::store(dequant<DT>(q, rp));
      }
    }
  }
}

int launch_unpack(const uint8_t* packed, const int64_t* row_offset, const float* scale_zp, int which,
                  const int32_t* kept_index, const uint8_t* labels, int64_t B, int64_t S, int64_t cap,
                  const int64_t* rows, int64_t H, int64_t D, int dt, const int32_t bits[3], void* out,
                  int64_t ob, int64_t os, int64_t oh, hipStream_t st) {
  RTKV_REQUIRE(packed && row_offset && scale_zp && labels && rows && out, "unpack: null pointer");
  RTKV_REQUIRE(B >= 1 && S >= 1 && cap >= 1 && H >= 1 && D >= 1, "unpack: bad shape");
  for (int g = 0; g < 3; ++g) RTKV_REQUIRE(field_width(dt, bits[g]) > 0, "unpack: unsupported bits");
  int64_t blocks = (B * cap + 3) / 4;
  if (blocks > 2048) blocks = 2048;
  switch (dt) {
#define RTKV_U(DT)                                                                                          \
  case DT:                                                                                                  \
    hipLaunchKernelGGL(unpack_kernel<DT>, dim3((unsigned)blocks), dim3(256), 0, st, packed, row_offset,     \
                       scale_zp, which, kept_index, labels, B, S, cap, rows, H, D, bits[0], bits[1],       \
                       bits[2], static_cast<typename Dt<DT>::S*>(out), ob, os, oh);                         \
    break;
    RTKV_U(RTKV_F32) RTKV_U(RTKV_F16) RTKV_U(RTKV_BF16)
#undef RTKV_U
    default:
      RTKV_REQUIRE(false, "unpack: bad dtype");
  }
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

// ------------------------------------------------------------------------------------ whole-tensor helpers
// get_quantization_params over all elements of the rows whose label equals label_value (or every row
// when row_labels is null): per-block min/max partials, then one block folds them.
template <int DT>
__global__ __launch_bounds__(256) void tensor_minmax_kernel(const typename Dt<DT>::S* __restrict__ x, int64_t n_rows,
                                                            int64_t row_len, const uint8_t* __restrict__ row_labels,
                                                            int label_value, float* __restrict__ partial) {
  __shared__ float red[2][4];
  float mn = INFINITY, mx = -INFINITY;
  const int64_t n = n_rows * row_len;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    if (row_labels && row_labels[e / row_len] != label_value) continue;
    const float v = Dt<DT>::load(x[e]);
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { red[0][wid] = mn; red[1][wid] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    mn = red[0][0];
    mx = red[1][0];
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) { mn = fminf(mn, red[0][k]); mx = fmaxf(mx, red[1][k]); }
    partial[2 * blockIdx.x] = mn;
    partial[2 * blockIdx.x + 1] = mx;
  }
}

template <int DT>
__global__ void tensor_params_kernel(const float* __restrict__ partial, int nblocks, int bits, float* __restrict__ scale_zp) {
  if (threadIdx.x != 0) return;
  float mn = INFINITY, mx = -INFINITY;
  for (int k = 0; k < nblocks; ++k) { mn = fminf(mn, partial[2 * k]); mx = fmaxf(mx, partial[2 * k + 1]); }
  if (!(mn <= mx)) { mn = mx = 0.f; }  // no element selected
  const RowParams rp = row_params<DT>(mn, mx, bits);
  scale_zp[0] = rp.scale;
  scale_zp[1] = rp.zp;
}

template <int DT>
__global__ __launch_bounds__(256) void tensor_fake_quant_kernel(const typename Dt<DT>::S* __restrict__ x, int64_t n_rows,
                                                                int64_t row_len, const uint8_t* __restrict__ row_labels,
                                                                int label_value, int bits, const float* __restrict__ scale_zp,
                                                                typename Dt<DT>::S* __restrict__ out) {
  const RowParams rp0 = {scale_zp[0], scale_zp[1], 0.f};
  RowParams rp = rp0;
  rp.qmaxT = Dt<DT>::rnd((float)((1u << bits) - 1u));
  const int64_t n = n_rows * row_len;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    if (row_labels && row_labels[e / row_len] != label_value) continue;
    out[e] = Dt<DT>::store(dequant<DT>(quant_code<DT>(Dt<DT>::load(x[e]), rp), rp));
  }
}

int launch_tensor_params(const void* x, int dt, int64_t n_rows, int64_t row_len, const uint8_t* row_labels,
                         int label_value, int bits, float* scale_zp, void* ws, size_t ws_bytes, hipStream_t st) {
  RTKV_REQUIRE(x && scale_zp && ws, "tensor_quant_params: null pointer");
  RTKV_REQUIRE(n_rows >= 1 && row_len >= 1, "tensor_quant_params: empty tensor");
  RTKV_REQUIRE(bits >= 1 && bits <= 16, "tensor_quant_params: bits must be in [1, 16]");
  int64_t nblocks = (n_rows * row_len + 255) / 256;
  if (nblocks > 1024) nblocks = 1024;
  RTKV_REQUIRE(ws_bytes >= (size_t)nblocks * 8, "tensor_quant_params: workspace too small");
  float* partial = static_cast<float*>(ws);
  switch (dt) {
#define RTKV_T(DT)                                                                                                   \
  case DT:                                                                                                           \
    hipLaunchKernelGGL(tensor_minmax_kernel<DT>, dim3((unsigned)nblocks), dim3(256), 0, st,                          \
                       static_cast<const typename Dt<DT>::S*>(x), n_rows, row_len, row_labels, label_value, partial); \
    hipLaunchKernelGGL(tensor_params_kernel<DT>, dim3(1), dim3(64), 0, st, partial, (int)nblocks, bits, scale_zp);   \
    break;
    RTKV_T(RTKV_F32) RTKV_T(RTKV_F16) RTKV_T(RTKV_BF16)
#undef RTKV_T
    default:
      RTKV_REQUIRE(false, "tensor_quant_params: bad dtype");
  }
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

int launch_tensor_fake_quant(const void* x, int dt, int64_t n_rows, int64_t row_len, const uint8_t* row_labels,
                             int label_value, int bits, const float* scale_zp, void* out, hipStream_t st) {
  RTKV_REQUIRE(x && scale_zp && out, "tensor_fake_quant: null pointer");
  RTKV_REQUIRE(n_rows >= 1 && row_len >= 1, "tensor_fake_quant: empty tensor");
  RTKV_REQUIRE(bits >= 1 && bits <= 16, "tensor_fake_quant: bits must be in [1, 16]");
  int64_t nblocks = (n_rows * row_len + 255) / 256;
  if (nblocks > 4096) nblocks = 4096;
  switch (dt) {
#define RTKV_T(DT)                                                                                          \
  case DT:                                                                                                  \
    hipLaunchKernelGGL(tensor_fake_quant_kernel<DT>, dim3((unsigned)nblocks), dim3(256), 0, st,             \
                       static_cast<const typename Dt<DT>::S*>(x), n_rows, row_len, row_labels, label_value, \
                       bits, scale_zp, static_cast<typename Dt<DT>::S*>(out));                               \
    break;
    RTKV_T(RTKV_F32) RTKV_T(RTKV_F16) RTKV_T(RTKV_BF16)
#undef RTKV_T
    default:
      RTKV_REQUIRE(false, "tensor_fake_quant: bad dtype");
  }
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}


// ------------------------------------------------------------------------------------ self-check
// Exhaustive proof obligation of fast_quotient: every (dividend, positive divisor) pair of the 16-bit
// dtype admitted by fast_div_ok is compared bitwise with the IEEE division.  counts = {checked, bad}.
template <int DT>
__global__ __launch_bounds__(256) void selfcheck_division_kernel(unsigned long long* counts) {
  const float s = Dt<DT>::load((uint16_t)(blockIdx.x + 1));  // 0x0001 .. 0x7fff: every positive pattern
  const float r = 1.f / s;
  unsigned long long checked = 0, bad = 0;
  for (uint32_t xb = threadIdx.x; xb < 65536u; xb += blockDim.x) {
    const float x = Dt<DT>::load((uint16_t)xb);
    const float ax = __builtin_fabsf(x);
    if (!(ax < INFINITY)) continue;  // finite dividends only (NaN fails the test)
    // a row admits x iff fast_div_ok(s, amax, amin_nz) with amax >= |x| and, for x != 0, amin_nz <= |x|;
    // the pair is therefore reachable iff fast_div_ok(s, |x|, x != 0 ? |x| : +inf)
    if (!fast_div_ok<DT>(s, ax, x != 0.f ? ax : INFINITY)) continue;
    const float q = fast_quotient(x, s, r);
    const float ref = x / s;
    ++checked;
    bad += __builtin_bit_cast(uint32_t, q) != __builtin_bit_cast(uint32_t, ref);
  }
  for (int o = 32; o > 0; o >>= 1) {
    checked += __shfl_xor(checked, o);
    bad += __shfl_xor(bad, o);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(counts, checked);
    atomicAdd(counts + 1, bad);
  }
}

// fp32: the pairs (x, s) = (X·2^ex, S·2^es) with X = 1 + xm·2^-23 over EVERY mantissa xm, and
// S = 1 + sm·2^-23 for sm in [s_lo, s_hi) (one workgroup per divisor); ex = es = 0 is the
// mantissa-exhaustive proof obligation (see fast_div_ok), other exponents check the scaling
// argument.  neg: negative dividends.  Only pairs the row gate admits are counted.
__global__ __launch_bounds__(256) void selfcheck_division_f32_kernel(int64_t s_lo, float xscale, float sscale,
                                                                     int neg, unsigned long long* counts) {
  const uint32_t sm = (uint32_t)(s_lo + blockIdx.x);
  const float s = __uint_as_float(0x3f800000u | sm) * sscale;
  const float r = 1.f / s;
  const float sg = neg ? -xscale : xscale;
  unsigned long long checked = 0, bad = 0;
  for (uint32_t xm = threadIdx.x; xm < (1u << 23); xm += blockDim.x) {
    const float x = __uint_as_float(0x3f800000u | xm) * sg;
    const float ax = __builtin_fabsf(x);
    if (!fast_div_ok<RTKV_F32>(s, ax, ax)) continue;
    const float q = fast_quotient(x, s, r);
    const float ref = x / s;
    ++checked;
    bad += __builtin_bit_cast(uint32_t, q) != __builtin_bit_cast(uint32_t, ref);
  }
  for (int o = 32; o > 0; o >>= 1) {
    checked += __shfl_xor(checked, o);
    bad += __shfl_xor(bad, o);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(counts, checked);
    atomicAdd(counts + 1, bad);
  }
}

int launch_selfcheck_division_f32(int64_t s_lo, int64_t s_hi, int ex, int es, int neg, unsigned long long* counts,
                                  hipStream_t st) {
  RTKV_REQUIRE(counts, "selfcheck_division_f32: null counts");
  RTKV_REQUIRE(0 <= s_lo && s_lo < s_hi && s_hi <= ((int64_t)1 << 23), "selfcheck_division_f32: bad divisor range");
  RTKV_REQUIRE(ex >= -126 && ex <= 127 && es >= -126 && es <= 127, "selfcheck_division_f32: bad exponents");
  hipLaunchKernelGGL(selfcheck_division_f32_kernel, dim3((unsigned)(s_hi - s_lo)), dim3(256), 0, st, s_lo,
                     ldexpf(1.f, ex), ldexpf(1.f, es), neg, counts);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

int launch_selfcheck_division(int dt, unsigned long long* counts, hipStream_t st) {
  RTKV_REQUIRE(counts, "selfcheck_division: null counts");
  RTKV_HIP_CHECK(hipMemsetAsync(counts, 0, 2 * sizeof(unsigned long long), st));
  if (dt == RTKV_F16) hipLaunchKernelGGL((selfcheck_division_kernel<RTKV_F16>), dim3(0x7fff), dim3(256), 0, st, counts);
  else if (dt == RTKV_BF16) hipLaunchKernelGGL((selfcheck_division_kernel<RTKV_BF16>), dim3(0x7fff), dim3(256), 0, st, counts);
  else {
    set_error("rtkv: selfcheck_division: fp32 is checked per divisor range (rtkv_selfcheck_division_f32)");
    return RTKV_ERR_UNSUPPORTED;
  }
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

}  // namespace rtkv
