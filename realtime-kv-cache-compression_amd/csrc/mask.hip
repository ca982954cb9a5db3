// mask.hip — the model-side mask check of the fused importance mode.
//
// The reference layer adds the model's additive attention_mask to the logits before its softmax
// (src/models/modified_llama.py:90-91) and passes its first S' columns to the attention after
// compression (:131-134).  The fused importance mode replaces the [B, H, S, S] softmax by the row LSE and
// K1', which take the mask as a per-key bias: exact only when the mask IS causal ∧ key padding.  This
// kernel checks that in one pass over the mask (one read per element; the last query row, which sees
// every unpadded key, is re-read from L2) and derives the key validity from that last row:
//   valid[b, j] = !(m[b, S-1, j] <= thr)           thr = finfo(dtype).min / 2 rounded to the dtype
//   entry ok    = m == 0 and (j <= i and valid[b, j])  or  m <= thr and not (j <= i and valid[b, j])
// counts[0] += entries that are not ok; counts[1] += padded keys (from the last row).  The host reads
// both with one sync.
#include "common.h"

namespace rtkv {

namespace {

template <int DT>
__global__ __launch_bounds__(256) void mask_check_kernel(const typename Dt<DT>::S* __restrict__ m, int64_t S,
                                                         int64_t sb, int64_t si, int64_t sj, float thr,
                                                         uint8_t* __restrict__ valid, int64_t valid_sb,
                                                         unsigned long long* __restrict__ counts) {
  const int64_t i = blockIdx.x;
  const int b = blockIdx.y;
  const auto* row = m + b * sb + i * si;
  const auto* last = m + b * sb + (S - 1) * si;
  uint32_t bad = 0, pad = 0;
  for (int64_t j = threadIdx.x; j < S; j += blockDim.x) {
    const float v = Dt<DT>::load(row[j * sj]);
    const bool vk = !(Dt<DT>::load(last[j * sj]) <= thr);
    const bool vis = j <= i && vk;
    const bool ok = vis ? (v == 0.f) : (v <= thr);
    bad += ok ? 0u : 1u;
    if (i == S - 1) {
      valid[b * valid_sb + j] = vk ? 1 : 0;
      pad += vk ? 0u : 1u;
    }
  }
  // one atomic per wave that has something to add
  for (int o = kWave / 2; o > 0; o >>= 1) {
    bad += __shfl_xor(bad, o, kWave);
    pad += __shfl_xor(pad, o, kWave);
  }
  if ((threadIdx.x & (kWave - 1)) == 0) {
    if (bad) atomicAdd(&counts[0], (unsigned long long)bad);
    if (pad) atomicAdd(&counts[1], (unsigned long long)pad);
  }
}

}  // namespace

}  // namespace rtkv

using namespace rtkv;

extern "C" int rtkv_mask_key_padding(const void* mask_dev, int32_t dtype, int64_t B, int64_t S, int64_t stride_b,
                                     int64_t stride_i, int64_t stride_j, float thr, uint8_t* valid_dev,
                                     int64_t valid_stride_b, unsigned long long* counts_dev, void* stream) {
  RTKV_REQUIRE(mask_dev && valid_dev && counts_dev, "mask_key_padding: null pointer");
  RTKV_REQUIRE(B >= 1 && B <= 65535 && S >= 1 && S < ((int64_t)1 << 31), "mask_key_padding: bad shape");
  const dim3 grid((unsigned)S, (unsigned)B);
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case RTKV_F32:
      hipLaunchKernelGGL(mask_check_kernel<RTKV_F32>, grid, dim3(256), 0, st, (const float*)mask_dev, S, stride_b,
                         stride_i, stride_j, thr, valid_dev, valid_stride_b, counts_dev);
      break;
    case RTKV_F16:
      hipLaunchKernelGGL(mask_check_kernel<RTKV_F16>, grid, dim3(256), 0, st, (const uint16_t*)mask_dev, S, stride_b,
                         stride_i, stride_j, thr, valid_dev, valid_stride_b, counts_dev);
      break;
    case RTKV_BF16:
      hipLaunchKernelGGL(mask_check_kernel<RTKV_BF16>, grid, dim3(256), 0, st, (const uint16_t*)mask_dev, S,
                         stride_b, stride_i, stride_j, thr, valid_dev, valid_stride_b, counts_dev);
      break;
    default:
      RTKV_REQUIRE(false, "mask_key_padding: bad dtype");
  }
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}
