// decode.hip — decode attention over packed KV: the split merge, the launch
// geometry and the C-ABI side; the split kernel and its design notes are in decode_kernel.h (fp16
// instantiations: decode_f16.hip).
#include "decode_kernel.h"

namespace rtkv {

namespace {

// out[b, hq, d] = Σ_s e^{m_s - m*} acc_s / Σ_s e^{m_s - m*} l_s over the splits.  Workgroup of
// 16 features × 64 split phases (phase p takes splits ≡ p mod 64), combined through LDS.
constexpr int kMF = 16, kMP = 64;
__global__ __launch_bounds__(kMF * kMP) void decode_merge_kernel(DecodeArgs a) {
  __shared__ float red[3][kMP][kMF];
  const int F = a.Hkv * a.D;
  const int fl = threadIdx.x % kMF, ph = threadIdx.x / kMF;
  const int f = blockIdx.x * kMF + fl;
  const int g = blockIdx.y, b = blockIdx.z;
  const bool ok = f < F;
  const int hk = ok ? f / a.D : 0, d = f - hk * a.D;
  const int64_t base = ((int64_t)b * a.G + g) * a.splits;
  float mm = -INFINITY;
  for (int s = ph; s < a.splits; s += kMP) mm = fmaxf(mm, a.part_m[(base + s) * a.Hkv + hk]);
  red[0][ph][fl] = mm;
  __syncthreads();
  mm = red[0][0][fl];
#pragma unroll
  for (int p = 1; p < kMP; ++p) mm = fmaxf(mm, red[0][p][fl]);
  float num = 0.f, den = 0.f;
  if (mm != -INFINITY && ok) {
#pragma unroll 4
    for (int s = ph; s < a.splits; s += kMP) {
      const float ms = a.part_m[(base + s) * a.Hkv + hk];
      const float fct = ms == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(ms - mm);
      num += fct * a.part_acc[(base + s) * F + f];
      den += fct * a.part_l[(base + s) * a.Hkv + hk];
    }
  }
  red[1][ph][fl] = num;
  red[2][ph][fl] = den;
  __syncthreads();
  if (ph != 0 || !ok) return;
#pragma unroll
  for (int p = 1; p < kMP; ++p) {
    num += red[1][p][fl];
    den += red[2][p][fl];
  }
  const int Hq = a.Hkv * a.G;
  a.out[((int64_t)b * Hq + (int64_t)hk * a.G + g) * a.D + d] = den > 0.f ? num / den : 0.f;
}

// Per-lane shape: GQ query heads of a kv head share each decoded K'/V' chunk; NCH chunks per lane
// (GQ · NCH ≤ 4 keeps the accumulators at ≤ 32 VGPRs).
struct DecodeShape {
  int nch, gq, hg, gs;
};
DecodeShape decode_shape(int64_t F, int64_t G) {
  DecodeShape d;
  d.gq = G % 4 == 0 ? 4 : (G % 2 == 0 ? 2 : 1);
  d.nch = ((F / 512) % 2 == 0 && d.gq == 1) ? 2 : 1;
  d.hg = (int)(F / 512) / d.nch;
  d.gs = (int)(G / d.gq);
  return d;
}

int decode_target_wgs() {
  static const int t = [] {
    const char* e = std::getenv("RTKV_DECODE_WGS");  // tuning knob, default 1024 workgroups
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : 1024;
  }();
  return t;
}

int decode_splits(int64_t B, int64_t G, int64_t F, int64_t cap) {
  const DecodeShape d = decode_shape(F, G);
  int64_t s = (cap + 16 * kDW - 1) / (16 * kDW);    // at least ~16 rows per wave
  const int64_t wg = B * d.gs * (d.hg > 0 ? d.hg : 1);
  const int64_t target = decode_target_wgs() / (wg > 0 ? wg : 1);
  if (s > target) s = target;
  if (s < 1) s = 1;
  return (int)s;
}

}  // namespace

size_t decode_workspace_bytes(int64_t B, int64_t Hq, int64_t Hkv, int64_t D, int64_t cap) {
  const int64_t G = Hkv > 0 ? Hq / Hkv : 1;
  const int64_t s = decode_splits(B, G, Hkv * D, cap);
  return (size_t)(B * G * s) * (size_t)(2 * Hkv + Hkv * D) * sizeof(float) + 256;
}

int launch_decode(const uint8_t* codes_k, const uint8_t* codes_v, int64_t codes_bytes, const int64_t* row_offset,
                  const float* scale_zp,
                  const int32_t* kept_index, const uint8_t* labels, int64_t B, int64_t S, int64_t cap,
                  const int64_t* rows, int64_t Hkv, int64_t D, int dt, const int32_t bits[3], const void* q,
                  int64_t Hq, float scale, float* out, void* ws, size_t ws_bytes, hipStream_t st) {
  RTKV_REQUIRE(codes_k && codes_v && row_offset && scale_zp && kept_index && labels && rows && q && out,
               "decode: null pointer");
  RTKV_REQUIRE(B >= 1 && S >= 1 && cap >= 1 && Hkv >= 1 && D >= 1 && Hq >= Hkv && Hq % Hkv == 0,
               "decode: bad shape");
  RTKV_REQUIRE(B <= 65535, "decode: grid too large");
  const int64_t F = Hkv * D;
  const int64_t G = Hq / Hkv;
  RTKV_REQUIRE(F % 512 == 0, "decode: Hkv*D must be a multiple of 512");
  RTKV_REQUIRE(D % 8 == 0 && 64 % (D / 8) == 0, "decode: head_dim must be 8·2^k with 8 <= head_dim <= 512");
  DecodeArgs a;
  std::memset(&a, 0, sizeof(a));
  for (int k = 0; k < 3; ++k) {
    a.w[k] = field_width(dt, bits[k]);
    RTKV_REQUIRE(a.w[k] == 2 || a.w[k] == 4 || a.w[k] == 8 || a.w[k] == 16,
                 "decode: packed field widths 2/4/8/16 only");
  }
  RTKV_REQUIRE(((uintptr_t)q & 15) == 0 && ((uintptr_t)scale_zp & 15) == 0, "decode: q and scale_zp must be 16-byte aligned");
  const int splits = decode_splits(B, G, F, cap);
  RTKV_REQUIRE(ws && ws_bytes >= decode_workspace_bytes(B, Hq, Hkv, D, cap), "decode: workspace too small");
  RTKV_REQUIRE(codes_bytes >= 0, "decode: negative code buffer size");
  a.codes_k = codes_k; a.codes_v = codes_v; a.codes_bytes = codes_bytes; a.row_offset = row_offset; a.scale_zp = scale_zp;
  a.kept_index = kept_index; a.labels = labels; a.rows = rows;
  a.S = S; a.cap = cap; a.Hkv = (int)Hkv; a.D = (int)D; a.G = (int)G;
  a.q = q; a.scale = scale * 1.4426950408889634f; a.splits = splits;
  float* p = static_cast<float*>(ws);
  a.part_m = p;
  p += B * G * splits * Hkv;
  a.part_l = p;
  p += B * G * splits * Hkv;
  a.part_acc = p;
  a.out = out;
  const DecodeShape sh = decode_shape(F, G);
  a.HG = sh.hg;
  a.GS = sh.gs;
  a.nrest = (int)((int64_t)splits * a.HG * B);
  const int64_t nblk = ((int64_t)a.nrest + 7) / 8 * 8 * a.GS;
  RTKV_REQUIRE(nblk < (1ll << 31), "decode: grid too large");
  const dim3 grid((unsigned)nblk);
  const size_t lds = (size_t)kDW * 64 * sh.nch * sh.gq * 10 * sizeof(float);
  int rc;
  if (dt == RTKV_F16) rc = launch_decode_split_f16(a, sh.nch, sh.gq, (int)D, grid, lds, st);
  else if (dt == RTKV_BF16) rc = launch_decode_split<RTKV_BF16>(a, sh.nch, sh.gq, (int)D, grid, lds, st);
  else rc = launch_decode_split<RTKV_F32>(a, sh.nch, sh.gq, (int)D, grid, lds, st);
  if (rc != RTKV_OK) return rc;
  hipLaunchKernelGGL(decode_merge_kernel, dim3((unsigned)((F + kMF - 1) / kMF), (unsigned)G, (unsigned)B),
                     dim3(kMF * kMP), 0, st, a);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

}  // namespace rtkv
