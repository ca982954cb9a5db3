// select_fast.hip — host side of the one-launch K2 (device code: select_fast.h) and of the fused
// K2 + K4 launch (fused.h; per-dtype instantiations in fused_{f32,f16,bf16}.hip).
#include "select_fast.h"

namespace rtkv {

// ------------------------------------------------------------------------------------ host
bool select_fast_shape(int64_t B, int64_t S) { return B == 1 && S >= 1 && S <= kMaxS; }

bool select_fast_eligible(const FinalizeArgs& f) {
  return select_fast_shape(f.B, f.S) && !(f.p.flags & RTKV_SELECT_PIPELINE) && f.mode_scores && f.mode_labels &&
         (f.mode_select == 1 || f.mode_select == 2) && f.mask && f.kept_index;
}

// Workspace: [FastHead][hist][partials][slots]; the first select_fast_zero_bytes() must be zero
// before the launch (K1 clears them in rtkv_compress_layer).
size_t select_fast_zero_bytes() { return sizeof(FastHead) + (size_t)kGrp * kNBin * 4; }
size_t select_fast_workspace_bytes(int64_t) {
  return select_fast_zero_bytes() + kMaxG * sizeof(FastPartial) + 256 + (size_t)kGrp * kNBin * kCap * 8;
}

template <int TPT, bool HAS_T2, int DT> static int launch_fsel(const FastArgs& g, int G, hipStream_t st) {
  const size_t lds = (size_t)kGrp * kNBin * sizeof(uint32_t);
  static bool attr = false;  // per instantiation
  if (!attr) {
    RTKV_HIP_CHECK(hipFuncSetAttribute((const void*)fsel_kernel<TPT, HAS_T2, DT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  hipLaunchKernelGGL((fsel_kernel<TPT, HAS_T2, DT>), dim3(G), dim3(kST), lds, st, g);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

template <int TPT, bool HAS_T2> static int launch_fsel_dt(const FastArgs& g, int G, hipStream_t st) {
  switch (g.f.a_dtype) {
    case RTKV_F16: return launch_fsel<TPT, HAS_T2, RTKV_F16>(g, G, st);
    case RTKV_BF16: return launch_fsel<TPT, HAS_T2, RTKV_BF16>(g, G, st);
    default: return launch_fsel<TPT, HAS_T2, RTKV_F32>(g, G, st);
  }
}

int launch_select_fast(const FinalizeArgs& f, void* ws, bool zeroed, hipStream_t st) {
  RTKV_REQUIRE(select_fast_eligible(f), "select_fast: not eligible");
  FastArgs g = make_fast_args(f, ws);
  if (!zeroed) {  // else K1 cleared them
    RTKV_HIP_CHECK(hipMemsetAsync(ws, 0, select_fast_zero_bytes(), st));
    RTKV_HIP_CHECK(hipMemsetAsync(f.stats, 0, rtkv_stats_bytes(f.B), st));
  }
  // All G <= 32 workgroups (1024 threads, 64 KB of LDS: one per CU) are resident at once, which the
  // waits of phases 2 and 3 rely on; a busy GPU only delays the last ones.
  const int G = (int)((f.S + kST - 1) / kST);
  if (f.S <= 16 * kST) return f.T2 ? launch_fsel_dt<16, true>(g, G, st) : launch_fsel_dt<16, false>(g, G, st);
  return f.T2 ? launch_fsel_dt<32, true>(g, G, st) : launch_fsel_dt<32, false>(g, G, st);
}

// ------------------------------------------------------------------------------------ fused K2 + K4
int launch_fused_f32(const FinalizeArgs& f, void* sel_ws, const QuantArgs& q, hipStream_t st);
int launch_fused_f16(const FinalizeArgs& f, void* sel_ws, const QuantArgs& q, hipStream_t st);
int launch_fused_bf16(const FinalizeArgs& f, void* sel_ws, const QuantArgs& q, hipStream_t st);

bool fused_eligible(const FinalizeArgs& f, const QuantArgs& q) {
  if (!(f.p.flags & RTKV_FUSED_QUANT) || !select_fast_eligible(f) || !f.T2 || !f.row_label) return false;
  const rtkv_kv_desc& kv = q.kv;
  if (kv.B != 1 || kv.S != f.S || q.S_glob != 0 || q.shard_ranges || q.kept_index != f.kept_index) return false;
  const int64_t F = kv.H * kv.D;
  if (F != f.F || !(F == 4096 || (F == 5120 && kv.dtype != RTKV_F32))) return false;
  if (!(kv.dtype == f.a_dtype || f.a_dtype == RTKV_F32)) return false;
  const int esz = kv.dtype == RTKV_F32 ? 4 : 2;
  auto al16 = [](const void* p) { return p == nullptr || ((uintptr_t)p % 16) == 0; };
  // contiguous rows: element e of a row at e (input and dequantized output), 16-byte aligned
  if (!(kv.H == 1 || kv.stride_h == kv.D) || (kv.stride_s * esz) % 16 != 0 || !al16(kv.k_dev) || !al16(kv.v_dev))
    return false;
  if (q.out.k_out_dev && (!(kv.H == 1 || q.out.o_stride_h == kv.D) || (q.out.o_stride_s * esz) % 16 != 0 ||
                          !al16(q.out.k_out_dev) || !al16(q.out.v_out_dev)))
    return false;
  if (q.out.packed_k_dev) {
    if (!al16(q.out.packed_k_dev) || !al16(q.out.packed_v_dev) || !q.out.row_offset_dev) return false;
    for (int g = 0; g < 3; ++g) {
      const int w = field_width(kv.dtype, q.bits[g]);
      if (!(w == 2 || w == 4 || w == 8 || w == 16)) return false;
    }
  }
  return q.out.row_capacity >= f.S;
}

int launch_select_quant_fused(const FinalizeArgs& f, void* sel_ws, const QuantArgs& q, hipStream_t st) {
  RTKV_REQUIRE(fused_eligible(f, q), "fused selection + quantization: not eligible");
  switch (q.kv.dtype) {
    case RTKV_F32: return launch_fused_f32(f, sel_ws, q, st);
    case RTKV_F16: return launch_fused_f16(f, sel_ws, q, st);
    case RTKV_BF16: return launch_fused_bf16(f, sel_ws, q, st);
  }
  RTKV_REQUIRE(false, "fused selection + quantization: bad dtype");
}

}  // namespace rtkv
