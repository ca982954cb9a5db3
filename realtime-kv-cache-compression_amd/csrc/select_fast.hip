// select_fast.hip — host side of the one-launch K2 (device code: select_fast.h).
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

template <bool HAS_T2> static int launch_fsel_quant(const FastArgs& g, int G, hipStream_t st) {
  switch (g.f.a_dtype) {
    case RTKV_F16: hipLaunchKernelGGL((fsel_quant_kernel<HAS_T2, RTKV_F16>), dim3(G), dim3(kST), 0, st, g); break;
    case RTKV_BF16: hipLaunchKernelGGL((fsel_quant_kernel<HAS_T2, RTKV_BF16>), dim3(G), dim3(kST), 0, st, g); break;
    default: hipLaunchKernelGGL((fsel_quant_kernel<HAS_T2, RTKV_F32>), dim3(G), dim3(kST), 0, st, g); break;
  }
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
  // All G <= 64 workgroups (1024 threads, 64 KB of LDS: one per CU) are resident at once, which the
  // waits of phases 2 and 3 rely on; a busy GPU only delays the last ones.
  const int G = (int)((f.S + kST - 1) / kST);
  // quantization only (RTKV_NO_SELECTION): scores, classes and row offsets, no selection phases
  // (RTKV_SELECT_QUANT_FULL keeps the selection kernel's mode 2 for A/B checks)
  static const bool quant_full = getenv("RTKV_SELECT_QUANT_FULL") != nullptr;
  if (f.mode_select == 2 && !quant_full) return f.T2 ? launch_fsel_quant<true>(g, G, st) : launch_fsel_quant<false>(g, G, st);
  if (f.S <= 16 * kST) return f.T2 ? launch_fsel_dt<16, true>(g, G, st) : launch_fsel_dt<16, false>(g, G, st);
  if (f.S <= 32 * kST) return f.T2 ? launch_fsel_dt<32, true>(g, G, st) : launch_fsel_dt<32, false>(g, G, st);
  return f.T2 ? launch_fsel_dt<64, true>(g, G, st) : launch_fsel_dt<64, false>(g, G, st);
}

}  // namespace rtkv
