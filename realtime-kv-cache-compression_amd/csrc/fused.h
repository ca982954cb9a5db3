// fused.h — K2 + K4 in ONE launch for one batch row (B = 1, S <= 32768): the selection of
// select_fast.h in workgroups 0..G−1, and the per-row quantization + pack + compaction of quant_impl.h
// in the workgroups after them, which start on the selection's early hand-offs instead of waiting for
// the end of a separate K2 launch.
//
// Reference, as the two kernels it fuses: token_importance.py:134-176, dynamic_quantization.py:21-196,
// selective_propagation.py:68-232 (one layer of unified_compressor.py:95-172).
//
// Why: the reference caller compresses one layer at a time (modified_llama.py:113-157), so K2's ~20 µs
// chain of cross-workgroup round trips is fully exposed between K1 and K4, with 240 of 256 CUs idle.
// Here the quantization waves are resident from the start of the launch and
//   1. wait for the MODE word (sel[6]: per group ALL / PART / NONE and the fallback flag), which the
//      selecting workgroup publishes as soon as the class counts give the quotas — before any
//      histogram or threshold work;
//   2. take one task each (token i, tensor K or V) in token order, read the token's score and class
//      (tokinfo[i], a tagged word phase 1 stores), and skip dropped tokens without reading their row: NONE → dropped, ALL → kept, PART → compare with the group's
//      threshold key (sel[q], published at the end of phase 2); ties at the threshold are decided by
//      phase 3;
//   3. load the row, reduce min/max and the row parameters, and only then wait for the token's output
//      position (tokrow[i]: the kept rows of each class before it, from phase 3's look-back) to store
//      the scale/zero-point, the packed codes and the dequantized row.
// Every wait is bounded (wait_word): a hand-off that never comes flags RTKV_FLAG_SPIN_TIMEOUT and the
// waves drain their remaining tasks without reading rows.
//
// Forward progress: workgroups are dispatched in index order, so the G selection workgroups are
// resident before any quantization workgroup (which only ever waits on them); they are the same
// co-resident set the one-launch K2 already relies on.
#pragma once
#include "quant_impl.h"
#include "select_fast.h"

namespace rtkv {
namespace {

struct FusedArgs {
  FastArgs g;
  QuantArgs q;
};

__device__ __forceinline__ uint64_t uni64(uint64_t w) {  // wave-uniform copy (every lane loaded the same word)
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)w), hi = __builtin_amdgcn_readfirstlane((uint32_t)(w >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// Wave-uniform bounded wait for a tagged word (every lane loads the same address).  `broken`: a wait
// of this wave already timed out (or another wave's did), so the layer is lost: return at once.
__device__ __forceinline__ uint64_t wait_word(const uint64_t* p, uint32_t limit, rtkv_layer_stats* stats, bool& broken) {
  if (broken) return 0;
  uint64_t w = ld_sc1(p);
  for (uint32_t it = 0; !(w & kTag); ++it) {
    if (it >= limit || ((it & 1023u) == 1023u && (ld_sc1(&stats->error_flags) & RTKV_FLAG_SPIN_TIMEOUT))) {
      if ((threadIdx.x & (kWave - 1)) == 0) atomicOr(&stats->error_flags, (int)RTKV_FLAG_SPIN_TIMEOUT);
      broken = true;
      return 0;
    }
    __builtin_amdgcn_s_sleep(1);
    w = ld_sc1(p);
  }
  return uni64(w);
}

template <typename T> __device__ __forceinline__ T pick3(int k, T a0, T a1, T a2) { return k == 0 ? a0 : (k == 1 ? a1 : a2); }
template <typename T> __device__ __forceinline__ T pick4(int k, const T (&v)[4]) {
  return k == 0 ? v[0] : (k == 1 ? v[1] : (k == 2 ? v[2] : v[3]));
}

// The quantization waves (workgroups G.. of the launch).  ADT: dtype of A (scores are computed in it),
// KDT: dtype of K/V; rows are contiguous [S, F] with F = NCH * 512.
template <int ADT, int KDT, int NCH>
__device__ __forceinline__ void k4_tasks(const FusedArgs& x) {
  using S_ = typename Dt<KDT>::S;
  const FastArgs& g = x.g;
  const FinalizeArgs& a = g.f;
  const QuantArgs& q = x.q;
  const int lane = threadIdx.x & (kWave - 1);
  const int S = (int)a.S;
  const uint32_t ntask = 2u * (uint32_t)S;
  FastHead* head = g.L.head;
  bool broken = false;
  // ---- per-class packed widths and row bytes (selective_propagation.py byte offsets of the codes)
  int wid3[3];
  int64_t rb[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    wid3[k] = field_width(KDT, a.p.bits[k]);
    rb[k] = ((int64_t)a.F * wid3[k] + 7) / 8;
  }
  const bool emit_deq = q.out.k_out_dev != nullptr;
  const bool emit_pk = q.out.packed_k_dev != nullptr;
  const int nch = NCH * 64;
  // One task (token*2 + tensor) per wave, in token order over the quantization workgroups.  Not a
  // persistent loop: on gfx9 one counter (vmcnt) tracks loads and stores in order, so a wave that went
  // on to its next task would wait for its previous task's stores before its next loads could be used;
  // a wave that ends after its stores lets them drain while a new wave starts.
  const uint32_t t = (uint32_t)(blockIdx.x - (a.S + kST - 1) / kST) * (kST / kWave) + (uint32_t)(threadIdx.x / kWave);
  if (t >= ntask) return;
  {
    const int r = (int)(t >> 1), which = (int)(t & 1u);
    // ---- the kept row count (published with the quotas): rows beyond it end here, long before the
    // selection is done; then this row's token, class and packed offset (phase 3)
    const uint64_t m6 = wait_word(&head->sel[6], g.spin_limit, a.stats, broken);
    if (broken || r >= (int)((m6 >> 16) & 0xffffffu)) return;
    uint64_t w0 = uni64(ld_sc1(&head->rowinfo[r][0]));
    uint64_t w1 = uni64(ld_sc1(&head->rowinfo[r][1]));
    if (!(w0 & kTag)) w0 = wait_word(&head->rowinfo[r][0], g.spin_limit, a.stats, broken);
    if (!(w1 & kTag)) w1 = wait_word(&head->rowinfo[r][1], g.spin_limit, a.stats, broken);
    if (broken) return;
    const int i = (int)(uint32_t)w0, l = (int)((w0 >> 32) & 3u);
    if ((unsigned)i >= (unsigned)S) return;
    const int64_t k0 = (int64_t)(w1 & 0xffffu), k1 = (int64_t)((w1 >> 16) & 0xffffu), k2 = (int64_t)((w1 >> 32) & 0xffffu);
    // ---- the row: loads in flight, min/max and the row parameters before its position is known.
    // The lane index is made opaque here so that the per-lane offsets of every pack width are computed
    // where they are used instead of early (as 64-bit values that overflowed the 128 registers into
    // scratch, each reload followed by a full vmcnt wait inside the store loop).
    int ln = lane;
    asm volatile("" : "+v"(ln));
    int off[NCH];
#pragma unroll
    for (int k = 0; k < NCH; ++k) off[k] = (k * 64 + ln) * 8;
    const S_* src = static_cast<const S_*>(which ? q.kv.v_dev : q.kv.k_dev) + (int64_t)i * q.kv.stride_s;
    Chunk<KDT> raw[NCH];
#pragma unroll
    for (int k = 0; k < NCH; ++k) raw[k] = load_chunk_nt<KDT>(src + off[k]);
    float mn, mx, anz;
    bool row_nan;
    row_minmax<KDT, NCH, true>(raw, nch, ln, mn, mx, anz, row_nan);
    const int bits = pick3(l, a.p.bits[0], a.p.bits[1], a.p.bits[2]);
    const RowParams rp = row_params<KDT>(mn, mx, bits, anz);
    if (q.out.scale_zp_dev && lane < 2) q.out.scale_zp_dev[r * 4 + which * 2 + lane] = lane == 0 ? rp.scale : rp.zp;
    S_* orow = emit_deq ? static_cast<S_*>(which ? q.out.v_out_dev : q.out.k_out_dev) + r * q.out.o_stride_s : nullptr;
    uint8_t* pk = emit_pk ? (which ? q.out.packed_v_dev : q.out.packed_k_dev) + (k0 * rb[0] + k1 * rb[1] + k2 * rb[2])
                          : nullptr;
    emit_row<KDT, NCH, true, true>(raw, rp, row_nan, pick3(l, wid3[0], wid3[1], wid3[2]), orow, off, pk, nch, ln,
                                   emit_deq, emit_pk);
  }
}

template <int ADT, int KDT, int NCH>
__global__ __launch_bounds__(kST) void fused_kernel(FusedArgs x) {
  extern __shared__ uint32_t hist_lds[];  // [kGrp][kNBin] (the selection's rescan path)
  const int G = (int)((x.g.f.S + kST - 1) / kST);
  if ((int)blockIdx.x < G) {
    k2_body<32, true, ADT>(x.g, hist_lds);
    return;
  }
  k4_tasks<ADT, KDT, NCH>(x);
}

template <int ADT, int KDT, int NCH> int launch_fused_inst(const FusedArgs& x, hipStream_t st) {
  const size_t lds = (size_t)kGrp * kNBin * sizeof(uint32_t);
  const void* fn = (const void*)fused_kernel<ADT, KDT, NCH>;
  static bool attr = false;  // per instantiation
  if (!attr) {
    RTKV_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  const int G = (int)((x.g.f.S + kST - 1) / kST);
  const int nq = (int)((2 * x.g.f.S + kST / kWave - 1) / (kST / kWave));  // one wave per (token, tensor)
  hipLaunchKernelGGL((fused_kernel<ADT, KDT, NCH>), dim3(G + nq), dim3(kST), lds, st, x);
  RTKV_HIP_CHECK(hipGetLastError());
  return RTKV_OK;
}

// Host dispatcher for one K/V dtype (explicitly instantiated in fused_{f32,f16,bf16}.hip).
template <int KDT> int launch_fused_kv(const FusedArgs& x, int nch, hipStream_t st) {
  const int adt = x.g.f.a_dtype;
  if (nch == 8 * 64) {
    if (adt == KDT) return launch_fused_inst<KDT, KDT, 8>(x, st);
    if constexpr (KDT != RTKV_F32) if (adt == RTKV_F32) return launch_fused_inst<RTKV_F32, KDT, 8>(x, st);
  }
  if constexpr (KDT != RTKV_F32) {  // fp32 rows of 5120 do not fit the 128 registers of a 1024-thread workgroup
    if (nch == 10 * 64) {
      if (adt == KDT) return launch_fused_inst<KDT, KDT, 10>(x, st);
      if (adt == RTKV_F32) return launch_fused_inst<RTKV_F32, KDT, 10>(x, st);
    }
  }
  RTKV_REQUIRE(false, "fused selection + quantization: unsupported dtype / row width");
}

}  // namespace
}  // namespace rtkv
