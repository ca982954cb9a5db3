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
//   1. wait for the MODE word (sel[6], sel[7]: per group ALL / PART / NONE, the fallback flag and
//      min/max of A), which the selecting workgroup publishes as soon as the class counts give the
//      quotas — before any histogram or threshold work;
//   2. take tasks (token i, tensor K or V) in token order from an atomic counter, recompute the
//      token's score with the very code phase 1 runs (token_score: bit-identical), and skip dropped
//      tokens without reading their row: NONE → dropped, ALL → kept, PART → compare with the group's
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
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)w), hi = __builtin_amdgcn_readfirstlane((uint32_t)(w >> 32));
  return ((uint64_t)hi << 32) | lo;
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
  // ---- the modes and the range of A (published with the quotas)
  const uint64_t m6 = wait_word(&head->sel[6], g.spin_limit, a.stats, broken);
  const uint64_t m7 = wait_word(&head->sel[7], g.spin_limit, a.stats, broken);
  const float amin = __builtin_bit_cast(float, (uint32_t)(m6 >> 16)), amax = __builtin_bit_cast(float, (uint32_t)m7);
  const bool fallback = ((m6 >> 8) & 1u) != 0;
  int mode[kGrp];
#pragma unroll
  for (int k = 0; k < kGrp; ++k) mode[k] = broken ? (int)M_NONE : (int)((m6 >> (2 * k)) & 3u);
  const float den = Dt<ADT>::rnd(amax - amin), eps = Dt<ADT>::rnd(1e-8f);
  uint32_t thr[kGrp] = {0u, 0u, 0u, 0u};
  bool have_thr = false;
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
  auto grab = [&]() -> uint32_t {
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(&head->task, 1u);
    return __builtin_amdgcn_readfirstlane(v);
  };
  uint32_t t = broken ? ntask : grab();
  while (t < ntask) {
    const uint32_t tn = grab();  // the next task, in flight under this one
    const int i = (int)(t >> 1), which = (int)(t & 1u);
    t = tn;
    // ---- keep decision from the modes (and the threshold of a partially kept group)
    const float s = token_score<ADT, true>(a, i, a.A[i], amin, den, eps);
    const int l = class_of(s, a.p);
    const int e = fallback ? 3 : l;
    const int md = pick4(e, mode);
    if (md == M_NONE) continue;
    if (md == M_PART) {
      if (!have_thr) {
#pragma unroll
        for (int k = 0; k < kGrp; ++k) thr[k] = (uint32_t)wait_word(&head->sel[k], g.spin_limit, a.stats, broken);
        have_thr = true;
      }
      if (broken || score_key(s) < pick4(e, thr)) continue;  // below the threshold: dropped, never read
    }
    // ---- the row: loads in flight, min/max and the row parameters before its position is known.
    // The lane index is made opaque per task so that the per-lane offsets of every pack width are
    // recomputed here (a few shifts) instead of being hoisted out of the task loop as 64-bit
    // invariants, which overflowed the 128 registers into scratch reloads (each followed by a full
    // vmcnt wait inside the store loop).
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
    // ---- its output position (phase 3): kept rows of each class before it
    const uint64_t tr = wait_word(&head->tokrow[i], g.spin_limit, a.stats, broken);
    if (!((tr >> 48) & 1u)) continue;  // a tie at the threshold that phase 3 did not take (or broken)
    const int64_t k0 = (int64_t)(tr & 0xffffu), k1 = (int64_t)((tr >> 16) & 0xffffu), k2 = (int64_t)((tr >> 32) & 0xffffu);
    const int64_t r = k0 + k1 + k2;
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
  static int per_cu = 0, cus = 0;  // per instantiation (one device type per process)
  if (!per_cu) {
    RTKV_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int dev = 0;
    RTKV_HIP_CHECK(hipGetDevice(&dev));
    RTKV_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    RTKV_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kST, lds));
    if (per_cu < 1) per_cu = 1;
  }
  const int G = (int)((x.g.f.S + kST - 1) / kST);
  // enough quantization workgroups to fill the rest of the chip once; each drains the task queue
  const int nq = cus * per_cu - G > 16 ? cus * per_cu - G : 16;
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
