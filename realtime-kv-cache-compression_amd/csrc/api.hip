// api.hip — the C ABI of include/rtkv.h: argument validation, workspace carving, host-side scalar
// preparation (the Python-float → fp32 casts the reference performs) and stream-ordered launches.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>

#include <chrono>

#include "common.h"

namespace rtkv {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Workspace layout (256-byte aligned regions):
//   [A: B*S fp32][T2: S fp32][A partials: B*S*2 fp32][labels scratch: B*S u8][stats scratch]
//   [selection pipeline scratch: select_workspace_bytes(B, S)]
struct Workspace {
  float* A;
  float* T2;
  float* Apart;
  uint8_t* labels;
  rtkv_layer_stats* stats;
  void* sel;
};
static size_t ws_bytes(int64_t B, int64_t S) {
  return align_up((size_t)(B * S) * 4, 256) + align_up((size_t)S * 4, 256) + align_up((size_t)(B * S) * 8, 256) +
         align_up((size_t)(B * S), 256) + align_up(rtkv_stats_bytes(B), 256) + align_up(select_workspace_bytes(B, S), 256);
}
static int carve(void* ws, size_t bytes, int64_t B, int64_t S, Workspace& w) {
  if (!ws || bytes < ws_bytes(B, S)) {
    set_error("rtkv: workspace too small (need rtkv_workspace_size(B, S) bytes)");
    return RTKV_ERR_WORKSPACE;
  }
  char* p = static_cast<char*>(ws);
  w.A = reinterpret_cast<float*>(p);
  p += align_up((size_t)(B * S) * 4, 256);
  w.T2 = reinterpret_cast<float*>(p);
  p += align_up((size_t)S * 4, 256);
  w.Apart = reinterpret_cast<float*>(p);
  p += align_up((size_t)(B * S) * 8, 256);
  w.labels = reinterpret_cast<uint8_t*>(p);
  p += align_up((size_t)(B * S), 256);
  w.stats = reinterpret_cast<rtkv_layer_stats*>(p);
  p += align_up(rtkv_stats_bytes(B), 256);
  w.sel = p;
  return RTKV_OK;
}

// The early line is published by one 128-byte wave store and taken as complete when its first and last
// words carry the call's seq: it must not straddle two 128-byte lines (rtkv_host_alloc blocks are
// page-aligned).
static inline bool early_aligned(const void* early) { return ((uintptr_t)early & 127u) == 0; }
static const char* const kEarlyAlignMsg = "early_host must be 128-byte aligned (allocate it with rtkv_host_alloc)";

static int check_params(const rtkv_layer_params* p) {
  RTKV_REQUIRE(p != nullptr, "null params");
  for (int g = 0; g < 3; ++g) RTKV_REQUIRE(p->bits[g] >= 1 && p->bits[g] <= 16, "bits must be in [1, 16]");
  return RTKV_OK;
}

static FinalizeArgs finalize_args(const rtkv_layer_params* p, int64_t B, int64_t S) {
  FinalizeArgs a;
  std::memset(&a, 0, sizeof(a));
  a.p = *p;
  a.B = B;
  a.S = S;
  a.kv_dtype = -1;
  a.a_dtype = RTKV_F32;
  // compute_position_bias divides by math.log(seq_len) (a C double log), cast to fp32 against the
  // fp32 tensor; compute_context_relevance is torch.full((S,), min(1.0, P/S)) in fp32.
  a.logS = (float)std::log((double)S);
  const double rel = (double)p->prompt_len / (double)S;
  a.ctx = (float)(rel < 1.0 ? rel : 1.0);
  return a;
}

}  // namespace rtkv

using namespace rtkv;

extern "C" {

const char* rtkv_version(void) { return "rtkv 0.1.0 (gfx950, HIP)"; }
const char* rtkv_last_error(void) { return g_last_error.c_str(); }
int rtkv_field_width(int dtype, int bits) { return field_width(dtype, bits); }
size_t rtkv_workspace_size(int64_t B, int64_t S) { return ws_bytes(B, S); }

int64_t rtkv_packed_capacity(int64_t B, int64_t S, int64_t F, int dtype, const int32_t bits[3]) {
  int w = 0;
  for (int g = 0; g < 3; ++g) {
    const int fw = field_width(dtype, bits[g]);
    if (fw > w) w = fw;
  }
  return B * S * ((F * w + 7) / 8);
}

int rtkv_attention_aggregation(const rtkv_attn_desc* w, int32_t prompt_len, float* A_dev, void* workspace_dev,
                               size_t workspace_bytes, void* stream) {
  (void)workspace_dev;
  (void)workspace_bytes;
  RTKV_REQUIRE(w != nullptr, "null attention descriptor");
  return launch_aggregation(*w, prompt_len, A_dev, (hipStream_t)stream);
}

int rtkv_minmax_normalize(const void* x_dev, int dtype, int64_t B, int64_t S, void* out_dev, void* stream) {
  return launch_minmax_normalize(x_dev, dtype, B, S, out_dev, (hipStream_t)stream);
}

int rtkv_position_bias(int64_t S, float* pos_dev, void* stream) {
  return launch_position_bias(S, pos_dev, (hipStream_t)stream);
}

int rtkv_importance_scores(const float* A_dev, int a_dtype, int64_t B, int64_t S, const rtkv_layer_params* p,
                           float* scores_dev, void* workspace_dev, size_t workspace_bytes, void* stream) {
  RTKV_REQUIRE(p != nullptr, "null params");
  RTKV_REQUIRE(B >= 1 && S >= 1, "empty shape");
  Workspace ws;
  int rc = carve(workspace_dev, workspace_bytes, B, S, ws);
  if (rc) return rc;
  FinalizeArgs a = finalize_args(p, B, S);
  a.A = A_dev;
  a.a_dtype = a_dtype;
  a.scores = scores_dev;
  a.labels = ws.labels;
  a.stats = ws.stats;
  a.mode_scores = 1;
  a.mode_labels = 1;
  a.mode_select = 0;
  return launch_select(a, ws.sel, false, (hipStream_t)stream);
}

int rtkv_assign_precision(const float* scores_dev, int64_t B, int64_t S, const rtkv_layer_params* p,
                          uint8_t* labels_dev, rtkv_layer_stats* stats_dev, void* workspace_dev,
                          size_t workspace_bytes, void* stream) {
  RTKV_REQUIRE(p != nullptr && labels_dev && stats_dev, "null argument");
  RTKV_REQUIRE(B >= 1 && S >= 1, "empty shape");
  Workspace ws;
  int rc = carve(workspace_dev, workspace_bytes, B, S, ws);
  if (rc) return rc;
  FinalizeArgs a = finalize_args(p, B, S);
  a.scores = const_cast<float*>(scores_dev);
  a.labels = labels_dev;
  a.stats = stats_dev;
  a.mode_scores = 0;
  a.mode_labels = 1;
  a.mode_select = 0;
  return launch_select(a, ws.sel, false, (hipStream_t)stream);
}

int rtkv_select_tokens(const float* scores_dev, const uint8_t* labels_dev, int64_t B, int64_t S,
                       const rtkv_layer_params* p, uint8_t* mask_dev, int32_t* kept_index_dev, int64_t row_capacity,
                       int64_t* row_offset_dev, int64_t F, int kv_dtype, rtkv_layer_stats* stats_dev,
                       void* workspace_dev, size_t workspace_bytes, void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  RTKV_REQUIRE(scores_dev && labels_dev && mask_dev && kept_index_dev && stats_dev, "null argument");
  RTKV_REQUIRE(B >= 1 && S >= 1, "empty shape");
  RTKV_REQUIRE(row_capacity >= S, "row_capacity must be >= S");
  Workspace ws;
  rc = carve(workspace_dev, workspace_bytes, B, S, ws);
  if (rc) return rc;
  FinalizeArgs a = finalize_args(p, B, S);
  a.scores = const_cast<float*>(scores_dev);
  a.labels = const_cast<uint8_t*>(labels_dev);
  a.mask = mask_dev;
  a.kept_index = kept_index_dev;
  a.row_offset = row_offset_dev;
  a.row_capacity = row_capacity;
  a.F = F;
  a.kv_dtype = kv_dtype;
  a.stats = stats_dev;
  a.mode_scores = 0;
  a.mode_labels = 0;
  a.mode_select = (p->flags & RTKV_NO_SELECTION) ? 2 : 1;
  return launch_select(a, ws.sel, false, (hipStream_t)stream);
}

// the rtkv_layer_times trailer of a stats block (include/rtkv.h)
static rtkv_layer_times* layer_times(rtkv_layer_stats* stats, int64_t B) {
  if (!stats) return nullptr;
  return reinterpret_cast<rtkv_layer_times*>(reinterpret_cast<char*>(stats) + rtkv_stats_bytes(B) -
                                             sizeof(rtkv_layer_times));
}

int64_t rtkv_wall_clock_khz(int32_t device) {
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, device) != hipSuccess) return 0;
  return v;
}

static QuantArgs make_quant_args(const rtkv_kv_desc* kv, const uint8_t* labels_dev, const int32_t* kept_index_dev,
                                 const rtkv_layer_params* p, const rtkv_layer_out* out, const uint8_t* row_label) {
  QuantArgs q;
  std::memset(&q, 0, sizeof(q));
  q.kv = *kv;
  q.labels = labels_dev;
  q.kept_index = kept_index_dev;
  q.row_label = row_label;
  q.stats = out->stats_dev;
  for (int g = 0; g < 3; ++g) q.bits[g] = p->bits[g];
  q.out = *out;
  if (!(p->flags & RTKV_EMIT_DEQUANT)) { q.out.k_out_dev = nullptr; q.out.v_out_dev = nullptr; }
  if (!(p->flags & RTKV_EMIT_PACKED)) { q.out.packed_k_dev = nullptr; q.out.packed_v_dev = nullptr; }
  return q;
}

static int quantize_rows_impl(const rtkv_kv_desc* kv, const uint8_t* labels_dev, const int32_t* kept_index_dev,
                              const rtkv_layer_params* p, const rtkv_layer_out* out, void* stream,
                              const uint8_t* row_label) {
  int rc = check_params(p);
  if (rc) return rc;
  RTKV_REQUIRE(kv && out, "null descriptor");
  return launch_quant(make_quant_args(kv, labels_dev, kept_index_dev, p, out, row_label), (hipStream_t)stream);
}

int rtkv_quantize_rows(const rtkv_kv_desc* kv, const uint8_t* labels_dev, const int32_t* kept_index_dev,
                       const rtkv_layer_params* p, const rtkv_layer_out* out, void* stream) {
  return quantize_rows_impl(kv, labels_dev, kept_index_dev, p, out, stream, nullptr);
}

// The fused layer: K1 (W aggregation, or K1' on MFMA when q != null) → K2 → K4.  stop_after_select: the
// first half of rtkv_compress_layer_begin / _finish (K1 and K2 only; the caller sizes the outputs).
static int compress_layer_impl(const rtkv_kv_desc* kv, const rtkv_attn_desc* w, const rtkv_qk_desc* qk,
                               const rtkv_layer_params* p, const rtkv_layer_out* out, void* workspace_dev,
                               size_t workspace_bytes, void* stream, void* const events[4],
                               rtkv_early_stats* early = nullptr, uint64_t early_seq = 0,
                               int32_t* published = nullptr, bool stop_after_select = false) {
  if (published) *published = 0;
  int rc = check_params(p);
  if (rc) return rc;
  RTKV_REQUIRE(kv && (w || qk) && out, "null descriptor");
  RTKV_REQUIRE(early_aligned(early), kEarlyAlignMsg);
  if (w) RTKV_REQUIRE(kv->B == w->B && kv->S == w->S, "K/V and attention weights disagree on B or S");
  if (qk) RTKV_REQUIRE(kv->B == qk->B && kv->S == qk->S, "K/V and queries disagree on B or S");
  RTKV_REQUIRE(out->scores_dev && out->labels_dev && out->mask_dev && out->kept_index_dev && out->stats_dev,
               "compress_layer needs scores, labels, mask, kept_index and stats outputs");
  RTKV_REQUIRE(out->row_capacity >= kv->S, "row_capacity must be >= S (every token may be kept)");
  if (p->flags & RTKV_EMIT_PACKED) {
    RTKV_REQUIRE(out->row_offset_dev && out->scale_zp_dev, "EMIT_PACKED needs row_offset and scale_zp outputs");
    for (int g = 0; g < 3; ++g)
      RTKV_REQUIRE(field_width(kv->dtype, p->bits[g]) > 0, "packed codes unsupported for this dtype/bits");
    if (!stop_after_select) {
      RTKV_REQUIRE(out->packed_k_dev && out->packed_v_dev, "EMIT_PACKED needs packed_k and packed_v outputs");
      RTKV_REQUIRE(out->packed_capacity >= rtkv_packed_capacity(kv->B, out->row_capacity < kv->S ? out->row_capacity : kv->S,
                                                               kv->H * kv->D, kv->dtype, p->bits),
                   "packed_capacity too small");
    }
  }
  if ((p->flags & RTKV_EMIT_DEQUANT) && !stop_after_select)
    RTKV_REQUIRE(out->k_out_dev && out->v_out_dev, "EMIT_DEQUANT needs k_out and v_out");
  Workspace ws;
  rc = carve(workspace_dev, workspace_bytes, kv->B, kv->S, ws);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  auto mark = [&](int k) -> int {
    if (events && events[k]) RTKV_HIP_CHECK(hipEventRecord((hipEvent_t)events[k], st));
    return RTKV_OK;
  };
  if ((rc = mark(0))) return rc;
  FinalizeArgs a = finalize_args(p, kv->B, kv->S);
  AggExtras x;
  int nparts = 0;
  x.t2 = ws.T2;
  x.beta = p->beta;
  x.logS = a.logS;
  x.part = ws.Apart;
  x.nparts = &nparts;
  x.zero0 = ws.sel;  // the selection scratch that must start zeroed (fast path: counter + histograms)
  x.zero0_bytes = (select_fast_shape(kv->B, kv->S) && !(p->flags & RTKV_SELECT_PIPELINE)) ? select_fast_zero_bytes()
                                                                                         : select_zero_bytes(kv->B);
  x.zero1 = out->stats_dev;
  // everything but rtkv_layer_times.begin, which the first block stamps meanwhile (end starts at 0)
  x.zero1_bytes = rtkv_stats_bytes(kv->B) - sizeof(uint64_t);
  x.t_begin = out->stats_dev ? reinterpret_cast<unsigned long long*>(&layer_times(out->stats_dev, kv->B)->begin) : nullptr;
  if (w) {
    rc = launch_aggregation(*w, p->prompt_len, ws.A, st, x);
  } else {
    x.S_total = kv->S;
    x.row0 = 0;
    // the head-major K1' uses the workspace past the base layout when the caller sized it with
    // rtkv_workspace_size_qk
    const size_t base = ws_bytes(kv->B, kv->S);
    float* scratch = workspace_bytes > base ? reinterpret_cast<float*>(static_cast<char*>(workspace_dev) + base) : nullptr;
    rc = launch_qk_importance(*qk, p->prompt_len, ws.A, st, x, &nparts, scratch, scratch ? workspace_bytes - base : 0);
  }
  if (rc) return rc;
  if ((rc = mark(1))) return rc;
  a.A = ws.A;
  a.A_part = ws.Apart;
  a.A_nparts = nparts;
  a.T2 = ws.T2;
  a.a_dtype = w ? w->dtype : RTKV_F32;
  a.scores = out->scores_dev;
  a.labels = out->labels_dev;
  a.mask = out->mask_dev;
  a.kept_index = out->kept_index_dev;
  a.row_offset = out->row_offset_dev;
  a.row_capacity = out->row_capacity;
  a.F = kv->H * kv->D;
  a.kv_dtype = kv->dtype;
  a.stats = out->stats_dev;
  a.mode_scores = 1;
  a.mode_labels = 1;
  a.mode_select = (p->flags & RTKV_NO_SELECTION) ? 2 : 1;
  const bool row_labels = select_fast_eligible(a);  // the fast path also writes each kept row's class
  a.row_label = row_labels ? ws.labels : nullptr;
  if (early && row_labels) {  // the fast path's F1 publishes the final counts to the host
    a.early = early;
    a.early_seq = early_seq;
    if (published) *published = 1;
  }
  if (stop_after_select) {
      rc = launch_select(a, ws.sel, true, st);
    if (rc) return rc;
    return mark(2);
  }
  // (the one-call driver leaves rtkv_layer_times.end at 0: callers that time it use events)
  const QuantArgs q = make_quant_args(kv, out->labels_dev, out->kept_index_dev, p, out, row_labels ? ws.labels : nullptr);
  rc = launch_select(a, ws.sel, true, st);
  if (rc) return rc;
  if ((rc = mark(2))) return rc;
  rc = launch_quant(q, st);
  if (rc) return rc;
  return mark(3);
}

int rtkv_compress_layer_events(const rtkv_kv_desc* kv, const rtkv_attn_desc* w, const rtkv_layer_params* p,
                               const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes, void* stream,
                               void* const events[4]) {
  RTKV_REQUIRE(w != nullptr, "null attention descriptor");
  return compress_layer_impl(kv, w, nullptr, p, out, workspace_dev, workspace_bytes, stream, events);
}

int rtkv_compress_layer(const rtkv_kv_desc* kv, const rtkv_attn_desc* w, const rtkv_layer_params* p,
                        const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes, void* stream) {
  return rtkv_compress_layer_events(kv, w, p, out, workspace_dev, workspace_bytes, stream, nullptr);
}

int rtkv_compress_layer_early(const rtkv_kv_desc* kv, const rtkv_attn_desc* w, const rtkv_layer_params* p,
                              const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes, void* stream,
                              rtkv_early_stats* early_host, uint64_t seq, int32_t* published) {
  RTKV_REQUIRE(w != nullptr && early_host != nullptr, "null attention descriptor or early-stats buffer");
  return compress_layer_impl(kv, w, nullptr, p, out, workspace_dev, workspace_bytes, stream, nullptr, early_host,
                             seq, published);
}

int rtkv_compress_layer_qk_early(const rtkv_kv_desc* kv, const rtkv_qk_desc* q, const rtkv_layer_params* p,
                                 const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes, void* stream,
                                 rtkv_early_stats* early_host, uint64_t seq, int32_t* published) {
  RTKV_REQUIRE(q != nullptr && early_host != nullptr, "null query descriptor or early-stats buffer");
  return compress_layer_impl(kv, nullptr, q, p, out, workspace_dev, workspace_bytes, stream, nullptr, early_host,
                             seq, published);
}

int rtkv_compress_layer_begin(const rtkv_kv_desc* kv, const rtkv_attn_desc* w, const rtkv_layer_params* p,
                              const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes, void* stream,
                              rtkv_early_stats* early_host, uint64_t seq, int32_t* published, void* start_event) {
  RTKV_REQUIRE(w != nullptr, "null attention descriptor");
  void* const ev[4] = {start_event, nullptr, nullptr, nullptr};
  return compress_layer_impl(kv, w, nullptr, p, out, workspace_dev, workspace_bytes, stream, start_event ? ev : nullptr,
                             early_host, seq, published, true);
}

int rtkv_compress_layer_qk_begin(const rtkv_kv_desc* kv, const rtkv_qk_desc* q, const rtkv_layer_params* p,
                                 const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes, void* stream,
                                 rtkv_early_stats* early_host, uint64_t seq, int32_t* published, void* start_event) {
  RTKV_REQUIRE(q != nullptr, "null query descriptor");
  void* const ev[4] = {start_event, nullptr, nullptr, nullptr};
  return compress_layer_impl(kv, nullptr, q, p, out, workspace_dev, workspace_bytes, stream, start_event ? ev : nullptr,
                             early_host, seq, published, true);
}

int rtkv_compress_layer_finish(const rtkv_kv_desc* kv, const rtkv_layer_params* p, const rtkv_layer_out* out,
                               int64_t out_rows, void* workspace_dev, size_t workspace_bytes, void* stream,
                               rtkv_early_stats* early_host, uint64_t seq) {
  int rc = check_params(p);
  if (rc) return rc;
  RTKV_REQUIRE(kv && out && out->labels_dev && out->kept_index_dev && out->stats_dev,
               "compress_layer_finish needs the labels, kept_index and stats of rtkv_compress_layer_begin");
  RTKV_REQUIRE(out->row_capacity >= kv->S, "row_capacity must be the capacity rtkv_compress_layer_begin used (>= S)");
  RTKV_REQUIRE(early_aligned(early_host), kEarlyAlignMsg);
  if (p->flags & RTKV_EMIT_PACKED)
    RTKV_REQUIRE(out->packed_k_dev && out->packed_v_dev && out->row_offset_dev && out->scale_zp_dev &&
                     out->packed_capacity >= 1,
                 "EMIT_PACKED needs packed_k, packed_v (>= the published packed bytes), row_offset and scale_zp");
  if (p->flags & RTKV_EMIT_DEQUANT)
    RTKV_REQUIRE(out->k_out_dev && out->v_out_dev && out->o_stride_b < 0 && out_rows >= 1,
                 "EMIT_DEQUANT needs k_out / v_out of [B, out_rows >= 1, F] rows packed at the kept count "
                 "(o_stride_b = -1)");
  Workspace ws;
  rc = carve(workspace_dev, workspace_bytes, kv->B, kv->S, ws);
  if (rc) return rc;
  // the one-launch K2 (B = 1, S <= 65536) left each kept row's class in the workspace
  const bool row_labels = select_fast_shape(kv->B, kv->S) && !(p->flags & RTKV_SELECT_PIPELINE);
  QuantArgs q = make_quant_args(kv, out->labels_dev, out->kept_index_dev, p, out, row_labels ? ws.labels : nullptr);
  // the buffers were sized on the host from the published statistics: K4 checks them on the device
  q.out_rows = (p->flags & RTKV_EMIT_DEQUANT) ? out_rows : ((int64_t)1 << 62);
  if (!(p->flags & RTKV_EMIT_PACKED)) q.out.packed_capacity = (int64_t)1 << 62;
  q.exact_sizes = (p->flags & RTKV_FINISH_EXACT) ? 1 : 0;
  q.final_host = early_host;
  q.final_seq = seq;
  q.t_end = reinterpret_cast<unsigned long long*>(layer_times(out->stats_dev, kv->B)->end);
  return launch_quant(q, (hipStream_t)stream);
}

int rtkv_prefetch_kept_rows(const rtkv_kv_desc* kv, const rtkv_layer_out* out, int64_t max_bytes, void* stream) {
  RTKV_REQUIRE(out != nullptr, "null output descriptor");
  return launch_prefetch_rows(kv, out->kept_index_dev, out->stats_dev, max_bytes, (hipStream_t)stream);
}

int rtkv_wait_early(const rtkv_early_stats* early_host, uint64_t seq, int64_t timeout_us) {
  RTKV_REQUIRE(early_host != nullptr, "null early-stats buffer");
  RTKV_REQUIRE(early_aligned(early_host), kEarlyAlignMsg);
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t it = 0;; ++it) {
    if (__atomic_load_n(&early_host->seq, __ATOMIC_ACQUIRE) == seq &&
        __atomic_load_n(&early_host->seq_tail, __ATOMIC_ACQUIRE) == seq)
      return RTKV_OK;
    if ((it & 255u) == 255u &&
        std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count() >
            timeout_us) {
      set_error("rtkv: wait_early: the device did not publish the layer statistics in time");
      return RTKV_ERR_TIMEOUT;
    }
    __builtin_ia32_pause();
  }
}

int rtkv_wait_final(const rtkv_early_stats* early_host, uint64_t seq, int64_t timeout_us) {
  RTKV_REQUIRE(early_host != nullptr, "null early-stats buffer");
  RTKV_REQUIRE(early_aligned(early_host), kEarlyAlignMsg);
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t it = 0;; ++it) {
    if ((__atomic_load_n(&early_host->final_word, __ATOMIC_ACQUIRE) >> 16) == (seq & ((1ull << 48) - 1)))
      return RTKV_OK;
    if ((it & 255u) == 255u &&
        std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count() >
            timeout_us) {
      set_error("rtkv: wait_final: the layer's K4 did not publish its final flags in time");
      return RTKV_ERR_TIMEOUT;
    }
    __builtin_ia32_pause();
  }
}

void* rtkv_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return nullptr;
  std::memset(p, 0, bytes);
  return p;
}

void rtkv_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

int rtkv_compress_layer_qk_events(const rtkv_kv_desc* kv, const rtkv_qk_desc* q, const rtkv_layer_params* p,
                                  const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes, void* stream,
                                  void* const events[4]) {
  RTKV_REQUIRE(q != nullptr, "null query descriptor");
  return compress_layer_impl(kv, nullptr, q, p, out, workspace_dev, workspace_bytes, stream, events);
}

int rtkv_compress_layer_qk(const rtkv_kv_desc* kv, const rtkv_qk_desc* q, const rtkv_layer_params* p,
                           const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes, void* stream) {
  return rtkv_compress_layer_qk_events(kv, q, p, out, workspace_dev, workspace_bytes, stream, nullptr);
}

int rtkv_importance_qk_lse(const rtkv_qk_desc* q, int32_t prompt_len, float* A_dev, void* stream) {
  RTKV_REQUIRE(q != nullptr, "null query descriptor");
  AggExtras x;
  return launch_qk_importance(*q, prompt_len, A_dev, (hipStream_t)stream, x, nullptr);
}

size_t rtkv_qk_scratch_size(int64_t B, int64_t H, int64_t S) { return qk_scratch_bytes(B, H, S); }

size_t rtkv_workspace_size_qk(int64_t B, int64_t H, int64_t S) {
  return ws_bytes(B, S) + align_up(qk_scratch_bytes(B, H, S), 256);
}

int rtkv_importance_qk_lse_ws(const rtkv_qk_desc* q, int32_t prompt_len, float* A_dev, void* scratch_dev,
                              size_t scratch_bytes, void* stream) {
  RTKV_REQUIRE(q != nullptr, "null query descriptor");
  AggExtras x;
  x.S_total = q->row0 + q->S;  // only the β·pos epilogue would read it (t2 is null here)
  x.row0 = q->row0;
  return launch_qk_importance(*q, prompt_len, A_dev, (hipStream_t)stream, x, nullptr,
                              static_cast<float*>(scratch_dev), scratch_bytes);
}

int rtkv_attention_lse(const rtkv_qk_desc* q, float* lse_dev, void* stream) {
  RTKV_REQUIRE(q != nullptr, "null query descriptor");
  return launch_attention_lse(*q, lse_dev, (hipStream_t)stream);
}

// ---------------------------------------------------------------------------------- sequence shards
int rtkv_attention_aggregation_shard(const rtkv_attn_desc* w, int32_t prompt_len, int64_t row0, int64_t S_total,
                                     float* A_dev, void* stream) {
  RTKV_REQUIRE(w != nullptr, "null attention descriptor");
  RTKV_REQUIRE(row0 >= 0 && S_total >= row0 + w->S, "shard rows [row0, row0 + S) must lie inside [0, S_total)");
  AggExtras x;
  x.row0 = row0;
  x.S_total = S_total;
  return launch_aggregation(*w, prompt_len, A_dev, (hipStream_t)stream, x);
}

// the selection scratch a finalize call needs zeroed: the one-launch K2's, or the pipeline's
static size_t finalize_zero_bytes(int64_t B, int64_t S, const rtkv_layer_params* p) {
  return (select_fast_shape(B, S) && !(p->flags & RTKV_SELECT_PIPELINE)) ? select_fast_zero_bytes() : select_zero_bytes(B);
}

int rtkv_attention_aggregation_shard_ws(const rtkv_attn_desc* w, int32_t prompt_len, int64_t row0, int64_t S_total,
                                        float* A_dev, const rtkv_layer_params* p, const rtkv_layer_out* out,
                                        void* workspace_dev, size_t workspace_bytes, void* stream) {
  RTKV_REQUIRE(w != nullptr && p != nullptr && out != nullptr && out->stats_dev, "null descriptor, params or stats");
  RTKV_REQUIRE(row0 >= 0 && S_total >= row0 + w->S, "shard rows [row0, row0 + S) must lie inside [0, S_total)");
  Workspace ws;
  int rc = carve(workspace_dev, workspace_bytes, w->B, S_total, ws);
  if (rc) return rc;
  AggExtras x;
  x.row0 = row0;
  x.S_total = S_total;
  x.zero0 = ws.sel;  // what rtkv_finalize_select_shard(..., scratch_zeroed = 1) would otherwise memset
  x.zero0_bytes = finalize_zero_bytes(w->B, S_total, p);
  x.zero1 = out->stats_dev;
  x.zero1_bytes = rtkv_stats_bytes(w->B);
  return launch_aggregation(*w, prompt_len, A_dev, (hipStream_t)stream, x);
}

int rtkv_finalize_select_shard(const float* A_dev, int a_dtype, int64_t B, int64_t S, const rtkv_layer_params* p,
                               const rtkv_layer_out* out, int64_t F, int kv_dtype, int64_t S_local, int32_t nranks,
                               int64_t* ranges_dev, int32_t scratch_zeroed, void* workspace_dev, size_t workspace_bytes,
                               void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  RTKV_REQUIRE(A_dev && out && ranges_dev, "null argument");
  RTKV_REQUIRE(B >= 1 && S >= 1 && F >= 1, "empty shape");
  RTKV_REQUIRE(nranks >= 1 && S_local >= 1 && S_local * nranks == S, "S must be nranks * S_local");
  RTKV_REQUIRE(out->scores_dev && out->labels_dev && out->mask_dev && out->kept_index_dev && out->stats_dev,
               "finalize_select needs scores, labels, mask, kept_index and stats outputs");
  RTKV_REQUIRE(out->row_capacity >= S, "row_capacity must be >= S (every token may be kept)");
  if (p->flags & RTKV_EMIT_PACKED) {
    RTKV_REQUIRE(out->row_offset_dev, "EMIT_PACKED needs row offsets");
    for (int g = 0; g < 3; ++g)
      RTKV_REQUIRE(field_width(kv_dtype, p->bits[g]) > 0, "packed codes unsupported for this dtype/bits");
  }
  Workspace ws;
  rc = carve(workspace_dev, workspace_bytes, B, S, ws);
  if (rc) return rc;
  FinalizeArgs a = finalize_args(p, B, S);
  a.A = A_dev;
  a.a_dtype = a_dtype;
  a.scores = out->scores_dev;
  a.labels = out->labels_dev;
  a.mask = out->mask_dev;
  a.kept_index = out->kept_index_dev;
  a.row_offset = out->row_offset_dev;
  a.row_capacity = out->row_capacity;
  a.F = F;
  a.kv_dtype = kv_dtype;
  a.stats = out->stats_dev;
  a.mode_scores = 1;
  a.mode_labels = 1;
  a.mode_select = (p->flags & RTKV_NO_SELECTION) ? 2 : 1;
  const bool fused = select_fast_eligible(a);
  if (fused) {  // the one-launch K2's compaction writes the rank table (no rtkv_shard_ranges launch)
    a.shard_ranges = ranges_dev;
    a.shard_S_local = S_local;
    a.shard_nranks = nranks;
  }
  rc = launch_select(a, ws.sel, scratch_zeroed != 0, (hipStream_t)stream);
  if (rc || fused) return rc;
  return launch_shard_ranges(out->kept_index_dev, out->row_offset_dev, out->stats_dev, B, out->row_capacity, S_local,
                             nranks, ranges_dev, (hipStream_t)stream);
}

int rtkv_finalize_select(const float* A_dev, int a_dtype, int64_t B, int64_t S, const rtkv_layer_params* p,
                         const rtkv_layer_out* out, int64_t F, int kv_dtype, void* workspace_dev,
                         size_t workspace_bytes, void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  RTKV_REQUIRE(A_dev && out, "null argument");
  RTKV_REQUIRE(B >= 1 && S >= 1 && F >= 1, "empty shape");
  RTKV_REQUIRE(out->scores_dev && out->labels_dev && out->mask_dev && out->kept_index_dev && out->stats_dev,
               "finalize_select needs scores, labels, mask, kept_index and stats outputs");
  RTKV_REQUIRE(out->row_capacity >= S, "row_capacity must be >= S (every token may be kept)");
  if (p->flags & RTKV_EMIT_PACKED) {
    RTKV_REQUIRE(out->row_offset_dev, "EMIT_PACKED needs row offsets");
    for (int g = 0; g < 3; ++g)
      RTKV_REQUIRE(field_width(kv_dtype, p->bits[g]) > 0, "packed codes unsupported for this dtype/bits");
  }
  Workspace ws;
  rc = carve(workspace_dev, workspace_bytes, B, S, ws);
  if (rc) return rc;
  FinalizeArgs a = finalize_args(p, B, S);
  a.A = A_dev;
  a.a_dtype = a_dtype;
  a.scores = out->scores_dev;
  a.labels = out->labels_dev;
  a.mask = out->mask_dev;
  a.kept_index = out->kept_index_dev;
  a.row_offset = out->row_offset_dev;
  a.row_capacity = out->row_capacity;
  a.F = F;
  a.kv_dtype = kv_dtype;
  a.stats = out->stats_dev;
  a.mode_scores = 1;
  a.mode_labels = 1;
  a.mode_select = (p->flags & RTKV_NO_SELECTION) ? 2 : 1;
  return launch_select(a, ws.sel, false, (hipStream_t)stream);
}

int rtkv_quantize_rows_shard(const rtkv_kv_desc* kv, int64_t row0, int64_t S_total, int32_t rank, int32_t nranks,
                             const int64_t* ranges_dev, const uint8_t* labels_dev, const int32_t* kept_index_dev,
                             const rtkv_layer_params* p, const rtkv_layer_out* out, void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  RTKV_REQUIRE(kv && out && kept_index_dev && out->stats_dev, "quantize_rows_shard needs kept_index and stats");
  RTKV_REQUIRE(row0 >= 0 && S_total >= row0 + kv->S, "shard rows [row0, row0 + S) must lie inside [0, S_total)");
  RTKV_REQUIRE(out->row_capacity >= S_total, "row_capacity must be >= S_total");
  QuantArgs q;
  std::memset(&q, 0, sizeof(q));
  q.kv = *kv;
  q.labels = labels_dev;
  q.kept_index = kept_index_dev;
  q.stats = out->stats_dev;
  for (int g = 0; g < 3; ++g) q.bits[g] = p->bits[g];
  q.out = *out;
  RTKV_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "rank must be in [0, nranks)");
  RTKV_REQUIRE(!ranges_dev || !(p->flags & RTKV_EMIT_DEQUANT) || out->o_stride_b >= 0,
               "local dequant rows (ranges_dev) need an explicit o_stride_b");
  q.S_glob = S_total;
  q.row0 = row0;
  q.pad_owner = (rank == 0 && !ranges_dev) ? 1 : 0;
  q.shard_rank = rank;
  q.shard_nranks = nranks;
  q.shard_ranges = ranges_dev;
  if (!(p->flags & RTKV_EMIT_DEQUANT)) { q.out.k_out_dev = nullptr; q.out.v_out_dev = nullptr; }
  if (!(p->flags & RTKV_EMIT_PACKED)) { q.out.packed_k_dev = nullptr; q.out.packed_v_dev = nullptr; }
  return launch_quant(q, (hipStream_t)stream);
}

int rtkv_shard_ranges(const int32_t* kept_index_dev, const int64_t* row_offset_dev, const rtkv_layer_stats* stats_dev,
                      int64_t B, int64_t row_capacity, int64_t S_local, int32_t nranks, int64_t* ranges_dev,
                      void* stream) {
  return launch_shard_ranges(kept_index_dev, row_offset_dev, stats_dev, B, row_capacity, S_local, nranks, ranges_dev,
                             (hipStream_t)stream);
}

int rtkv_unpack_dequant(const uint8_t* packed_dev, const int64_t* row_offset_dev, const float* scale_zp_dev,
                        int which, const int32_t* kept_index_dev, const uint8_t* labels_dev, int64_t B, int64_t S,
                        int64_t row_capacity, const int64_t* rows_dev, int64_t H, int64_t D, int dtype,
                        const int32_t bits[3], void* out_dev, int64_t o_stride_b, int64_t o_stride_s,
                        int64_t o_stride_h, void* stream) {
  RTKV_REQUIRE(bits != nullptr, "null bits");
  return launch_unpack(packed_dev, row_offset_dev, scale_zp_dev, which, kept_index_dev, labels_dev, B, S, row_capacity,
                       rows_dev, H, D, dtype, bits, out_dev, o_stride_b, o_stride_s, o_stride_h, (hipStream_t)stream);
}

size_t rtkv_decode_workspace_size(int64_t B, int64_t Hq, int64_t Hkv, int64_t D, int64_t row_capacity) {
  if (B < 1 || Hkv < 1 || Hq < Hkv || D < 1 || row_capacity < 1) return 0;
  return decode_workspace_bytes(B, Hq, Hkv, D, row_capacity);
}

int rtkv_decode_attention_packed(const uint8_t* packed_k_dev, const uint8_t* packed_v_dev, int64_t packed_bytes,
                                 const int64_t* row_offset_dev,
                                 const float* scale_zp_dev, const int32_t* kept_index_dev, const uint8_t* labels_dev,
                                 int64_t B, int64_t S, int64_t row_capacity, const int64_t* rows_dev, int64_t Hkv,
                                 int64_t D, int dtype, const int32_t bits[3], const void* q_dev, int64_t Hq,
                                 float scale, float* out_dev, void* workspace_dev, size_t workspace_bytes,
                                 void* stream) {
  RTKV_REQUIRE(bits != nullptr, "null bits");
  return launch_decode(packed_k_dev, packed_v_dev, packed_bytes, row_offset_dev, scale_zp_dev, kept_index_dev, labels_dev, B, S,
                       row_capacity, rows_dev, Hkv, D, dtype, bits, q_dev, Hq, scale, out_dev, workspace_dev,
                       workspace_bytes, (hipStream_t)stream);
}

int rtkv_gather_rows(const void* src_dev, int64_t B, int64_t S, int64_t row_bytes, const int32_t* kept_index_dev,
                     int64_t row_capacity, int64_t src_stride_b, void* dst_dev, int64_t dst_stride_b, int64_t src_stride_s,
                     const rtkv_layer_stats* stats_dev, void* stream) {
  return launch_gather(src_dev, B, S, row_bytes, kept_index_dev, row_capacity, src_stride_b, dst_dev, dst_stride_b,
                       src_stride_s, stats_dev, (hipStream_t)stream);
}

int rtkv_tensor_quant_params(const void* x_dev, int dtype, int64_t n_rows, int64_t row_len, const uint8_t* row_labels_dev,
                             int32_t label_value, int bits, float* scale_zp_dev, void* workspace_dev,
                             size_t workspace_bytes, void* stream) {
  return launch_tensor_params(x_dev, dtype, n_rows, row_len, row_labels_dev, label_value, bits, scale_zp_dev,
                              workspace_dev, workspace_bytes, (hipStream_t)stream);
}

int rtkv_tensor_fake_quant(const void* x_dev, int dtype, int64_t n_rows, int64_t row_len, const uint8_t* row_labels_dev,
                           int32_t label_value, int bits, const float* scale_zp_dev, void* out_dev, void* stream) {
  return launch_tensor_fake_quant(x_dev, dtype, n_rows, row_len, row_labels_dev, label_value, bits, scale_zp_dev,
                                  out_dev, (hipStream_t)stream);
}

int rtkv_selfcheck_division(int32_t dtype, unsigned long long* counts_dev, void* stream) {
  return launch_selfcheck_division(dtype, counts_dev, (hipStream_t)stream);
}

int rtkv_selfcheck_division_f32(int64_t s_lo, int64_t s_hi, int32_t ex, int32_t es, int32_t negative,
                                unsigned long long* counts_dev, void* stream) {
  return launch_selfcheck_division_f32(s_lo, s_hi, ex, es, negative, counts_dev, (hipStream_t)stream);
}

}  // extern "C"
