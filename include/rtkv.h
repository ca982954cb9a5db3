/*
 * rtkv.h — C ABI of the MI355X (gfx950) streaming prefill KV-cache compression path.
 *
 * This library replaces the PyTorch eager hot path of the reference
 * (EvelynHung-79/RealTime-KV-cache-Compression):
 *
 *   RealTimePrefillCompressor.compress_layer_kv_cache      src/compression/unified_compressor.py:95-172
 *     ├─ PromptGuidedImportanceScorer.*                    src/compression/token_importance.py:21-176
 *     ├─ DynamicPrecisionQuantizer.*                       src/compression/dynamic_quantization.py:21-196
 *     └─ SelectiveTokenPropagator.*                        src/compression/selective_propagation.py:68-244
 *
 * Conventions
 *   - Every pointer argument named *_dev is a device pointer (hipMalloc / torch CUDA tensor).
 *   - All work is stream-ordered on `stream` (a hipStream_t passed as void*; NULL = default stream).
 *     No entry point allocates, frees or synchronises; scratch comes from a caller-owned workspace
 *     sized by rtkv_workspace_size().  Inputs are never mutated.
 *   - Return value: 0 on success, a negative RTKV_ERR_* code otherwise; rtkv_last_error() returns a
 *     human-readable message for the calling thread.  Errors that depend on device data (e.g. the
 *     fp16 16-bit overflow) are reported through rtkv_layer_stats.error_flags after the stream syncs.
 *   - dtype codes: RTKV_F32 / RTKV_F16 / RTKV_BF16.  Arithmetic follows the reference's PyTorch CPU
 *     semantics: every elementwise op is computed in fp32 and rounded to the tensor dtype
 *     (round-to-nearest-even), division is IEEE, no FMA contraction.
 *   - Token precision classes ("labels") are 0 = LOW, 1 = MEDIUM, 2 = HIGH
 *     (dynamic_quantization.py:41-45), stored as uint8.
 */
#ifndef RTKV_H
#define RTKV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTKV_ABI_VERSION 1

enum rtkv_dtype { RTKV_F32 = 0, RTKV_F16 = 1, RTKV_BF16 = 2 };

enum rtkv_status {
  RTKV_OK = 0,
  RTKV_ERR_INVALID = -1,     /* bad shape / stride / parameter */
  RTKV_ERR_UNSUPPORTED = -2, /* configuration outside the implemented envelope */
  RTKV_ERR_HIP = -3,         /* a HIP runtime call failed */
  RTKV_ERR_WORKSPACE = -4,   /* workspace too small */
  RTKV_ERR_TIMEOUT = -5      /* rtkv_wait_early: the device did not publish in time */
};

/* rtkv_layer_stats.error_flags bits (device-detected, read after the stream syncs) */
enum rtkv_error_flag {
  /* A populated class uses a bit width whose qmax = 2^b-1 overflows fp16 (b >= 16).  The reference
   * raises "value cannot be converted to type c10::Half without overflow" at
   * dynamic_quantization.py:121 in that case; the host wrapper raises the same RuntimeError. */
  RTKV_FLAG_F16_QMAX_OVERFLOW = 1,
  /* A cross-workgroup hand-off of the one-launch selection did not arrive within its poll bound
   * (a workgroup that never became resident, or a withheld hand-off in the test below): the waiting
   * workgroups gave up, so the layer's outputs are invalid.  The host wrapper raises
   * RTKV_ERR_TIMEOUT. */
  RTKV_FLAG_SPIN_TIMEOUT = 2,
  /* rtkv_compress_layer_finish: the layer's S'_max or packed byte count exceeds the buffers the caller
   * declared (out_rows, packed_capacity); K4 wrote nothing. */
  RTKV_FLAG_OUTPUT_OVERFLOW = 4
};

/* Flags for rtkv_layer_params.flags */
enum rtkv_layer_flag {
  RTKV_EMIT_DEQUANT = 1,   /* write the dequantized K'/V' (the reference's return value) */
  RTKV_EMIT_PACKED = 2,    /* write bit-packed integer codes + per-row scale/zero-point */
  RTKV_NO_SELECTION = 4,   /* keep every token (quantization only, BASELINE config 2) */
  RTKV_NO_FALLBACK = 8,    /* skip the top-10% emergency fallback (select_tokens_with_budget alone) */
  RTKV_SELECT_PIPELINE = 16, /* use the multi-workgroup selection pipeline even where the one-workgroup
                              selection applies (B = 1, S <= 65536); same results, for cross-checks */
  RTKV_FINISH_EXACT = 32,  /* rtkv_compress_layer_finish: the caller sized its buffers EXACTLY from the published
                              statistics — out_rows = max(S'_max, 1), packed_capacity = max(packed bytes, 1)
                              rounded up to 256 — and any other size (a torn or stale read of the early line)
                              raises RTKV_FLAG_OUTPUT_OVERFLOW (nothing written) instead of returning rows the
                              device never wrote.  The drop-in sets it. */
  RTKV_TEST_WITHHOLD_SELECTION = 1 << 16, /* test only: the one-launch selection never publishes its
                              thresholds, so every waiting workgroup runs into its poll bound and the
                              layer reports RTKV_FLAG_SPIN_TIMEOUT instead of hanging */
  RTKV_TEST_WITHHOLD_LOOKBACK = 1 << 17 /* test only: the one-launch selection publishes its early
                              statistics, then workgroup 0 never publishes its kept counts, so the other
                              workgroups' look-back runs into its poll bound AFTER the early publication */
};

/* ------------------------------------------------------------------------------------------------
 * Parameter block.  Field-by-field mirror of configs/base_config.py:4-56 as consumed on the path.
 * The host fills the float fields with the float32 rounding of the config's Python floats, exactly
 * as PyTorch casts a Python scalar against an fp32 tensor.
 * ---------------------------------------------------------------------------------------------- */
typedef struct rtkv_layer_params {
  float alpha;             /* token_importance.py:163  (config.alpha) */
  float beta;              /* token_importance.py:167  (config.beta) */
  float gamma;             /* token_importance.py:171  (config.gamma) */
  float layer_weight;      /* token_importance.py:162  (config.layer_weights[layer_idx]) */
  float theta_h;           /* dynamic_quantization.py:41 */
  float theta_m;           /* dynamic_quantization.py:42 */
  int32_t bits[3];         /* bits by class {LOW, MEDIUM, HIGH}: dynamic_quantization.py:169-174 */
  int32_t prompt_len;      /* P = max(1, min(S // 5, 128)): unified_compressor.py:55 */
  double propagation_ratio;/* selective_propagation.py:23-38 for this layer */
  int32_t flags;           /* RTKV_EMIT_* | RTKV_NO_SELECTION */
  int32_t reserved;
} rtkv_layer_params;

/* Attention input.  W[b, h, i, c] at w + b*stride_b + h*stride_h + i*stride_s + c (elements);
 * only columns c < prompt_len are read (token_importance.py:41 reads W[..., prompt_indices] with
 * prompt_indices = arange(P)).  Either the reference's full [B,H,S,S] matrix or a [B,H,S,P] prompt
 * slice can be passed: both give bit-identical results. */
typedef struct rtkv_attn_desc {
  const void* w_dev;
  int32_t dtype;
  int32_t reserved;
  int64_t B, H, S, cols;               /* cols >= prompt_len */
  int64_t stride_b, stride_h, stride_s;
} rtkv_attn_desc;

/* Key/value states.  x[b, i, h, d] at base + b*stride_b + i*stride_s + h*stride_h + d.
 * The reference layout [B, S, Hkv*D] (modified_llama.py:105-108) is stride_s = Hkv*D, stride_h = D;
 * the model's native [B, Hkv, S, D] layout is stride_h = S*D, stride_s = D (no transpose copy). */
typedef struct rtkv_kv_desc {
  const void* k_dev;
  const void* v_dev;
  int32_t dtype;
  int32_t reserved;
  int64_t B, S, H, D;
  int64_t stride_b, stride_s, stride_h;
} rtkv_kv_desc;

/* Fused importance input (no attention matrix): queries, the P prompt keys and the row log-sum-exp
 * of the model's softmax.  W[b,h,i,p] = exp(q[b,h,i]·k[b,h/(H/Hkv),p]·scale − lse[b,h,i]) for p < P
 * (and p <= row0 + i when causal), which is the reference's
 * softmax(Q·Kᵀ/√d + mask) (modified_llama.py:88-94) restricted to the prompt columns.
 * q[b,h,i,d] at q_dev + b*q_stride_b + h*q_stride_h + i*q_stride_s + d; k likewise with p for i;
 * lse[b,h,i] at lse_dev + b*lse_stride_b + h*lse_stride_h + i (fp32). */
typedef struct rtkv_qk_desc {
  const void* q_dev;
  const void* k_dev;
  const float* lse_dev;
  int32_t dtype;                       /* RTKV_F16, RTKV_BF16 (bf16/f16 MFMA) or RTKV_F32 (three-way bf16 split; exact f32 MFMA with RTKV_LSE_F32_EXACT) */
  int32_t causal;
  int64_t B, H, Hkv, S, D;
  int64_t q_stride_b, q_stride_h, q_stride_s;
  int64_t k_stride_b, k_stride_h, k_stride_s;
  int64_t lse_stride_b, lse_stride_h;
  float scale;                         /* 1/sqrt(head_dim) in the reference (modified_llama.py:89) */
  int32_t reserved;
  int64_t row0;                        /* global position of query row 0 (sequence shards), else 0 */
  /* Optional additive key bias kbias[b, j] (fp32, at kbias_dev + b*kbias_stride_b + j; null: none): the
   * key-padding part of the model's attention_mask (modified_llama.py:90-91), 0 for a real key and
   * -inf (or any value below -1e30, e.g. the mask's finfo.min) for a padding key.  A query row that
   * sees no key at all (a padding row) gets lse = -inf, and its softmax is the uniform 1/S the
   * reference's all-masked row has (every logit equal).  Supported by rtkv_attention_lse and the
   * fused-mode K1' with head_dim 128. */
  const float* kbias_dev;
  int64_t kbias_stride_b;
} rtkv_qk_desc;

/* Per-batch-row statistics (device-resident; one entry per batch row after the header). */
typedef struct rtkv_batch_stats {
  int64_t class_count[3];    /* tokens per class, dynamic_quantization.py:50-57 */
  int64_t kept;              /* selected tokens S'_b */
  int64_t kept_class[3];     /* selected tokens per class (selective_propagation.py:126-133) */
  int64_t cost_units;        /* Σ bits of the selected tokens = 8 * current_cost (:122-131) */
  int64_t packed_bytes;      /* bytes of packed codes per tensor for this row */
  int32_t fallback;          /* 1 if the top-10% emergency fallback ran (:205-211) */
  int32_t reserved;
  double kept_score_sum;     /* Σ scores of selected tokens (avg_importance, :139) */
} rtkv_batch_stats;

typedef struct rtkv_layer_stats {
  int64_t max_kept;          /* S'_max = max_b S'_b: rows of the padded output (:183) */
  int64_t total_packed_bytes;/* bytes used in each packed code buffer */
  double score_sum;          /* Σ scores over B*S   (unified_compressor.py:159) */
  double score_m2;           /* Σ (s - mean)^2      (unified_compressor.py:160, unbiased std) */
  float score_min;           /* unified_compressor.py:161 */
  float score_max;           /* unified_compressor.py:162 */
  int32_t error_flags;       /* RTKV_FLAG_* */
  int32_t B;
  /* followed by B x rtkv_batch_stats */
} rtkv_layer_stats;

/* After the B batch stats: the layer's device time span, read from the GPU's 100 MHz real-time counter
 * (s_memrealtime; rtkv_wall_clock_khz gives its rate).  begin: when the first block of the layer's
 * first kernel (K1 / K1') started; end: when the quantization kernel (K4) wrote its last row — the
 * largest of end[16·k], k < RTKV_TIME_SLOTS (every K4 wave that wrote a row takes an atomic max on slot
 * (its wave index mod RTKV_TIME_SLOTS), one 128-byte line per slot: on one address the atomics
 * serialised and doubled K4).  begin is written by every fused call (rtkv_compress_layer*, _begin), end
 * by rtkv_compress_layer_finish only (all slots 0 otherwise, or when K4 did not run).  The drop-in's
 * processing_time comes from here, with no event on the stream (a timing event right before K1 cost
 * ~4.6 us of device idle per layer). */
#define RTKV_TIME_SLOTS 32
typedef struct rtkv_layer_times {
  uint64_t end[16 * RTKV_TIME_SLOTS];
  uint64_t begin;
} rtkv_layer_times;

static inline size_t rtkv_stats_bytes(int64_t B) {
  return sizeof(rtkv_layer_stats) + (size_t)B * sizeof(rtkv_batch_stats) + sizeof(rtkv_layer_times);
}

/* Rate of the device's real-time counter (rtkv_layer_times), kHz. */
int64_t rtkv_wall_clock_khz(int32_t device);

/* Outputs of one layer.  Any pointer may be NULL to skip that output (scores/labels/mask/kept_index
 * /stats are always needed by the fused driver and must be non-NULL there).
 *
 * Output rows are the selected tokens in ascending original index (selective_propagation.py:224-232),
 * zero-padded per batch row up to S'_max (:214-222).
 *
 * Packed codes: for output row r of batch row b with class c, bits w = rtkv_field_width(dtype,
 * bits[c]) per element; the row's F = H*D codes form a little-endian bit stream (element f at stream
 * bits [f*w, f*w + w), stream bit k = bit (k & 7) of byte k >> 3) of ceil(F*w/8) bytes stored at
 * packed_{k,v}_dev + row_offset[b*row_capacity + r].  The same offsets serve K and V.
 * scale_zp[(b*row_capacity + r)*4 + {0,1,2,3}] = {k_scale, k_zero_point, v_scale, v_zero_point}
 * (values exactly representable in the K/V dtype, stored as fp32). */
typedef struct rtkv_layer_out {
  /* dequantized K' in the K/V dtype, [B, rows, H, D] via strides.  o_stride_b = -1 packs batch rows
   * back to back at the RUNTIME row count: batch stride = S'_max * o_stride_s, so a contiguous
   * [B, S'_max, H*D] result needs no host round trip before the launch. */
  void* k_out_dev;
  void* v_out_dev;
  int64_t o_stride_b, o_stride_s, o_stride_h;
  int64_t row_capacity;      /* rows available per batch row (>= S'_max; S is always enough) */
  float* scores_dev;         /* [B, S] fp32 importance scores */
  uint8_t* labels_dev;       /* [B, S] precision classes */
  uint8_t* mask_dev;         /* [B, S] 1 = selected */
  int32_t* kept_index_dev;   /* [B, row_capacity] original token index per output row, -1 = pad */
  uint8_t* packed_k_dev;     /* packed code buffers (capacity packed_capacity bytes each) */
  uint8_t* packed_v_dev;
  int64_t packed_capacity;
  int64_t* row_offset_dev;   /* [B, row_capacity] byte offset of each row's codes */
  float* scale_zp_dev;       /* [B, row_capacity, 4] */
  rtkv_layer_stats* stats_dev;
} rtkv_layer_out;

/* ------------------------------------------------------------------------------------------------
 * Library / sizing
 * ---------------------------------------------------------------------------------------------- */
const char* rtkv_version(void);
const char* rtkv_last_error(void);

/* Bits per packed element for a class of `bits` on `dtype`: bits, or bits+1 when the clamp bound
 * qmax = 2^bits-1 is not representable in dtype (then PyTorch's clamp rounds it up to 2^bits and a
 * code can equal 2^bits; dynamic_quantization.py:121).  0 if unsupported (bits outside 1..16, or
 * fp16 with bits = 16, which the reference rejects). */
int rtkv_field_width(int dtype, int bits);

/* Scratch bytes needed by the entry points below for B batch rows of S tokens. */
size_t rtkv_workspace_size(int64_t B, int64_t S);

/* Upper bound of packed bytes per tensor for B*S rows of F elements at the widest class. */
int64_t rtkv_packed_capacity(int64_t B, int64_t S, int64_t F, int dtype, const int32_t bits[3]);

/* ------------------------------------------------------------------------------------------------
 * Stage entry points (each replaces one reference method; used by the Python mirror classes)
 * ---------------------------------------------------------------------------------------------- */

/* A[b,i] = Σ_{p<P} mean_h W[b,h,i,p], rounded to W's dtype and stored as fp32.
 * Replaces PromptGuidedImportanceScorer.compute_attention_aggregation (token_importance.py:21-47).
 * The summation order reproduces PyTorch's CPU cascade sum (AVX2 kernels), so results are
 * bit-identical to the reference's CPU path. */
int rtkv_attention_aggregation(const rtkv_attn_desc* w, int32_t prompt_len, float* A_dev,
                               void* workspace_dev, size_t workspace_bytes, void* stream);

/* Per-row min-max normalisation of x[B,S] (dtype), output in the same dtype.
 * Replaces PromptGuidedImportanceScorer.normalize_attention_scores (token_importance.py:49-85). */
int rtkv_minmax_normalize(const void* x_dev, int dtype, int64_t B, int64_t S, void* out_dev,
                          void* stream);

/* pos[i] = log(i+1)/log(S) in fp32 (0 if S <= 1), bit-identical to torch.log on CPU.
 * Replaces PromptGuidedImportanceScorer.compute_position_bias (token_importance.py:87-110). */
int rtkv_position_bias(int64_t S, float* pos_dev, void* stream);

/* scores[b,i] from A (values rounded to a_dtype): α·N·w_l + β·pos + γ·min(1, P/S).
 * Replaces compute_importance_scores given its aggregation (token_importance.py:134-176). */
int rtkv_importance_scores(const float* A_dev, int a_dtype, int64_t B, int64_t S,
                           const rtkv_layer_params* p, float* scores_dev,
                           void* workspace_dev, size_t workspace_bytes, void* stream);

/* labels[b,i] ∈ {0,1,2} from thresholds; per-class counts into stats (class_count).
 * Replaces DynamicPrecisionQuantizer.assign_precision_levels (dynamic_quantization.py:21-60). */
int rtkv_assign_precision(const float* scores_dev, int64_t B, int64_t S, const rtkv_layer_params* p,
                          uint8_t* labels_dev, rtkv_layer_stats* stats_dev,
                          void* workspace_dev, size_t workspace_bytes, void* stream);

/* Budgeted greedy selection + emergency fallback + ordered compaction map.
 * Replaces SelectiveTokenPropagator.select_tokens_with_budget (selective_propagation.py:68-161) and
 * the selection half of apply_token_selection (:163-211).  Tie order among equal scores is
 * (score desc, index asc). */
int rtkv_select_tokens(const float* scores_dev, const uint8_t* labels_dev, int64_t B, int64_t S,
                       const rtkv_layer_params* p, uint8_t* mask_dev, int32_t* kept_index_dev,
                       int64_t row_capacity, int64_t* row_offset_dev, int64_t F, int kv_dtype,
                       rtkv_layer_stats* stats_dev, void* workspace_dev, size_t workspace_bytes,
                       void* stream);

/* Quantize/dequantize/pack the rows listed in kept_index (or every token when kept_index_dev is
 * NULL: output row r = token r), with per-row class from labels.  Row count per batch row is read
 * from stats_dev->batch[b].kept (or S when kept_index_dev is NULL).
 * Replaces DynamicPrecisionQuantizer.apply_mixed_precision_quantization
 * (dynamic_quantization.py:128-196) fused with the gather of apply_token_selection (:214-232). */
int rtkv_quantize_rows(const rtkv_kv_desc* kv, const uint8_t* labels_dev,
                       const int32_t* kept_index_dev, const rtkv_layer_params* p,
                       const rtkv_layer_out* out, void* stream);

/* Fused driver: aggregation → scores → labels → selection → quantize+pack+compact for one layer.
 * Replaces RealTimePrefillCompressor.compress_layer_kv_cache (unified_compressor.py:95-172).
 * Three kernel launches, no host synchronisation; read out->stats_dev after the stream syncs. */
int rtkv_compress_layer(const rtkv_kv_desc* kv, const rtkv_attn_desc* w, const rtkv_layer_params* p,
                        const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes,
                        void* stream);

/* rtkv_compress_layer that also records hipEvent_t events[0..3] on `stream` before K1, after K1
 * (aggregation), after K2 (scores/classes/selection) and after K4 (quantize+pack+compact), so a
 * caller can time each kernel of the fused path without changing it (bench.py's roofline). */
int rtkv_compress_layer_events(const rtkv_kv_desc* kv, const rtkv_attn_desc* w,
                               const rtkv_layer_params* p, const rtkv_layer_out* out,
                               void* workspace_dev, size_t workspace_bytes, void* stream,
                               void* const events[4]);

/* Early statistics (no reference counterpart: it serves the drop-in's host sync).  The reference
 * caller needs the layer's output shape S' before compress_layer_kv_cache returns (the K'/V' views),
 * so the drop-in waits for the statistics once per layer.  S' and every count are final as soon as
 * the selection thresholds are (K2's first kernel), so with rtkv_compress_layer_early the device
 * writes them into `early_host` (host memory from rtkv_host_alloc) and then `seq`; the host spins on
 * that word (rtkv_wait_early) while the rest of K2 and all of K4 still run, and only score_m2 and
 * kept_score_sum must be read from stats_dev after the stream syncs.  *published = 1 when this call
 * will publish (the one-launch K2: B = 1, S <= 65536); 0: read stats_dev after a stream sync.
 * complete = 0 on publication means the top-10% fallback ran: read stats_dev after a sync too. */
/* The published statistics are ONE 128-byte line (this struct's first 128 bytes, 128-byte aligned: the
 * start of an rtkv_host_alloc block) written by ONE wave store instruction (16 lanes x 8 bytes), with the
 * call's seq in its first AND last word: a line that reaches host memory in two 64-byte halves is never
 * taken as complete, and no ordering wait (nor a system-scope release, whose L2 write-back cost the
 * selection kernel ~4 us) is needed before the seq.  B = 1: kept = max_kept, packed_bytes =
 * total_packed_bytes; score_m2 and kept_score_sum are not part of it (read after the layer). */
typedef struct rtkv_early_stats {
  uint64_t seq;                 /* word 0 */
  int64_t max_kept;             /* S' (= the batch row's kept count) */
  int64_t total_packed_bytes;   /* (= the batch row's packed bytes) */
  double score_sum;
  float score_min, score_max;
  int32_t error_flags;
  int32_t complete;             /* 1: complete (0: the top-10% fallback ran, read stats_dev after a sync) */
  int64_t class_count[3];
  int64_t kept_class[3];
  int64_t cost_units;
  int64_t reserved[2];
  uint64_t seq_tail;            /* word 15: seq again */
  /* Written by K4 (rtkv_compress_layer_finish) when it starts, all selection waits being over: ONE
   * 8-byte store of (seq mod 2^48) << 16 | the layer's complete RTKV_FLAG_* word.  A flag raised after the
   * early publication (a look-back timeout) or by K4 itself (RTKV_FLAG_OUTPUT_OVERFLOW) is seen here
   * without a stream sync. */
  uint64_t final_word;
  uint64_t reserved2[15];
} rtkv_early_stats;

int rtkv_compress_layer_early(const rtkv_kv_desc* kv, const rtkv_attn_desc* w, const rtkv_layer_params* p,
                              const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes,
                              void* stream, rtkv_early_stats* early_host, uint64_t seq, int32_t* published);
int rtkv_compress_layer_qk_early(const rtkv_kv_desc* kv, const rtkv_qk_desc* q, const rtkv_layer_params* p,
                                 const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes,
                                 void* stream, rtkv_early_stats* early_host, uint64_t seq, int32_t* published);
/* Spin until early_host->seq == seq_tail == seq (RTKV_OK) or timeout_us passes (RTKV_ERR_TIMEOUT). */
int rtkv_wait_early(const rtkv_early_stats* early_host, uint64_t seq, int64_t timeout_us);

/* The layer in two calls, for exactly-sized outputs (the drop-in: the reference returns K'/V' of S'
 * rows, unified_compressor.py:170 / selective_propagation.py:214-232).  rtkv_compress_layer_begin runs
 * K1 and K2 and publishes the early statistics as rtkv_compress_layer_early does; `out` needs only
 * the per-token buffers (scores, labels, mask, kept_index, row_offset, scale_zp, stats; row_capacity
 * >= S).  With S' and the packed byte count known (rtkv_wait_early, or stats_dev after a stream sync
 * when *published = 0), the caller allocates K'/V' of [B, S', F] and packed buffers of exactly that
 * many bytes and calls rtkv_compress_layer_finish (K4) with the same per-token buffers, the same
 * row_capacity and workspace, o_stride_b = -1, on the same stream.
 *
 * Between begin and finish the workspace and the per-token buffers BELONG TO THE PENDING LAYER: K2
 * leaves each kept row's class and the selection scratch there for K4, so a begin or compress call
 * that reuses the same workspace before finish corrupts the pending layer (stream order hides it).
 *
 * finish: out_rows = the rows per batch row K'/V' hold (>= the published S'_max; ignored without
 * EMIT_DEQUANT), out->packed_capacity = the bytes of each packed buffer; both must come from THIS
 * layer's published statistics.  K4 compares them with the device statistics and, if either is too
 * small, writes nothing and sets RTKV_FLAG_OUTPUT_OVERFLOW.  If the selection timed out
 * (RTKV_FLAG_SPIN_TIMEOUT, possibly after the early publication) K4 writes NaN rows and NaN
 * scale/zero-points instead of codes.  early_host (nullable, the begin call's buffer) + seq: K4
 * publishes the layer's final flags there (final_flags / final_seq), so the host can check the
 * layer before it trusts the outputs without syncing the stream. */
int rtkv_compress_layer_begin(const rtkv_kv_desc* kv, const rtkv_attn_desc* w, const rtkv_layer_params* p,
                              const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes, void* stream,
                              rtkv_early_stats* early_host, uint64_t seq, int32_t* published, void* start_event);
int rtkv_compress_layer_qk_begin(const rtkv_kv_desc* kv, const rtkv_qk_desc* q, const rtkv_layer_params* p,
                                 const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes, void* stream,
                                 rtkv_early_stats* early_host, uint64_t seq, int32_t* published, void* start_event);
int rtkv_compress_layer_finish(const rtkv_kv_desc* kv, const rtkv_layer_params* p, const rtkv_layer_out* out,
                               int64_t out_rows, void* workspace_dev, size_t workspace_bytes, void* stream,
                               rtkv_early_stats* early_host, uint64_t seq);
/* Spin until early_host->final_word carries seq, i.e. until the finish call's K4 has started and published
 * the layer's final flags (RTKV_OK; read final_flags then), or timeout_us passes (RTKV_ERR_TIMEOUT).
 * The drop-in's strict mode (RealTimePrefillCompressor(strict=True)) waits here before it returns, so a
 * selection that timed out after the early publication raises in the layer's own call — where the
 * reference caller's try/except falls back for that layer (modified_llama.py:144-149). */
int rtkv_wait_final(const rtkv_early_stats* early_host, uint64_t seq, int64_t timeout_us);
/* start_event (nullable, a hipEvent_t): recorded on the stream right before K1, in the same call —
 * the start of the drop-in's processing_time.  (Recorded from the host separately before this call,
 * the timing event cost ~4.5 us of device idle per layer; recorded here, as rtkv_compress_layer_events
 * does, nothing measurable.) */
/* Between begin and finish (drop-in path, no reference counterpart): read the first kept rows of K
 * and V — K4's first tasks — up to max_bytes in total, with the default cache policy, so that they are
 * in the Infinity Cache when K4 starts.  Enqueue right after begin, on its stream: it runs while the
 * host waits for the early statistics and allocates the outputs.  Loads only (no output); a no-op for
 * B > 1 or rows that are not contiguous and 16-byte aligned. */
int rtkv_prefetch_kept_rows(const rtkv_kv_desc* kv, const rtkv_layer_out* out, int64_t max_bytes, void* stream);
/* Pinned, device-coherent host memory for rtkv_early_stats (hipHostMalloc, coherent + mapped). */
void* rtkv_host_alloc(size_t bytes);
void rtkv_host_free(void* p);

/* ------------------------------------------------------------------------------------------------
 * Sequence shards (multi-GPU prefill; no reference counterpart — the reference is single-device).
 * Rank j of N owns tokens [row0, row0 + S_local) of an S_total-token prefill.  Per layer:
 *   1. rtkv_attention_aggregation_shard on its W rows          → A_local [B, S_local]
 *   2. all-gather A (4 B/token)                                 → A [B, S_total] on every rank
 *   3. rtkv_finalize_select on A (replicated, deterministic)    → scores, labels, selection, offsets
 *   4. rtkv_shard_ranges                                        → per-rank output row / byte bounds
 *   5. rtkv_quantize_rows_shard on its K/V rows                 → its kept rows: packed codes at
 *      their global byte offsets (the single-GPU layout), dequantized rows local
 * and one exchange of every rank's row/byte ranges at the end: every rank then holds the
 * single-GPU result byte for byte.
 * ---------------------------------------------------------------------------------------------- */

/* rtkv_attention_aggregation of W rows [row0, row0 + w->S) of an S_total-row attention matrix:
 * bit-identical to rows [row0, row0 + S) of the unsharded aggregation. */
int rtkv_attention_aggregation_shard(const rtkv_attn_desc* w, int32_t prompt_len, int64_t row0,
                                     int64_t S_total, float* A_dev, void* stream);

/* Scores → classes → budgeted selection → compaction map from a (gathered) aggregation A [B, S]
 * (values rounded to a_dtype): the second kernel group of rtkv_compress_layer.  Writes out->scores,
 * labels, mask, kept_index, row_offset (when RTKV_EMIT_PACKED) and stats. */
int rtkv_finalize_select(const float* A_dev, int a_dtype, int64_t B, int64_t S, const rtkv_layer_params* p,
                         const rtkv_layer_out* out, int64_t F, int kv_dtype, void* workspace_dev,
                         size_t workspace_bytes, void* stream);

/* Step 1 that also clears what the same layer's rtkv_finalize_select_shard needs zeroed (the selection
 * scratch in workspace_dev — sized by rtkv_workspace_size(B, S_total) — and out->stats_dev), so that call,
 * with scratch_zeroed = 1 and the same params, runs without its two memset launches.  Same A as
 * rtkv_attention_aggregation_shard. */
int rtkv_attention_aggregation_shard_ws(const rtkv_attn_desc* w, int32_t prompt_len, int64_t row0,
                                        int64_t S_total, float* A_dev, const rtkv_layer_params* p,
                                        const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes,
                                        void* stream);

/* Steps 3 and 4 in one call: rtkv_finalize_select on the gathered A (S = nranks·S_local tokens), then the
 * rtkv_shard_ranges table of this layer.  Where the one-launch selection applies (B = 1, S <= 65536) its
 * compaction phase writes the table itself: one launch instead of two (three with the memsets; none when
 * scratch_zeroed = 1 after rtkv_attention_aggregation_shard_ws).  Same outputs as the separate calls. */
int rtkv_finalize_select_shard(const float* A_dev, int a_dtype, int64_t B, int64_t S, const rtkv_layer_params* p,
                               const rtkv_layer_out* out, int64_t F, int kv_dtype, int64_t S_local, int32_t nranks,
                               int64_t* ranges_dev, int32_t scratch_zeroed, void* workspace_dev,
                               size_t workspace_bytes, void* stream);

/* rtkv_quantize_rows for the kept rows whose token lies in [row0, row0 + kv->S) (rank `rank` of
 * `nranks`); kv describes the local K/V rows (token row0 + i at local row i).  Packed codes and
 * scale/zero-point land at their global positions.  Dequantized rows: with ranges_dev (the
 * rtkv_shard_ranges table of this layer) at LOCAL output row r - first_row(b, rank), batch stride
 * out->o_stride_b (required >= 0); without it at the global output row, rank 0 writing the zero
 * padding rows. */
int rtkv_quantize_rows_shard(const rtkv_kv_desc* kv, int64_t row0, int64_t S_total, int32_t rank,
                             int32_t nranks, const int64_t* ranges_dev, const uint8_t* labels_dev,
                             const int32_t* kept_index_dev, const rtkv_layer_params* p,
                             const rtkv_layer_out* out, void* stream);

/* ranges_dev[(b*(nranks+1) + j)*2 + {0,1}] = {first output row, first packed byte} of rank j's tokens
 * [j*S_local, (j+1)*S_local) in batch row b; j = nranks is the end of the row.  row_offset_dev may be
 * NULL (bytes = 0). */
int rtkv_shard_ranges(const int32_t* kept_index_dev, const int64_t* row_offset_dev,
                      const rtkv_layer_stats* stats_dev, int64_t B, int64_t row_capacity, int64_t S_local,
                      int32_t nranks, int64_t* ranges_dev, void* stream);

/* Shard collectives on RCCL (xGMI), for a host without torch.distributed.  The communicator is
 * RCCL's (ncclComm_t), created from a 128-byte id that rank 0 makes and the host broadcasts by any
 * means (rtkv/sharded.py uses its process group).  RCCL is loaded on first use (dlopen
 * "librccl.so.1"); RTKV_ERR_UNSUPPORTED when it cannot be.  Both exchanges are grouped
 * point-to-point launches of exact ranges on `stream`, stream-ordered like the kernels.
 * Replace the torch.distributed calls of rtkv/sharded.py (ShardedPrefillCompressor: the A
 * all-gather and _send_recv), which have no reference counterpart (the reference is one device). */
#define RTKV_COMM_ID_BYTES 128
int rtkv_comm_unique_id(uint8_t* id, size_t id_bytes);
int rtkv_comm_init(void** comm, const uint8_t* id, size_t id_bytes, int32_t nranks, int32_t rank);
int rtkv_comm_destroy(void* comm);
/* Step 2: a_dev[b][j*S_local + i] = rank j's a_local_dev[b][i] on every rank (fp32, B batch rows). */
int rtkv_allgather_rows(void* comm, const float* a_local_dev, float* a_dev, int64_t B, int64_t S_local,
                        void* stream);
/* The end of a layer: rank j's packed K/V bytes [first byte(j), first byte(j+1)) and scale/zp rows
 * [first row(j), first row(j+1)) of every batch row, from j to every other rank, in place in `out`
 * (the single-GPU layout).  ranges_host: this layer's rtkv_shard_ranges table copied to the host. */
int rtkv_allgather_packed(void* comm, const int64_t* ranges_host, int64_t B, int64_t row_capacity,
                          const rtkv_layer_out* out, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Fused importance mode (MFMA): the aggregation A from Q, K_prompt and the row LSE instead of W.
 * A is fp32 (W is not rounded to the input dtype: the reference model runs in fp32); parity with the
 * W path is a tolerance, not bit-exact.  Replaces compute_attention_aggregation
 * (token_importance.py:21-47) fed by the materialised softmax of modified_llama.py:88-94.
 * ---------------------------------------------------------------------------------------------- */
int rtkv_importance_qk_lse(const rtkv_qk_desc* q, int32_t prompt_len, float* A_dev, void* stream);
/* The same with a [B][H][S] fp32 scratch (rtkv_qk_scratch_size bytes): the head-major kernel (the
 * prompt keys of one head staged once per workgroup, per-head row sums reduced in head order) when
 * S % 4 == 0, D = 128 and P > 64 — the kernel rtkv_compress_layer_qk uses when its workspace has
 * rtkv_workspace_size_qk(B, H, S) bytes.  Same tolerance as above; the two kernels differ in the
 * summation order only. */
size_t rtkv_qk_scratch_size(int64_t B, int64_t H, int64_t S);
size_t rtkv_workspace_size_qk(int64_t B, int64_t H, int64_t S);
int rtkv_importance_qk_lse_ws(const rtkv_qk_desc* q, int32_t prompt_len, float* A_dev, void* scratch_dev,
                              size_t scratch_bytes, void* stream);

/* Model-side mask check (the mask the reference adds before its softmax,
 * modified_llama.py:90-91).  mask[b*stride_b + i*stride_i + j*stride_j] for i, j < S, dtype fp32/f16/bf16
 * (B = the mask's batch rows).  thr = finfo(dtype).min / 2 rounded to the dtype (the host passes it).
 * Writes valid[b*valid_stride_b + j] = 1 unless the last query row masks key j, and ADDS to counts_dev
 * (two uint64, zeroed by the caller): counts[0] = entries that break "causal ∧ key padding" (an entry
 * must be 0 where j <= i and key j is valid, else <= thr), counts[1] = padded keys.  One pass over the
 * mask, no [B, S, S] temporaries; the caller reads both counts with one sync. */
int rtkv_mask_key_padding(const void* mask_dev, int32_t dtype, int64_t B, int64_t S, int64_t stride_b,
                          int64_t stride_i, int64_t stride_j, float thr, uint8_t* valid_dev, int64_t valid_stride_b,
                          unsigned long long* counts_dev, void* stream);

/* Row log-sum-exp of the prefill attention: lse[b,h,i] = log Σ_j exp(q_i·k_j·scale)
 * over j ≤ i (causal) or all j < S, without materialising the [B,H,S,S] softmax of
 * modified_llama.py:88-94 — the producer of the lse that rtkv_importance_qk_lse consumes.  Reads
 * q_dev / k_dev / strides / causal / scale of the descriptor (lse_dev is ignored; row0 must be 0) and
 * writes lse_out[b*lse_stride_b + h*lse_stride_h + i] (fp32).  head_dim 64 or 128, fp16/bf16. */
int rtkv_attention_lse(const rtkv_qk_desc* q, float* lse_out_dev, void* stream);

/* rtkv_compress_layer with the fused importance mode (K1' on MFMA, then K2 and K4 unchanged). */
int rtkv_compress_layer_qk(const rtkv_kv_desc* kv, const rtkv_qk_desc* q, const rtkv_layer_params* p,
                           const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes,
                           void* stream);
int rtkv_compress_layer_qk_events(const rtkv_kv_desc* kv, const rtkv_qk_desc* q, const rtkv_layer_params* p,
                                  const rtkv_layer_out* out, void* workspace_dev, size_t workspace_bytes,
                                  void* stream, void* const events[4]);

/* Reconstruct dequantized rows from packed codes (+ scale/zp, labels of the kept rows); bit-identical
 * to the RTKV_EMIT_DEQUANT output.  rows_per_batch[b] rows of batch row b are decoded.
 * Consumer side of the packed format (compression_layers.py:7-45 CompressedKVCache). */
int rtkv_unpack_dequant(const uint8_t* packed_dev, const int64_t* row_offset_dev,
                        const float* scale_zp_dev, int which /*0=K,1=V*/,
                        const int32_t* kept_index_dev, const uint8_t* labels_dev /*[B,S]*/,
                        int64_t B, int64_t S, int64_t row_capacity, const int64_t* rows_dev,
                        int64_t H, int64_t D, int dtype, const int32_t bits[3], void* out_dev,
                        int64_t o_stride_b, int64_t o_stride_s, int64_t o_stride_h, void* stream);

/* Decode attention over one layer's PACKED KV: for every batch row b and query head
 * h, out[b,h,:] = softmax_j(q[b,h]·K'[b,j,h/G]ᵀ·scale)·V'[b,j,h/G] over the kept rows j < rows[b],
 * where K'/V' are decoded from the packed codes on the fly, element for element the dequantized
 * rows rtkv_compress_layer writes.  Replaces the reference's attention over the dequantized cache
 * (modified_llama.py:140-142, 165-166) without materialising K'/V'.  Arguments as
 * rtkv_unpack_dequant (H = Hkv kv heads of head_dim D, F = Hkv·D a multiple of 512;
 * packed field widths 2/4/8/16), plus q [B, Hq, D] in the K/V dtype (Hq a multiple of Hkv: GQA),
 * scale (1/sqrt(D) in the reference, modified_llama.py:89) and out [B, Hq, D] fp32.  Workspace:
 * rtkv_decode_workspace_size(B, Hq, Hkv, D, row_capacity) bytes.  packed_bytes = size of each code
 * buffer: a row whose offset + F·w/8 passes it reads as zero codes, rows[b] is clamped to
 * row_capacity and kept indices to [0, S), so inconsistent metadata cannot read outside the buffers. */
size_t rtkv_decode_workspace_size(int64_t B, int64_t Hq, int64_t Hkv, int64_t D, int64_t row_capacity);
int rtkv_decode_attention_packed(const uint8_t* packed_k_dev, const uint8_t* packed_v_dev, int64_t packed_bytes,
                                 const int64_t* row_offset_dev, const float* scale_zp_dev,
                                 const int32_t* kept_index_dev, const uint8_t* labels_dev, int64_t B, int64_t S,
                                 int64_t row_capacity, const int64_t* rows_dev, int64_t Hkv, int64_t D, int dtype,
                                 const int32_t bits[3], const void* q_dev, int64_t Hq, float scale,
                                 float* out_dev, void* workspace_dev, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Extension "rtkv-gq/1": per-channel outlier detection + per-head group-wise 2/4/8-bit pack.
 * NO REFERENCE COUNTERPART — the reference quantizes each token with one (scale, zero_point) over all H·D
 * channels (dynamic_quantization.py:181-194).  Opt-in (rtkv.GroupQuantConfig; off by default, so the
 * reference path and its goldens are untouched); parity UNPINNED: oracle/rtkv_oracle.c rtkvo_gq_* defines
 * the mode and the kernels match it byte for byte.  B = 1, head_dim 128 (one group per head), K/V rows
 * [S, H·128] with contiguous heads, H a multiple of 4, class widths 2/4/8 bits.
 *   1. rtkv_gq_outlier_channels: every vote_stride-th kept row votes, per head, for its n_vote channels of
 *      largest |x| (ties: the lower channel; DPP row maxima over keys unique within the head); the
 *      n_outlier channels with the most votes (at least max(1, ceil(samples·min_votes_pm/1000))) are the
 *      layer's outlier channels of each head and tensor: outlier_idx[2][H][n_outlier] (channel within the
 *      head, -1 = unused slot).  One launch (the selection runs in the vote grid's last workgroup);
 *      workspace: rtkv_gq_workspace_size(H, D) bytes (the votes and a done count, zeroed by the call);
 *      row_capacity < 2^25.
 *   2. rtkv_gq_pack: per (kept row, tensor, head) the reference's per-token formulas (dynamic_quantization.py
 *      :62-126, each op rounded to the dtype) over the head's non-outlier channels: codes of the row's class
 *      width for every channel (outlier channels and NaN: code 0) at codes + row_offset[r] (the per-token
 *      layout's row slots: F·w/8 bytes), meta[r][tensor][h] = {scale, zero_point} and raw[r][tensor][h][s] =
 *      the outlier channels' input values, both in the K/V dtype.
 *   3. rtkv_gq_unpack: the dequantized rows ((q − zp)·scale, outlier channels restored bit for bit).
 *   4. rtkv_gq_decode_attention: decode attention over the format (as rtkv_decode_attention_packed).
 * Rows: the first min(stats->kept, row_capacity) kept rows (kept_index, labels: the layer's per-token
 * outputs). */
typedef struct rtkv_gq_params {
  int32_t n_outlier;      /* outlier channels per head and tensor, 0..16 */
  int32_t n_vote;         /* channels each sampled row votes for, per head */
  int32_t vote_stride;    /* every vote_stride-th kept row votes */
  int32_t min_votes_pm;   /* votes a channel needs, per mille of the sampled rows (rounded up, at least 1) */
} rtkv_gq_params;
size_t rtkv_gq_workspace_size(int64_t H, int64_t D);
int rtkv_gq_outlier_channels(const rtkv_kv_desc* kv, const int32_t* kept_index_dev, const uint8_t* labels_dev,
                             const rtkv_layer_stats* stats_dev, const rtkv_gq_params* g, int64_t row_capacity,
                             int16_t* outlier_idx_dev, void* workspace_dev, size_t workspace_bytes, void* stream);
int rtkv_gq_pack(const rtkv_kv_desc* kv, const int32_t* kept_index_dev, const uint8_t* labels_dev,
                 const rtkv_layer_stats* stats_dev, const int32_t bits[3], const rtkv_gq_params* g,
                 const int16_t* outlier_idx_dev, const int64_t* row_offset_dev, uint8_t* codes_k_dev,
                 uint8_t* codes_v_dev, int64_t codes_capacity, void* meta_dev, void* raw_dev, int64_t row_capacity,
                 void* stream);
int rtkv_gq_unpack(const rtkv_kv_desc* kv, const int32_t* kept_index_dev, const uint8_t* labels_dev,
                   const rtkv_layer_stats* stats_dev, const int32_t bits[3], const rtkv_gq_params* g,
                   const int16_t* outlier_idx_dev, const int64_t* row_offset_dev, const uint8_t* codes_dev,
                   int64_t codes_capacity, const void* meta_dev, const void* raw_dev, int64_t row_capacity, int which,
                   void* out_dev, void* stream);
size_t rtkv_gq_decode_workspace_size(int64_t Hq, int64_t Hkv);
int rtkv_gq_decode_attention(const rtkv_kv_desc* kv, const int32_t* kept_index_dev, const uint8_t* labels_dev,
                             const rtkv_layer_stats* stats_dev, const int32_t bits[3], const rtkv_gq_params* g,
                             const int16_t* outlier_idx_dev, const int64_t* row_offset_dev, const uint8_t* codes_k_dev,
                             const uint8_t* codes_v_dev, int64_t codes_capacity, const void* meta_dev,
                             const void* raw_dev, int64_t row_capacity, const void* q_dev, int64_t Hq, float scale,
                             float* out_dev, void* workspace_dev, size_t workspace_bytes, void* stream);

/* Copy the kept rows of a row-major tensor (row r of batch b = src row kept_index[b*cap + r]), zero
 * rows for r in [kept_b, S'_max), rows of row_bytes bytes, into dst (batch stride dst_stride_b bytes,
 * or S'_max*row_bytes when -1).  The pure gather of apply_token_selection (selective_propagation.py
 * :224-232) for tensors the caller did not quantize (K/V, scores, labels). */
int rtkv_gather_rows(const void* src_dev, int64_t B, int64_t S, int64_t row_bytes,
                     const int32_t* kept_index_dev, int64_t row_capacity, int64_t src_stride_b,
                     void* dst_dev, int64_t dst_stride_b, int64_t src_stride_s,
                     const rtkv_layer_stats* stats_dev, void* stream);

/* Whole-tensor helpers (one scale/zero-point over all elements of the selected rows of an
 * [n_rows, row_len] tensor; row_labels_dev = NULL selects every row, otherwise the rows whose
 * label equals label_value):
 *   rtkv_tensor_quant_params: DynamicPrecisionQuantizer.get_quantization_params
 *     (dynamic_quantization.py:62-95) → scale_zp_dev[0..1] (fp32 storage of dtype values);
 *     workspace >= 8 KiB;
 *   rtkv_tensor_fake_quant: DynamicPrecisionQuantizer.quantize_tensor (:97-126) with that pair,
 *     writing only the selected rows of out_dev.
 * AdaptiveQuantization.forward (compression_layers.py:150-175) is one params + fake_quant pair per
 * precision class. */
int rtkv_tensor_quant_params(const void* x_dev, int dtype, int64_t n_rows, int64_t row_len,
                             const uint8_t* row_labels_dev, int32_t label_value, int bits,
                             float* scale_zp_dev, void* workspace_dev, size_t workspace_bytes,
                             void* stream);
int rtkv_tensor_fake_quant(const void* x_dev, int dtype, int64_t n_rows, int64_t row_len,
                           const uint8_t* row_labels_dev, int32_t label_value, int bits,
                           const float* scale_zp_dev, void* out_dev, void* stream);

/* Numerics self-check (no reference counterpart; replaces nothing).  The quantizer divides by the
 * row scale with a reciprocal + one FMA correction instead of the IEEE division where a row-uniform
 * gate admits it; this enumerates every (dividend, positive divisor) pair of the 16-bit dtype that
 * the fast path admits and counts bitwise differences from the IEEE fp32 quotient.
 * counts_dev[0] = pairs checked, counts_dev[1] = mismatches (must be 0).  RTKV_ERR_UNSUPPORTED for
 * RTKV_F32: see rtkv_selfcheck_division_f32. */
int rtkv_selfcheck_division(int32_t dtype, unsigned long long* counts_dev, void* stream);

/* The fp32 counterpart, one divisor range per call (adds to counts_dev, which the caller zeroes):
 * dividends x = ±(1 + xm·2^-23)·2^ex for EVERY mantissa xm, divisors s = (1 + sm·2^-23)·2^es for
 * sm in [s_lo, s_hi) ⊆ [0, 2^23).  Over ex = es = 0 and the whole range this is every mantissa pair,
 * which proves the gated fp32 fast quotient (all its steps stay normal, so they commute with
 * power-of-two scaling); other exponents spot-check that argument. */
int rtkv_selfcheck_division_f32(int64_t s_lo, int64_t s_hi, int32_t ex, int32_t es, int32_t negative,
                                unsigned long long* counts_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RTKV_H */
