/*
 * bloomstage.h — C-ABI of libbloomstage.so, the MI355X-native per-stage BLOOM forward.
 *
 * Drop-in boundary for the reference's JNI stage library.  Every entry
 * point below names the reference interface it replaces:
 *
 *   bs_init_stage      <- Java_..._Communication_createSession (native-lib.cpp:671-678)
 *                         + SessionCache ctor (session_cache.h:26-35): load one module
 *   bs_release         <- Java_..._Communication_releaseSession (native-lib.cpp:1290-1303)
 *   bs_forward         <- runInferenceMasterResidual (native-lib.cpp:942-1034, header stage),
 *                         runInferenceWorkerResidual (:1036-1194, middle stage),
 *                         runInferenceWorkerResidualLastGeneration (:1368-1443, tail stage),
 *                         all of which end in inference::run_inference (inference.cpp:145-218)
 *   bs_reset_kv        <- (none: the reference has no KV cache; new sample == new slot)
 *   bs_last_error      <- (none: the reference throws C++ exceptions across JNI,
 *                         native-lib.cpp:986-988; here errors are status codes + this string)
 *   bs_forward on a BS_FLAG_CLASSIFIER stage
 *                      <- runInferenceWorkerResidualLastClassification (native-lib.cpp:1305-1366)
 *                         -> inference::run_inference_with_binary_classification (inference.cpp:220-270)
 *   bs_binary_classify <- Java_..._binaryClassify (native-lib.cpp:128-160) -> inference::binary_classify
 *                         (inference.cpp:57-69)
 *   bs_codec_*         <- utils::SerializeTensorVectorToBytes / DeserializeTensorVectorFromBytes
 *                         (utils.cpp:124-264 / :266-368), byte-exact wire format
 *   bs_serialize_int / bs_deserialize_int
 *                      <- utils::SerializeInt / DeserializeInt (utils.cpp:11-25),
 *                         Java_..._deserializeInt (native-lib.cpp:1445-1471)
 *
 * Conventions: no exceptions cross this ABI; every int-returning call returns BS_OK (0)
 * or a negative bs_status and sets a thread-local message readable via bs_last_error().
 * Plain pointers and sizes only.  Device pointers live on the stage's device.
 */
#ifndef BLOOMSTAGE_H
#define BLOOMSTAGE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BS_ABI_VERSION 3

typedef enum {
  BS_OK = 0,
  BS_ERR_INVALID = -1,   /* bad argument / shape outside the stage's capacity */
  BS_ERR_DEVICE = -2,    /* HIP runtime error */
  BS_ERR_OOM = -3,       /* device allocation failed */
  BS_ERR_STATE = -4,     /* call not valid in the stage's current state */
  BS_ERR_UNSUPPORTED = -5/* e.g. wire dtype the reference codec does not carry */
} bs_status;

/* Element types: values are ONNXTensorElementDataType (onnxruntime_c_api.h:175-191). */
typedef enum {
  BS_DT_FLOAT = 1, BS_DT_UINT8 = 2, BS_DT_INT8 = 3, BS_DT_UINT16 = 4, BS_DT_INT16 = 5,
  BS_DT_INT32 = 6, BS_DT_INT64 = 7, BS_DT_BOOL = 9, BS_DT_DOUBLE = 11, BS_DT_UINT32 = 12,
  BS_DT_UINT64 = 13, BS_DT_BFLOAT16 = 16
} bs_dtype;

typedef enum {
  BS_WEIGHTS_SYNTHETIC = 0, /* repo generator (DESIGN.md "Synthetic weights"), built on device */
  BS_WEIGHTS_HOST = 1       /* fp32 host buffer in canonical stage order (bs_stage_weight_count) */
} bs_weight_source;

/* desc->flags.  BS_FLAG_INT8_WEIGHTS (bf16 stages): weight-only int8 for the four block matrices
 * (qkv, dense, fc1, fc2) -- the reference's bloom*-int8 model variants (server.py:796-799,
 * data/Data.kt:19-30).  Per output row n: scale[n] = max_k |W[n][k]| / 127 (1 for a zero row),
 * Q[n][k] = round-half-even(W[n][k] / scale[n]) in [-127, 127], W = the bf16 weight.  Embeddings,
 * LayerNorms, biases and the tied lm_head stay bf16; activations stay bf16/fp32 (weight-only).
 * bs_read_weights returns Q * scale for the quantized matrices. */
#define BS_FLAG_INT8_WEIGHTS 1
/* desc->flags.  BS_FLAG_CLASSIFIER (last stage): the tail of a BLOOM sequence classifier -- the reference's
 * classification task (task_type "classification", Communication.java:532, :596) whose tail sub-model ends in
 * logits that inference::binary_classify reduces to a class (inference.cpp:57-69, :220-270).  The head is HF
 * BloomForSequenceClassification's: ln_f on each row's last position (the pooled token of an unpadded row), then
 * score = Linear(hidden, n_labels, bias=False) -- checkpoint tensor "score.weight" [n_labels][hidden], canonical
 * order after ln_f -- instead of the tied lm_head.  bs_forward's out is an int32 class per row, the FIRST index
 * of the largest logit (binary_classify's strict > scan); logits (BS_STEP_LOGITS) are fp32 [B][n_labels].
 * desc->n_labels in [1, 64] (the reference reads 2).  The stage holds word_embeddings only if it is also first;
 * no head slice, no top-k sampling. */
#define BS_FLAG_CLASSIFIER 2

typedef struct bs_stage_desc {
  /* model (HF BloomConfig fields) */
  int32_t hidden;        /* hidden_size */
  int32_t n_head;        /* n_head */
  int32_t n_layer;       /* n_layer (whole model) */
  int32_t vocab;         /* vocab_size */
  float ln_eps;          /* layer_norm_epsilon */
  /* stage = contiguous layer range (server.py:893-905 assignment) */
  int32_t layer_begin;
  int32_t layer_end;     /* exclusive */
  int32_t is_first;      /* owns word_embeddings + word_embeddings_layernorm */
  int32_t is_last;       /* owns ln_f + tied lm_head + token pick */
  /* storage */
  int32_t dtype;         /* BS_DT_BFLOAT16 (weights + KV in bf16) or BS_DT_FLOAT */
  int32_t device;        /* HIP device ordinal */
  int32_t max_batch;     /* KV-cache rows (slots) */
  int32_t max_ctx;       /* positions per KV row */
  int32_t max_tokens;    /* max B*S per bs_forward call (0 -> max_batch*128) */
  /* weights */
  int32_t weight_source; /* bs_weight_source */
  uint64_t seed;         /* BS_WEIGHTS_SYNTHETIC */
  const float *host_weights;  /* BS_WEIGHTS_HOST */
  uint64_t host_weight_count; /* floats in host_weights */
  /* vocabulary-parallel head slice: lm_head rows [head_vocab_begin, head_vocab_end) + ln_f
   * (0, 0 = none).  Used by pipelines that spread the tied lm_head over all stages. */
  int32_t head_vocab_begin;
  int32_t head_vocab_end;
  int32_t flags;         /* BS_FLAG_* (0 = none) */
  int32_t n_labels;      /* BS_FLAG_CLASSIFIER: classes of the score head (else ignored) */
} bs_stage_desc;

typedef struct bs_stage bs_stage;

/* One forward call over B rows x S new tokens.  Every KV row (slot) keeps its own position:
 * the reference keeps core_pool_size samples in flight, each at its own position
 * (Communication.java:418-464, :621-651), so rows of one call may sit at different positions. */
typedef struct bs_step {
  int32_t batch;     /* B rows */
  int32_t seq;       /* S new tokens per row */
  int32_t slot;      /* first KV-cache row used by these B rows */
  int32_t past_len;  /* positions already cached in every row (used when past_lens is NULL) */
  int32_t flags;     /* BS_STEP_* */
  const int32_t *past_lens;  /* host [B]: positions already cached in row slot+b (per-row context
                                lengths, SURVEY.md §8b ctx_lens); NULL = past_len for all rows */
} bs_step;

#define BS_STEP_HOST_IO 1  /* in/out/logits are host pointers (copied in/out, stream-synchronous) */
#define BS_STEP_LOGITS 2   /* last stage also writes fp32 logits [B][vocab] of each row's last position */

/* Create a stage on desc->device: allocates weights, KV cache and workspace in HBM. */
int bs_init_stage(const bs_stage_desc *desc, bs_stage **out);

/* createSession(model_path) (native-lib.cpp:671-678 -> SessionCache, session_cache.h:26-35): create a
 * stage whose weights come from a checkpoint file instead of desc->weight_source.  `path` is a
 * safetensors file or a sharded checkpoint's *.index.json ({"weight_map": {name: shard}}, shards
 * beside it) holding HF BloomModel tensors ("h.<i>.self_attention.query_key_value.weight", ...;
 * a "transformer." prefix is accepted; "lm_head.weight" stands in for a missing
 * "word_embeddings.weight").  The file is memory-mapped and only the stage's own tensors are read;
 * F32/F16/BF16 are accepted and stored in desc->dtype (bf16 from fp32 rounds to nearest even,
 * exactly as BS_WEIGHTS_HOST).  A missing or mis-shaped tensor fails before any allocation. */
int bs_init_stage_file(const bs_stage_desc *desc, const char *path, bs_stage **out);
/* Model dimensions a checkpoint implies (hidden and vocab from word_embeddings, n_layer = 1 + the
 * highest block index); -1 where the file does not say.  Host only, no device needed. */
int bs_weights_file_probe(const char *path, int32_t *hidden, int32_t *n_layer, int32_t *vocab);

/* Stage forward, stream-ordered on `stream` (hipStream_t, NULL = the stage's own stream).
 * One stage is single-producer: its forwards share the stage's workspace, so a caller that moves a
 * stage from one stream to another must order the new stream behind the old one (an event wait);
 * the library then re-writes every row's position on the new stream itself.
 *  in : first stage -> int32 token ids [B][S]; otherwise fp32 hidden [B][S][hidden]
 *  out: last stage  -> int32 token ids [B] (greedy argmax of each row's last position; a BS_FLAG_CLASSIFIER
 *       stage: int32 class ids [B]); otherwise fp32 hidden [B][S][hidden]
 *  logits: fp32 [B][vocab] ([B][n_labels] on a classifier) when step->flags & BS_STEP_LOGITS (last stage
 *       only), else NULL.
 * Appends S positions to KV rows [slot, slot+B): row b's new positions are p_b .. p_b+S-1 with
 * p_b = past_lens[b] (or past_len).  The last stage's token pick is greedy argmax unless
 * bs_set_sampling selected top-k sampling. */
int bs_forward(bs_stage *stage, const bs_step *step, const void *in, void *out, float *logits,
               void *stream);

/* ---- Vocabulary-parallel head (stages with a head slice, or the last stage) ----
 * Argmax keys: uint64 (order(logit) << 32) | (0xFFFFFFFF - vocab_index), where order() maps
 * fp32 monotonically to uint32; the max key is the greedy token (lowest index on ties). */
/* ln_f of each row's last position: hidden fp32 [B][S][hidden] -> xn [B][hidden] in the stage's
 * activation type (bf16 for BS_DT_BFLOAT16 stages, fp32 otherwise). */
int bs_head_norm(bs_stage *stage, const float *hidden, int32_t batch, int32_t seq, void *xn, void *stream);
/* Logits of the stage's vocabulary slice for xn [B][hidden]; writes per-row keys
 * max(keys_in[b], slice max) to keys_out (either may be NULL) and, when tokens is non-NULL,
 * the decoded token ids.  keys_out may equal keys_in (the merge is per row, in place).  Device pointers,
 * stream ordered. */
int bs_head_slice(bs_stage *stage, const void *xn, int32_t batch, const uint64_t *keys_in, uint64_t *keys_out,
                  int32_t *tokens, void *stream);

/* ---- Tail token pick (last stage) ----
 * top_k <= 1: greedy argmax (the default; lowest index on ties, like torch.argmax).
 * 2 <= top_k <= 16: seeded top-k sampling restating decoding::StaticDecoding (decoding.cpp:24-66):
 *   the top_k (logit, index) pairs of each row's last position in std::greater order (larger logit
 *   first, the HIGHER index first on equal logits: decoding.cpp:44-45), weights
 *   w_i = exp((l_i - l_0) / temperature) -- with temperature 1 exactly the reference's "normalise
 *   the top-k probabilities by their sum" (:56-57) applied to softmax probabilities -- and the pick
 *   = the first i whose running sum of w exceeds u * sum(w), u in [0, 1) from the stage's counter
 *   generator keyed by (seed, KV row, position): reproducible, unlike the reference's
 *   std::random_device seed (:61-63).  The reference never applies its temperature argument
 *   (:51-52); pass 1 to reproduce it.  Not available on vocabulary-slice (bs_head_slice) stages.
 *   The draw depends on nothing else: two requests decoded with the same seed in the same KV row
 *   draw the same u at each position, so a server gives every request its own seed (for example
 *   base_seed ^ request_id, set before the request's first sampled step). */
int bs_set_sampling(bs_stage *stage, int32_t top_k, float temperature, uint64_t seed);

/* Decode steps (S = 1) on device buffers are captured once per shape into a hipGraph and replayed
 * (the default, on = 1); on = 0 launches them eagerly every step (same kernels, same results: for
 * debugging and A/B timing).  Drops captured graphs.  Returns BS_OK.  A stage starts with graphs off
 * when the environment holds BS_GRAPHS=0 at bs_init_stage (rocprofv3 --pmc runs). */
int bs_set_graphs(bs_stage *stage, int32_t on);

/* Forget the cached positions of one KV row (slot), or of all rows when slot < 0. */
int bs_reset_kv(bs_stage *stage, int32_t slot);
/* Read back KV row `slot` of the stage's local layer `layer`, positions [pos0, pos0 + npos), as fp32
 * out[2 (K, V)][n_head][npos][head_dim].  Synchronizes the stage's own stream; the caller orders any
 * other stream it forwarded on.  For verification (parity tests hand a device cache to the checker). */
int bs_read_kv(const bs_stage *stage, int32_t layer, int32_t slot, int32_t pos0, int32_t npos, float *out);

void bs_release(bs_stage *stage);

const char *bs_last_error(void);

/* Introspection */
int bs_stage_info(const bs_stage *stage, bs_stage_desc *out_desc, uint64_t *weight_bytes,
                  uint64_t *kv_bytes, uint64_t *workspace_bytes);
/* fp32 count for BS_WEIGHTS_HOST.  Canonical order: [word_embeddings if first, or last and not a classifier]
 * [emb LN g,b if first]{per layer: ln1 g,b, qkv w,b, dense w,b, ln2 g,b, fc1 w,b, fc2 w,b}
 * [ln_f g,b if last][score [n_labels][hidden] if a classifier]
 * [head slice rows if a slice is set and the stage is neither first nor last]
 * [ln_f g,b if a slice is set and the stage is not last]. */
uint64_t bs_stage_weight_count(const bs_stage_desc *desc);
int bs_abi_version(void);
/* Build provenance: hex SHA-256 of the library's sources (csrc files and include/bloomstage.h) stamped at
 * compile time; the Python binding refuses a library whose stamp differs from the sources beside it. */
const char *bs_build_id(void);
/* Read back `count` weights starting at element `offset` of the canonical stage order
 * (the BS_WEIGHTS_HOST layout) as fp32.  For verification of loaded/generated weights. */
int bs_read_weights(const bs_stage *stage, uint64_t offset, uint64_t count, float *out);
/* Synthetic prompt ids of the repo generator (DESIGN.md "Synthetic weights"): ids[i] for the
 * flat index i of a [B][S] prompt, uniform over [0, vocab). */
int bs_prompt_ids(uint64_t seed, int32_t n, int32_t vocab, int32_t *out);

/* Profiling: time every launch of one kernel class with HIP events on the stage stream.
 * kernel_class: 0 off, 1 weight GEMV (decode), 2 GEMM (prefill), 3 attention.
 * bs_profile_read returns accumulated milliseconds, launch count and algorithmic bytes
 * (or flops for class 2) since the last bs_profile_enable; it synchronizes the stream. */
int bs_profile_enable(bs_stage *stage, int32_t kernel_class);
int bs_profile_read(bs_stage *stage, double *total_ms, uint64_t *launches, double *algo_units);
/* Enqueue a one-thread spin of `microseconds` (<= 100000) on `stream` (hipStream_t; NULL = the
 * default stream of the current device): lets the host enqueue a whole profiled step behind it,
 * so event-timed launches are not stretched by host submission gaps. */
int bs_stream_delay(void *stream, int32_t microseconds);

/* Measurement aid (bench.py "hbm_measured"): STREAM-like HBM rates of a device, best of 10 runs over
 * `bytes` (a multiple of 1 MiB) -- read: non-temporal 16-B loads; copy: read + write bytes / time. */
int bs_hbm_probe(int32_t device, uint64_t bytes, double *read_gbps, double *copy_gbps);
/* Measurement aid (bench.py "mfma_measured"): dense bf16 matrix-core TFLOP/s of a device, best of 5 runs of
 * register-operand v_mfma_f32_32x32x16_bf16 / v_mfma_f32_16x16x32_bf16 chains (8 independent chains per wave,
 * 8 waves per CU, no memory traffic).  The measured counterpart of the vendor dense peak. */
int bs_mfma_probe(int32_t device, double *tflops_32x32x16, double *tflops_16x16x32);

/* ---- Reference wire codec (utils.cpp:124-368): size_t n; per tensor {int32 dtype,
 * size_t ndim, int64 dims[ndim], raw little-endian data}. size_t is 8 bytes (LP64). ---- */
#define BS_CODEC_MAX_DIMS 8
typedef struct bs_tensor_view {
  int32_t dtype;                     /* bs_dtype */
  int32_t ndim;
  int64_t dims[BS_CODEC_MAX_DIMS];
  const void *data;                  /* may be unaligned when it points into a wire buffer */
} bs_tensor_view;

/* Serialize n tensors. Returns the total byte count (also when out is NULL or too small:
 * then nothing is written) or a negative bs_status. */
int64_t bs_codec_serialize(const bs_tensor_view *tensors, int32_t n, void *out, uint64_t out_cap);
/* Parse a wire buffer into zero-copy views. *n_out receives the tensor count; at most
 * max_views are filled. Returns BS_OK or a negative bs_status (truncated / unsupported). */
int bs_codec_deserialize(const void *bytes, uint64_t len, bs_tensor_view *views, int32_t max_views,
                         int32_t *n_out);
int64_t bs_dtype_size(int32_t dtype);
/* binaryClassify(byte[]) (native-lib.cpp:128-160): the first tensor of a wire buffer holds logits; *cls = the
 * first index of the larger of its first two floats (inference::binary_classify, inference.cpp:57-69).  Host
 * only.  BS_ERR_INVALID for an unparsable buffer, no tensor, a non-float tensor or fewer than two elements
 * (the reference returns -1 / -2 there, or reads past a short tensor). */
int bs_binary_classify(const void *bytes, uint64_t len, int32_t *cls);
/* 4-byte native (little-endian) int, as the tail stage returns a token id. */
void bs_serialize_int(int32_t value, uint8_t out[4]);
int bs_deserialize_int(const uint8_t *bytes, uint64_t len, int32_t *value);

#ifdef __cplusplus
}
#endif
#endif /* BLOOMSTAGE_H */
