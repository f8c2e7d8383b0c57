/*
 * oracle/bloom_oracle.c — TEST INFRASTRUCTURE: CPU restatement of one BLOOM pipeline
 * stage forward.  Used only as the checker by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  Never linked into or called by the product path.
 *
 * What it restates:
 *   The reference runs one ONNX sub-model per stage through ORT
 *   (inference.cpp:145-218, Session::Run :207-215).  The arithmetic inside those ONNX
 *   modules is HF BLOOM (the modules are exported from it by the absent util.model_card),
 *   so the math below follows transformers' modeling_bloom.py:
 *     - ALiBi slopes / positions  build_alibi_tensor (modeling_bloom.py:43-89)
 *     - tanh-GELU                 bloom_gelu_forward (:111-121)
 *     - attention                 BloomAttention.forward (:245-310): interleaved fused QKV
 *                                 [heads,3,hd], scores = alibi + q.k/sqrt(hd), causal
 *                                 mask, fp32 softmax, context, dense + bias, + residual
 *     - MLP                       BloomMLP.forward (:325-340)
 *     - block residual order      BloomBlock.forward (:359-403), residual = pre-LN input
 *     - embedding + emb LN, ln_f  BloomModel.forward (:448-536); tied lm_head (:561-566)
 *   The tail token pick is greedy argmax (first maximal index, like torch.argmax) instead
 *   of the reference's non-deterministic top-k sampler (decoding.cpp:24-66); see
 *   DESIGN.md "Token pick".
 *
 * Stage semantics = bs_forward() in include/bloomstage.h: first stage takes int32 ids
 * [B,S], others fp32 hidden [B,S,h]; last stage emits int32 ids [B] (+ optional fp32
 * logits [B,V] of the last position), others fp32 hidden [B,S,h].  KV cache rows
 * [slot, slot+B) hold positions [0, past_len) on entry; S new positions are appended.
 *
 * bf16 mode emulates the device path's storage roundings exactly (weights, LN outputs
 * feeding GEMMs, q, K/V cache, attention context, GELU output) while accumulating in fp32,
 * so GPU-vs-oracle differences are accumulation-order only.
 *
 * Parity pinning: checked against transformers' BloomForCausalLM on CPU fp32 with the
 * same generated weights (tests/golden/make_golden.py -> tests/golden/ fixtures,
 * tests/test_oracle_golden.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#include "gen.h"

typedef struct {
  float *ln1_g, *ln1_b, *qkv_w, *qkv_b, *dense_w, *dense_b;
  float *ln2_g, *ln2_b, *fc1_w, *fc1_b, *fc2_w, *fc2_b;
} or_layer;

typedef struct or_stage {
  int h, nh, hd, nl, V;
  float eps;
  int lb, le, first, last, bf16;
  int max_batch, max_ctx;
  float *wemb, *emb_g, *emb_b, *lnf_g, *lnf_b;
  int n_labels;   /* > 0: sequence-classification tail (or_set_classifier) */
  float *score;   /* [n_labels][h] */
  or_layer *layers;
  float *kv;      /* [L_s][2][max_batch][nh][max_ctx][hd] */
  float *slopes;  /* [nh] */
} or_stage;

/* ---- ALiBi slopes, restating build_alibi_tensor (modeling_bloom.py:60-78) ---- */
void or_alibi_slopes(int n_head, float *out) {
  int cp2 = 1;
  while (cp2 * 2 <= n_head) cp2 *= 2;
  double base = pow(2.0, -pow(2.0, -(log2((double)cp2) - 3.0)));
  float basef = (float)base;
  for (int i = 0; i < cp2; i++) out[i] = (float)pow((double)basef, (double)(i + 1));
  if (cp2 != n_head) {
    double eb = pow(2.0, -pow(2.0, -(log2((double)(2 * cp2)) - 3.0)));
    float ebf = (float)eb;
    int rem = n_head - cp2 < cp2 ? n_head - cp2 : cp2;
    for (int i = 0; i < rem; i++) out[cp2 + i] = (float)pow((double)ebf, (double)(2 * i + 1));
  }
}

static float *gen_tensor(uint64_t seed, int layer, int tid, size_t n, int kind, int bf16) {
  float *p = (float *)malloc(n * sizeof(float));
  uint64_t key = gen_tensor_key(seed, layer, (uint32_t)tid);
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < n; i++) {
    float v = gen_value(kind, key, (uint32_t)i);
    p[i] = bf16 ? gen_bf16_round(v) : v;
  }
  return p;
}

/* exported for the generator-agreement tests */
void or_gen_tensor(uint64_t seed, int layer, int tid, uint64_t n, float *out) {
  int kind = layer < 0 ? gen_model_kind(tid) : gen_layer_kind(tid);
  uint64_t key = gen_tensor_key(seed, layer, (uint32_t)tid);
  for (uint64_t i = 0; i < n; i++) out[i] = gen_value(kind, key, (uint32_t)i);
}

void or_prompt_ids(uint64_t seed, int n, int vocab, int32_t *out) {
  for (int i = 0; i < n; i++) out[i] = (int32_t)gen_prompt_id(seed, (uint32_t)i, (uint32_t)vocab);
}

void or_destroy(or_stage *s);

or_stage *or_create(int hidden, int n_head, int n_layer, int vocab, float eps, int layer_begin,
                    int layer_end, int is_first, int is_last, int bf16, int max_batch, int max_ctx,
                    uint64_t seed) {
  if (hidden <= 0 || n_head <= 0 || hidden % n_head || layer_begin < 0 || layer_end > n_layer ||
      layer_begin > layer_end || max_batch <= 0 || max_ctx <= 0)
    return NULL;
  or_stage *s = (or_stage *)calloc(1, sizeof(or_stage));
  s->h = hidden; s->nh = n_head; s->hd = hidden / n_head; s->nl = n_layer; s->V = vocab;
  s->eps = eps; s->lb = layer_begin; s->le = layer_end; s->first = is_first; s->last = is_last;
  s->bf16 = bf16; s->max_batch = max_batch; s->max_ctx = max_ctx;
  size_t h = (size_t)hidden;
  if (is_first || is_last) s->wemb = gen_tensor(seed, -1, GT_WEMB, (size_t)vocab * h, 0, bf16);
  if (is_first) {
    s->emb_g = gen_tensor(seed, -1, GT_EMB_G, h, 2, bf16);
    s->emb_b = gen_tensor(seed, -1, GT_EMB_B, h, 3, bf16);
  }
  if (is_last) {
    s->lnf_g = gen_tensor(seed, -1, GT_LNF_G, h, 2, bf16);
    s->lnf_b = gen_tensor(seed, -1, GT_LNF_B, h, 3, bf16);
  }
  int L = layer_end - layer_begin;
  s->layers = (or_layer *)calloc(L > 0 ? L : 1, sizeof(or_layer));
  for (int i = 0; i < L; i++) {
    int l = layer_begin + i;
    or_layer *w = &s->layers[i];
    size_t sz[GT_NUM_LAYER_TENSORS] = {h, h, 3 * h * h, 3 * h, h * h, h, h, h, 4 * h * h, 4 * h, 4 * h * h, h};
    float **dst[GT_NUM_LAYER_TENSORS] = {&w->ln1_g, &w->ln1_b, &w->qkv_w, &w->qkv_b, &w->dense_w, &w->dense_b,
                                         &w->ln2_g, &w->ln2_b, &w->fc1_w, &w->fc1_b, &w->fc2_w, &w->fc2_b};
    for (int t = 0; t < GT_NUM_LAYER_TENSORS; t++)
      *dst[t] = gen_tensor(seed, l, t, sz[t], gen_layer_kind(t), bf16);
  }
  size_t kvn = (size_t)(L > 0 ? L : 1) * 2 * max_batch * n_head * max_ctx * s->hd;
  s->kv = (float *)calloc(kvn, sizeof(float));
  s->slopes = (float *)malloc(sizeof(float) * n_head);
  or_alibi_slopes(n_head, s->slopes);
  if (!s->kv) { or_destroy(s); return NULL; }
  return s;
}

/* Sequence-classification tail (include/bloomstage.h BS_FLAG_CLASSIFIER): the last stage's head becomes
 * score [n_labels][h] (generator tensor GT_SCORE, model level), HF BloomForSequenceClassification's
 * `score = nn.Linear(hidden, num_labels, bias=False)`; the reference runs such a tail through
 * run_inference_with_binary_classification (inference.cpp:220-270) behind
 * runInferenceWorkerResidualLastClassification (native-lib.cpp:1305-1366).  Needs is_last. */
int or_set_classifier(or_stage *s, int n_labels, uint64_t seed) {
  if (!s || !s->last || n_labels < 1) return -1;
  free(s->score);
  s->score = gen_tensor(seed, -1, GT_SCORE, (size_t)n_labels * s->h, 0, s->bf16);
  s->n_labels = n_labels;
  return 0;
}

/* ---- Weight-only int8 (the reference's bloom*-int8 variants, server.py:796-799; the rule is
 * include/bloomstage.h BS_FLAG_INT8_WEIGHTS, whose device side is kernels.hip
 * quantize_rows_kernel).  The reference's int8 ONNX files come from the absent model_card export
 * (ORT quantization), so this scheme is the build's own and its parity is against this
 * restatement only ("parity unpinned" against the reference).  Per output row n of the four
 * block matrices: scale = max|W[n][:]| / 127 (1 for a zero row), Q = rint(W / scale) clamped to
 * [-127, 127]; the matrix is replaced by Q * scale (fp32).  Call on a bf16-mode stage. */
static void quantize_rows(float *W, size_t N, size_t K) {
#pragma omp parallel for schedule(static)
  for (size_t n = 0; n < N; n++) {
    float *w = W + n * K;
    float amax = 0.f;
    for (size_t k = 0; k < K; k++) amax = fmaxf(amax, fabsf(w[k]));
    const float sc = amax > 0.f ? amax / 127.f : 1.f;
    for (size_t k = 0; k < K; k++) {
      float q = rintf(w[k] / sc);
      q = fminf(fmaxf(q, -127.f), 127.f);
      w[k] = q * sc;
    }
  }
}

int or_quantize_int8(or_stage *s) {
  if (!s || !s->bf16) return -1;
  const size_t h = (size_t)s->h;
  for (int i = 0; i < s->le - s->lb; i++) {
    or_layer *w = &s->layers[i];
    quantize_rows(w->qkv_w, 3 * h, h);
    quantize_rows(w->dense_w, h, h);
    quantize_rows(w->fc1_w, 4 * h, h);
    quantize_rows(w->fc2_w, h, 4 * h);
  }
  return 0;
}

void or_destroy(or_stage *s) {
  if (!s) return;
  free(s->wemb); free(s->emb_g); free(s->emb_b); free(s->lnf_g); free(s->lnf_b); free(s->score);
  int L = s->le - s->lb;
  for (int i = 0; i < L; i++) {
    or_layer *w = &s->layers[i];
    free(w->ln1_g); free(w->ln1_b); free(w->qkv_w); free(w->qkv_b); free(w->dense_w); free(w->dense_b);
    free(w->ln2_g); free(w->ln2_b); free(w->fc1_w); free(w->fc1_b); free(w->fc2_w); free(w->fc2_b);
  }
  free(s->layers); free(s->kv); free(s->slopes); free(s);
}

static inline float rb(const or_stage *s, float v) { return s->bf16 ? gen_bf16_round(v) : v; }
/* v rounded to the nearest fp16 value (ties to even), as a float: 11 significant bits, subnormals below
 * 2^-14 in steps of 2^-24, |v| >= 65520 -> inf (what the device's float -> _Float16 conversion does) */
static inline float rf16(float v) {
  const float a = fabsf(v);
  if (a != a) return v;
  if (a >= 65520.f) return copysignf(INFINITY, v);
  float q;
  if (a < 6.103515625e-05f) {
    q = 5.9604644775390625e-08f;
  } else {
    int e;
    frexpf(a, &e);
    q = ldexpf(1.f, e - 11);
  }
  return copysignf(rintf(a / q) * q, v);
}
void or_round_fp16(const float *in, float *out, uint64_t n) { for (uint64_t i = 0; i < n; i++) out[i] = rf16(in[i]); }

/* test knob: dot-product accumulation order.  0: 16 fp32 lanes + a tree (default), 1: double,
 * 2: one sequential fp32 accumulator, 3: fp32 sums of 32-element chunks added in order (the K-step
 * grouping of the device's MFMA GEMMs).  Modes 0, 2 and 3 are three correct fp32 orders of the same
 * rounded math; their spread against mode 1 is the format's own noise (tools/parity_study.py). */
static int g_accum_mode = 0;
void or_set_accum_double(int on) { g_accum_mode = on ? 1 : 0; }
void or_set_accum_mode(int mode) { g_accum_mode = mode; }
/* test knob (bit mask) for the P.V product of the attention, emulating device roundings the bf16 mode does
 * not model: 1 = V rounded to fp16 (|V| > 65504 -> inf), 2 = P = fp16(p) + fp16(p - fp16(p)), 4 = P =
 * bf16(p) + bf16(p - bf16(p)); with any bit set P is exp(s - max) unnormalised and the context is divided
 * by the sum after the product (the device's order).  8 = the roundings of bits 1/2/4 apply to S > 1 calls
 * only (the prefill kernel, attn_prefill.hip); S = 1 calls keep fp32 P, unnormalised, divided after (the
 * decode kernel's order, kernels.hip attn_decode_block).  4 | 8 models the bf16 device library.
 * 0: the HF order (normalised p, fp32). */
static int g_emul_pv = 0;
void or_set_emul_pv(int mask) { g_emul_pv = mask; }
/* diagnostic knob: bits of bf16 rounding points to SKIP (1 LN out, 2 K/V, 4 q, 8 ctx, 16 GELU out) */
static int g_skip_round = 0;
void or_set_skip_round(int mask) { g_skip_round = mask; }
static inline float rbp(const or_stage *s, int point, float v) { return (g_skip_round & point) ? v : rb(s, v); }

static float dotf(const float *a, const float *b, int K) {
  if (g_accum_mode == 1) {
    double d = 0.0;
    for (int k = 0; k < K; k++) d += (double)a[k] * (double)b[k];
    return (float)d;
  }
  if (g_accum_mode == 2) {
    float t = 0.f;
    for (int k = 0; k < K; k++) t += a[k] * b[k];
    return t;
  }
  if (g_accum_mode == 3) {
    float t = 0.f;
    for (int k0 = 0; k0 < K; k0 += 32) {
      float c = 0.f;
      for (int k = k0; k < K && k < k0 + 32; k++) c += a[k] * b[k];
      t += c;
    }
    return t;
  }
  float acc[16] = {0};
  int k = 0;
  for (; k + 16 <= K; k += 16)
    for (int j = 0; j < 16; j++) acc[j] += a[k + j] * b[k + j];
  float t = 0.f;
  for (; k < K; k++) t += a[k] * b[k];
  for (int w = 8; w >= 1; w >>= 1)
    for (int j = 0; j < w; j++) acc[j] += acc[j + w];
  return acc[0] + t;
}

/* LayerNorm over rows, HF nn.LayerNorm semantics (biased variance, eps inside sqrt). */
static void layernorm(const float *x, float *y, int M, int K, const float *g, const float *b, float eps,
                      int round_out, const or_stage *s) {
#pragma omp parallel for schedule(static)
  for (int m = 0; m < M; m++) {
    const float *xr = x + (size_t)m * K;
    double mean = 0, var = 0;
    for (int k = 0; k < K; k++) mean += xr[k];
    mean /= K;
    for (int k = 0; k < K; k++) { double d = xr[k] - mean; var += d * d; }
    var /= K;
    float rstd = (float)(1.0 / sqrt(var + (double)eps));
    float mf = (float)mean;
    for (int k = 0; k < K; k++) {
      float v = (xr[k] - mf) * rstd * g[k] + b[k];
      y[(size_t)m * K + k] = round_out ? rbp(s, 1, v) : v;
    }
  }
}

/* y[m][n] = x[m].W[n] + bias[n]  (nn.Linear with weight [out][in]) */
static void linear(const float *x, const float *W, const float *bias, float *y, int M, int N, int K) {
#pragma omp parallel for schedule(static)
  for (int n = 0; n < N; n++) {
    const float *wr = W + (size_t)n * K;
    for (int m = 0; m < M; m++) {
      float v = dotf(x + (size_t)m * K, wr, K);
      y[(size_t)m * N + n] = bias ? v + bias[n] : v;
    }
  }
}

static inline float gelu_bloom(float x) {
  /* bloom_gelu_forward (modeling_bloom.py:111-121), same evaluation order */
  return x * 0.5f * (1.0f + tanhf(0.79788456f * x * (1.0f + 0.044715f * x * x)));
}

static float *kv_ptr(const or_stage *s, int li, int which, int row, int head, int pos) {
  size_t idx = ((((size_t)li * 2 + which) * s->max_batch + row) * s->nh + head);
  return s->kv + (idx * s->max_ctx + pos) * s->hd;
}

int or_forward(or_stage *s, int B, int S, int slot, int past_len, const void *in, void *out, float *logits) {
  if (B <= 0 || S <= 0 || slot < 0 || slot + B > s->max_batch || past_len < 0 || past_len + S > s->max_ctx)
    return -1;
  const int h = s->h, nh = s->nh, hd = s->hd, M = B * S;
  float *x = (float *)malloc(sizeof(float) * M * h);
  float *xn = (float *)malloc(sizeof(float) * M * h);
  float *a = (float *)malloc(sizeof(float) * M * h);
  float *ctx = (float *)malloc(sizeof(float) * M * h);
  float *qkv = (float *)malloc(sizeof(float) * M * 3 * h);
  float *g = (float *)malloc(sizeof(float) * (size_t)M * 4 * h);

  if (s->first) {
    const int32_t *ids = (const int32_t *)in;
    for (int m = 0; m < M; m++) {
      int id = ids[m];
      if (id < 0 || id >= s->V) { free(x); free(xn); free(a); free(ctx); free(qkv); free(g); return -2; }
      memcpy(x + (size_t)m * h, s->wemb + (size_t)id * h, sizeof(float) * h);
    }
    layernorm(x, x, M, h, s->emb_g, s->emb_b, s->eps, 0, s);
  } else {
    memcpy(x, in, sizeof(float) * M * h);
  }

  const float inv_norm = 1.0f / sqrtf((float)hd);
  int L = s->le - s->lb;
  for (int li = 0; li < L; li++) {
    or_layer *w = &s->layers[li];
    layernorm(x, xn, M, h, w->ln1_g, w->ln1_b, s->eps, 1, s);
    linear(xn, w->qkv_w, w->qkv_b, qkv, M, 3 * h, h);
    /* fused qkv is [heads][3][hd] per token (modeling_bloom.py _reshape) */
    for (int m = 0; m < M; m++) {
      int b = m / S, t = m % S, pos = past_len + t;
      for (int hh = 0; hh < nh; hh++) {
        const float *base = qkv + (size_t)m * 3 * h + (size_t)hh * 3 * hd;
        float *kd = kv_ptr(s, li, 0, slot + b, hh, pos), *vd = kv_ptr(s, li, 1, slot + b, hh, pos);
        for (int d = 0; d < hd; d++) { kd[d] = rbp(s, 2, base[hd + d]); vd[d] = rbp(s, 2, base[2 * hd + d]); }
      }
    }
#pragma omp parallel for collapse(2) schedule(dynamic)
    for (int b = 0; b < B; b++)
      for (int hh = 0; hh < nh; hh++) {
        int nk_max = past_len + S;
        float *sc = (float *)malloc(sizeof(float) * nk_max);
        for (int t = 0; t < S; t++) {
          int m = b * S + t, nk = past_len + t + 1; /* causal: keys 0..pos */
          const float *q0 = qkv + (size_t)m * 3 * h + (size_t)hh * 3 * hd;
          float q[256];  /* the device stores q in the activation dtype (bf16 mode: rounded) */
          for (int d = 0; d < hd; d++) q[d] = rbp(s, 4, q0[d]);
          float mx = -INFINITY;
          for (int j = 0; j < nk; j++) {
            float qk = dotf(q, kv_ptr(s, li, 0, slot + b, hh, j), hd);
            float v = s->slopes[hh] * (float)j + inv_norm * qk; /* alibi.baddbmm(beta=1, alpha=inv_norm) */
            sc[j] = v;
            if (v > mx) mx = v;
          }
          float sum = 0.f;
          for (int j = 0; j < nk; j++) { sc[j] = expf(sc[j] - mx); sum += sc[j]; }
          float inv = 1.0f / sum;
          float *o = ctx + (size_t)m * h + (size_t)hh * hd;
          for (int d = 0; d < hd; d++) o[d] = 0.f;
          const int emul = ((g_emul_pv & 8) && S == 1) ? 8 : g_emul_pv;
          if (emul) {
            for (int j = 0; j < nk; j++) {
              const float *vr = kv_ptr(s, li, 1, slot + b, hh, j);
              float e = sc[j], hi = e, lo = 0.f;
              if (emul & 2) { hi = rf16(e); lo = rf16(e - hi); }
              else if (emul & 4) { hi = gen_bf16_round(e); lo = gen_bf16_round(e - hi); }
              for (int d = 0; d < hd; d++) {
                float v = (emul & 1) ? rf16(vr[d]) : vr[d];
                o[d] += hi * v + lo * v;
              }
            }
            for (int d = 0; d < hd; d++) o[d] *= inv;
          } else {
            for (int j = 0; j < nk; j++) {
              const float *vr = kv_ptr(s, li, 1, slot + b, hh, j);
              float p = sc[j] * inv;
              for (int d = 0; d < hd; d++) o[d] += p * vr[d];
            }
          }
          for (int d = 0; d < hd; d++) o[d] = rbp(s, 8, o[d]);
        }
        free(sc);
      }
    /* a = x + dense(ctx) */
    linear(ctx, w->dense_w, w->dense_b, a, M, h, h);
    for (size_t i = 0; i < (size_t)M * h; i++) a[i] = a[i] + x[i];
    layernorm(a, xn, M, h, w->ln2_g, w->ln2_b, s->eps, 1, s);
    linear(xn, w->fc1_w, w->fc1_b, g, M, 4 * h, h);
    for (size_t i = 0; i < (size_t)M * 4 * h; i++) g[i] = rbp(s, 16, gelu_bloom(g[i]));
    linear(g, w->fc2_w, w->fc2_b, x, M, h, 4 * h);
    for (size_t i = 0; i < (size_t)M * h; i++) x[i] = x[i] + a[i];
  }

  if (s->last && s->n_labels > 0) {
    /* sequence-classification tail: ln_f on each row's last position (the pooled token of
     * BloomForSequenceClassification.forward for an unpadded row), score (no bias), and the first index of the
     * largest logit (inference.cpp:57-69 binary_classify: a strict > scan keeps the first maximum) */
    for (int b = 0; b < B; b++)
      memcpy(a + (size_t)b * h, x + ((size_t)b * S + S - 1) * h, sizeof(float) * h);
    layernorm(a, xn, B, h, s->lnf_g, s->lnf_b, s->eps, 1, s);
    const int nl = s->n_labels;
    float *lg = logits ? logits : (float *)malloc(sizeof(float) * (size_t)B * nl);
    linear(xn, s->score, NULL, lg, B, nl, h);
    int32_t *cls = (int32_t *)out;
    for (int b = 0; b < B; b++) {
      const float *r = lg + (size_t)b * nl;
      int best = 0;
      for (int c = 1; c < nl; c++) if (r[c] > r[best]) best = c;
      cls[b] = best;
    }
    if (!logits) free(lg);
  } else if (s->last) {
    /* ln_f on the last position of each row, tied lm_head, argmax */
    for (int b = 0; b < B; b++)
      memcpy(a + (size_t)b * h, x + ((size_t)b * S + S - 1) * h, sizeof(float) * h);
    layernorm(a, xn, B, h, s->lnf_g, s->lnf_b, s->eps, 1, s);
    float *lg = logits ? logits : (float *)malloc(sizeof(float) * (size_t)B * s->V);
    linear(xn, s->wemb, NULL, lg, B, s->V, h);
    int32_t *tok = (int32_t *)out;
    for (int b = 0; b < B; b++) {
      const float *r = lg + (size_t)b * s->V;
      int best = 0;
      for (int v = 1; v < s->V; v++) if (r[v] > r[best]) best = v;
      tok[b] = best;
    }
    if (!logits) free(lg);
  } else {
    memcpy(out, x, sizeof(float) * M * h);
  }
  free(x); free(xn); free(a); free(ctx); free(qkv); free(g);
  return 0;
}

/* Vocabulary-parallel head, restating the tail of the forward above for a vocab slice:
 * xn[b] = ln_f(hidden[b][S-1]) (bf16-rounded in bf16 mode); keys = max over the slice rows
 * [v0, v1) of (order(logit) << 32 | (0xFFFFFFFF - v)), merged with keys_in. */
int or_head_norm(or_stage *s, const float *hidden, int B, int S, float *xn) {
  if (!s->lnf_g || !s->wemb) return -1;
  float *rows = (float *)malloc(sizeof(float) * (size_t)B * s->h);
  for (int b = 0; b < B; b++) memcpy(rows + (size_t)b * s->h, hidden + ((size_t)b * S + S - 1) * s->h, sizeof(float) * s->h);
  layernorm(rows, xn, B, s->h, s->lnf_g, s->lnf_b, s->eps, 1, s);
  free(rows);
  return 0;
}

static uint64_t order_key(float f, uint32_t v) {
  union { float f; uint32_t u; } x; x.f = f;
  uint32_t k = (x.u & 0x80000000u) ? ~x.u : (x.u | 0x80000000u);
  return ((uint64_t)k << 32) | (0xFFFFFFFFu - v);
}

int or_head_slice(or_stage *s, const float *xn, int B, int v0, int v1, const uint64_t *keys_in, uint64_t *keys_out,
                  int32_t *tokens) {
  if (!s->wemb || v0 < 0 || v1 > s->V || v0 >= v1) return -1;
  int n = v1 - v0;
  float *lg = (float *)malloc(sizeof(float) * (size_t)B * n);
  linear(xn, s->wemb + (size_t)v0 * s->h, NULL, lg, B, n, s->h);
  for (int b = 0; b < B; b++) {
    uint64_t best = keys_in ? keys_in[b] : 0;
    for (int v = 0; v < n; v++) {
      uint64_t k = order_key(lg[(size_t)b * n + v], (uint32_t)(v0 + v));
      if (k > best) best = k;
    }
    if (keys_out) keys_out[b] = best;
    if (tokens) tokens[b] = (int32_t)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFu));
  }
  free(lg);
  return 0;
}

/* Copy of one KV row for tests: which 0=K 1=V, layer index local to the stage. */
int or_read_kv(const or_stage *s, int li, int which, int row, int head, int pos, float *out) {
  if (li < 0 || li >= s->le - s->lb) return -1;
  memcpy(out, kv_ptr(s, li, which, row, head, pos), sizeof(float) * s->hd);
  return 0;
}

/* Test infrastructure: overwrite KV row `row` of local layer li, positions [pos0, pos0+npos), from
 * in[2 (K, V)][nh][npos][hd] (a device cache read back through bs_read_kv), so a decode step at a long
 * context can be checked without the checker recomputing every earlier position. */
int or_write_kv(or_stage *s, int li, int row, int pos0, int npos, const float *in) {
  if (li < 0 || li >= s->le - s->lb || row < 0 || row >= s->max_batch || pos0 < 0 || npos < 0 ||
      pos0 + npos > s->max_ctx)
    return -1;
  for (int w = 0; w < 2; w++)
    for (int hh = 0; hh < s->nh; hh++)
      memcpy(kv_ptr(s, li, w, row, hh, pos0), in + ((size_t)(w * s->nh + hh) * npos) * s->hd,
             sizeof(float) * (size_t)npos * s->hd);
  return 0;
}

int or_num_threads(void) { return omp_get_max_threads(); }
