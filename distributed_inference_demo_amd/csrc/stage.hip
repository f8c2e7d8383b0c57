// stage.hip — libbloomstage C-ABI (include/bloomstage.h): stage lifetime + forward orchestration.
//
// Replaces the reference's per-device stage execution:
//   SessionCache / createSession (session_cache.h:20-35, native-lib.cpp:663-678)  -> bs_init_stage
//   run_inference + JNI wrappers (inference.cpp:145-218, native-lib.cpp:942-1443)  -> bs_forward
//   releaseSession (native-lib.cpp:1290-1303)                                       -> bs_release
// Everything the ONNX sub-model computed on the CPU is here a sequence of gfx950 kernels
// (kernels.hip) over weights, KV cache and workspace resident in the stage GPU's HBM.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bloomstage.h"
#include "common.h"
#include "kernels.h"
#include "safetensors.h"

static thread_local std::string g_err;

// BS_TRACE_CALLS=1: one stderr line (flushed) before each HIP runtime call bs_forward makes, so a host fault inside
// the runtime names the call it happened in (the round-5 SIGSEGV under rocprofv3).
static bool trace_calls() {
  static const bool on = [] { const char* e = getenv("BS_TRACE_CALLS"); return e && e[0] == '1'; }();
  return on;
}
#define BS_TRACE(...)                                         \
  do {                                                        \
    if (trace_calls()) {                                      \
      fprintf(stderr, "[bs_forward] " __VA_ARGS__);           \
      fputc('\n', stderr);                                    \
      fflush(stderr);                                         \
    }                                                         \
  } while (0)

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return fail(BS_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));        \
  } while (0)

namespace {

enum { T_LN1_G, T_LN1_B, T_QKV_W, T_QKV_B, T_DENSE_W, T_DENSE_B, T_LN2_G, T_LN2_B, T_FC1_W, T_FC1_B,
       T_FC2_W, T_FC2_B, T_NLAYER };
enum { M_WEMB = 0, M_EMB_G = 1, M_EMB_B = 2, M_LNF_G = 3, M_LNF_B = 4, M_SCORE = 5 };

struct Layer {
  void* t[T_NLAYER];
  float* sc[T_NLAYER];  // int8 stages: per-row scales of the four weight matrices (else null)
};

static bool is_matrix(int t) { return t == T_QKV_W || t == T_DENSE_W || t == T_FC1_W || t == T_FC2_W; }

struct GraphKey {
  int B, slot, flags;
  const void* in;
  void* out;
  float* logits;
  hipStream_t st;
  bool operator==(const GraphKey& o) const {
    return B == o.B && slot == o.slot && flags == o.flags && in == o.in && out == o.out && logits == o.logits &&
           st == o.st;
  }
};

struct ProfClass {
  int cls = 0;
  std::vector<hipEvent_t> ev;  // pairs
  size_t used = 0;
  double algo = 0.0;
};

}  // namespace

// Split-K workspace of the batched decode GEMV (kernels.hip gemv_tiles_dispatch): up to 16 splits
// of 32 rows x 4096 columns, one ticket per 16-column tile.  Used only by enqueue_forward's GEMVs
// (one stream per stage); head slices on another stream never split K.
// Also the prefill GEMMs' partials: gemm_mfma3's stream-K slabs (2 per block of a grid of up to 512) and
// gemm_split_k's 64x64 split-K tiles.
constexpr size_t kSkCap = (size_t)1024 * 128 * 128;
constexpr int kSkTickets = 4096;

static int graphs_default() {
  const char* e = getenv("BS_GRAPHS");
  return (e && e[0] == '0') ? 0 : 1;
}

struct bs_stage {
  bs_stage_desc d;
  int bf16 = 1;
  int q8 = 0;              // BS_FLAG_INT8_WEIGHTS: block matrices int8 + row scales
  size_t esz = 2;
  void* wtmp = nullptr;    // int8 stages: bf16 [4h][h] staging (init) and dequantized operand (prefill)
  int hd = 0, L = 0;
  hipStream_t own = nullptr;
  // HBM
  char* wbase = nullptr;
  size_t wbytes = 0;
  void* wemb = nullptr;
  void* emb_g = nullptr;
  void* emb_b = nullptr;
  void* lnf_g = nullptr;
  void* lnf_b = nullptr;
  void* hw = nullptr;     // head slice rows [hv0, hv1) of the tied lm_head (may point into wemb)
  int hv0 = 0, hv1 = 0;
  void* score = nullptr;  // BS_FLAG_CLASSIFIER: score [n_labels][hidden] (the head instead of the lm_head)
  int n_labels = 0;
  std::vector<Layer> layers;
  char* kv = nullptr;  // [L][2][max_batch][heads][max_ctx][hd]
  size_t kvbytes = 0;
  size_t kv_layer_stride = 0;  // bytes per (layer) = 2 * half
  size_t kv_half = 0;          // bytes for K (or V) of one layer
  char* ws = nullptr;
  size_t wsbytes = 0;
  float* xa = nullptr;   // fp32 [T][h]
  float* xb = nullptr;   // fp32 [T][h]
  float* attn = nullptr; // fp32 [T][h]
  void* q = nullptr;     // act [T][h]
  void* xn = nullptr;    // act [T][h]
  void* ctx = nullptr;   // act [T][h]
  void* g = nullptr;     // act [T][4h]
  float* part_acc = nullptr;
  float* part_ml = nullptr;
  int max_chunks = 0, chunk = 64;
  float* slopes = nullptr;
  unsigned long long* keys = nullptr;  // [max_batch][V/16]
  int* tok = nullptr;                  // [max_batch]
  int* ids = nullptr;                  // [T] staging for host ids
  int* past_dev = nullptr;
  unsigned* att_tickets = nullptr;     // [max_batch][n_head]
  std::vector<int> past_next;          // what past_dev[0..B) holds after the enqueued forwards (last stage)
  bool past_next_valid = false;
  hipStream_t past_stream = nullptr;   // the stream those forwards were enqueued on
  float* sk_ws = nullptr;              // batched-GEMV split-K partials (kSkCap floats)
  unsigned* sk_tickets = nullptr;      // [kSkTickets]
  ProfClass prof;
  std::vector<std::pair<void*, size_t>> order;  // canonical weight order (BS_WEIGHTS_HOST layout)
  std::vector<std::pair<const float*, int>> order_q8;  // per order entry: (row scales, K) if int8, else (null, 0)
  std::vector<std::pair<GraphKey, hipGraphExec_t>> graphs;  // captured decode steps
  float* logit_buf = nullptr;       // host-I/O logits staging
  size_t logit_cap = 0;
  // tail token pick (bs_set_sampling): top_k <= 1 greedy, else seeded top-k sampling
  int top_k = 1;
  float temperature = 1.f;
  uint64_t sample_seed = 0;
  float* sample_logits = nullptr;   // [max_batch][V] logits the sampler reads (device I/O without logits)
  // bs_set_graphs: decode steps on device buffers replay captured graphs.  Initial value: 1, or 0 when BS_GRAPHS=0 is
  // set (rocprofv3 --pmc runs: rocprofiler-sdk's counter-collection dispatch interception faulted on graph-launched
  // kernels)
  int graphs_on = graphs_default();
};

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

static uint64_t host_sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
static uint64_t tensor_key(uint64_t seed, int layer, uint32_t tid) {
  return host_sm64(seed ^ host_sm64(((uint64_t)(uint32_t)(layer + 1) << 8) | tid));
}
static int layer_kind(int tid) {
  switch (tid) {
    case T_LN1_G: case T_LN2_G: return 2;
    case T_LN1_B: case T_LN2_B: return 3;
    case T_QKV_W: case T_DENSE_W: case T_FC1_W: case T_FC2_W: return 0;
    default: return 1;
  }
}
static void layer_sizes(size_t h, size_t* sz) {
  const size_t s[T_NLAYER] = {h, h, 3 * h * h, 3 * h, h * h, h, h, h, 4 * h * h, 4 * h, 4 * h * h, h};
  for (int i = 0; i < T_NLAYER; i++) sz[i] = s[i];
}

// ALiBi slopes, build_alibi_tensor (modeling_bloom.py:60-78).
static void alibi_slopes(int n_head, float* out) {
  int cp2 = 1;
  while (cp2 * 2 <= n_head) cp2 *= 2;
  const float basef = (float)std::pow(2.0, -std::pow(2.0, -(std::log2((double)cp2) - 3.0)));
  for (int i = 0; i < cp2; i++) out[i] = (float)std::pow((double)basef, (double)(i + 1));
  if (cp2 != n_head) {
    const float ebf = (float)std::pow(2.0, -std::pow(2.0, -(std::log2((double)(2 * cp2)) - 3.0)));
    const int rem = std::min(n_head - cp2, cp2);
    for (int i = 0; i < rem; i++) out[cp2 + i] = (float)std::pow((double)ebf, (double)(2 * i + 1));
  }
}

static int validate(const bs_stage_desc* d, bool from_file = false) {
  if (!d) return fail(BS_ERR_INVALID, "desc is NULL");
  if (d->hidden <= 0 || d->n_head <= 0 || d->hidden % d->n_head)
    return fail(BS_ERR_INVALID, "hidden must be a positive multiple of n_head");
  if (d->hidden % 32) return fail(BS_ERR_INVALID, "hidden must be a multiple of 32");
  const int hd = d->hidden / d->n_head;
  if (hd % 8 || hd > 128) return fail(BS_ERR_INVALID, "head_dim must be a multiple of 8 and <= 128");
  if (d->n_layer <= 0 || d->layer_begin < 0 || d->layer_end > d->n_layer || d->layer_begin > d->layer_end)
    return fail(BS_ERR_INVALID, "bad layer range");
  if (d->vocab <= 0 || d->vocab % 16) return fail(BS_ERR_INVALID, "vocab must be a positive multiple of 16");
  if (d->dtype != BS_DT_BFLOAT16 && d->dtype != BS_DT_FLOAT) return fail(BS_ERR_INVALID, "dtype must be BFLOAT16 or FLOAT");
  if (d->max_batch <= 0 || d->max_ctx <= 0) return fail(BS_ERR_INVALID, "max_batch/max_ctx must be positive");
  if (!(d->ln_eps > 0.f)) return fail(BS_ERR_INVALID, "ln_eps must be positive");
  if (d->head_vocab_begin < 0 || d->head_vocab_end < d->head_vocab_begin || d->head_vocab_end > d->vocab ||
      d->head_vocab_begin % 16 || d->head_vocab_end % 16)
    return fail(BS_ERR_INVALID, "head vocab slice must be a 16-aligned sub-range of [0, vocab)");
  if (!from_file && d->weight_source != BS_WEIGHTS_SYNTHETIC && d->weight_source != BS_WEIGHTS_HOST)
    return fail(BS_ERR_INVALID, "unknown weight_source");
  if (d->flags & ~(BS_FLAG_INT8_WEIGHTS | BS_FLAG_CLASSIFIER)) return fail(BS_ERR_INVALID, "unknown desc flags");
  if (d->flags & BS_FLAG_CLASSIFIER) {
    if (!d->is_last) return fail(BS_ERR_INVALID, "BS_FLAG_CLASSIFIER needs the last stage");
    if (d->n_labels < 1 || d->n_labels > 64) return fail(BS_ERR_INVALID, "n_labels must be in [1, 64]");
    if (d->head_vocab_end > d->head_vocab_begin) return fail(BS_ERR_INVALID, "a classifier stage takes no head slice");
  }
  if ((d->flags & BS_FLAG_INT8_WEIGHTS) && d->dtype != BS_DT_BFLOAT16)
    return fail(BS_ERR_UNSUPPORTED, "BS_FLAG_INT8_WEIGHTS needs dtype BFLOAT16");
  return BS_OK;
}

extern "C" uint64_t bs_stage_weight_count(const bs_stage_desc* d) {
  if (validate(d) != BS_OK) return 0;
  const uint64_t h = (uint64_t)d->hidden;
  uint64_t n = 0;
  const bool cls = (d->flags & BS_FLAG_CLASSIFIER) != 0;
  if (d->is_first || (d->is_last && !cls)) n += (uint64_t)d->vocab * h;
  if (d->is_first) n += 2 * h;
  n += (uint64_t)(d->layer_end - d->layer_begin) * (12 * h * h + 13 * h);
  if (d->is_last) n += 2 * h;
  if (cls) n += (uint64_t)d->n_labels * h;
  const bool slice = d->head_vocab_end > d->head_vocab_begin;
  if (slice && !d->is_first && !d->is_last) n += (uint64_t)(d->head_vocab_end - d->head_vocab_begin) * h;
  if (slice && !d->is_last) n += 2 * h;
  return n;
}

extern "C" int bs_abi_version(void) { return BS_ABI_VERSION; }

#ifndef BS_BUILD_ID
#define BS_BUILD_ID "unstamped"
#endif
extern "C" const char* bs_build_id(void) { return BS_BUILD_ID; }

static uint32_t host_lb32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

extern "C" int bs_prompt_ids(uint64_t seed, int32_t n, int32_t vocab, int32_t* out) {
  if (n < 0 || vocab <= 0 || (n && !out)) return fail(BS_ERR_INVALID, "bad prompt_ids arguments");
  const uint64_t key = tensor_key(seed, -1, 255);
  for (int32_t i = 0; i < n; i++)
    out[i] = (int32_t)(host_lb32((uint32_t)key ^ host_lb32((uint32_t)i + (uint32_t)(key >> 32))) % (uint32_t)vocab);
  return BS_OK;
}
extern "C" const char* bs_last_error(void) { return g_err.c_str(); }

static void free_stage(bs_stage* s) {
  if (!s) return;
  hipSetDevice(s->d.device);
  if (s->own) hipStreamSynchronize(s->own);
  for (auto e : s->prof.ev) hipEventDestroy(e);
  for (auto& g : s->graphs) hipGraphExecDestroy(g.second);
  if (s->wbase) hipFree(s->wbase);
  if (s->kv) hipFree(s->kv);
  if (s->ws) hipFree(s->ws);
  if (s->logit_buf) hipFree(s->logit_buf);
  if (s->sample_logits) hipFree(s->sample_logits);
  if (s->wtmp) hipFree(s->wtmp);
  if (s->own) hipStreamDestroy(s->own);
  delete s;
}

// Checkpoint tensor of each canonical-order entry (the BS_WEIGHTS_HOST layout), HF BloomModel names
// (modeling_bloom.py; the names the reference's ONNX modules were exported from).
struct FileEntry {
  std::string name;
  uint64_t first;                // element offset inside the checkpoint tensor (head slice rows)
  std::vector<int64_t> shape;    // the checkpoint tensor's expected shape
};
static std::vector<FileEntry> file_entries(const bs_stage_desc* d) {
  const int64_t h = d->hidden, V = d->vocab;
  std::vector<FileEntry> e;
  const bool cls = (d->flags & BS_FLAG_CLASSIFIER) != 0;
  if (d->is_first || (d->is_last && !cls)) e.push_back({"word_embeddings.weight", 0, {V, h}});
  if (d->is_first) {
    e.push_back({"word_embeddings_layernorm.weight", 0, {h}});
    e.push_back({"word_embeddings_layernorm.bias", 0, {h}});
  }
  static const char* tn[T_NLAYER] = {
      "input_layernorm.weight", "input_layernorm.bias", "self_attention.query_key_value.weight",
      "self_attention.query_key_value.bias", "self_attention.dense.weight", "self_attention.dense.bias",
      "post_attention_layernorm.weight", "post_attention_layernorm.bias", "mlp.dense_h_to_4h.weight",
      "mlp.dense_h_to_4h.bias", "mlp.dense_4h_to_h.weight", "mlp.dense_4h_to_h.bias"};
  const std::vector<int64_t> ts[T_NLAYER] = {{h}, {h}, {3 * h, h}, {3 * h}, {h, h}, {h}, {h}, {h}, {4 * h, h}, {4 * h},
                                             {h, 4 * h}, {h}};
  for (int l = d->layer_begin; l < d->layer_end; l++)
    for (int t = 0; t < T_NLAYER; t++) e.push_back({"h." + std::to_string(l) + "." + tn[t], 0, ts[t]});
  if (d->is_last) { e.push_back({"ln_f.weight", 0, {h}}); e.push_back({"ln_f.bias", 0, {h}}); }
  if (cls) e.push_back({"score.weight", 0, {(int64_t)d->n_labels, h}});  // BloomForSequenceClassification.score
  const bool slice = d->head_vocab_end > d->head_vocab_begin;
  if (slice && !d->is_first && !d->is_last) e.push_back({"word_embeddings.weight", (uint64_t)d->head_vocab_begin * h, {V, h}});
  if (slice && !d->is_last) { e.push_back({"ln_f.weight", 0, {h}}); e.push_back({"ln_f.bias", 0, {h}}); }
  return e;
}
static const st::Tensor* find_entry(const st::Checkpoint& ck, const FileEntry& fe, std::string* why) {
  const st::Tensor* t = ck.find(fe.name);
  if (!t && fe.name == "word_embeddings.weight") t = ck.find("lm_head.weight");  // tied head saved alone
  if (!t) { *why = "checkpoint has no tensor '" + fe.name + "'"; return nullptr; }
  if (t->shape != fe.shape) {
    std::string a, b;
    for (auto v : t->shape) a += std::to_string(v) + ",";
    for (auto v : fe.shape) b += std::to_string(v) + ",";
    *why = "tensor '" + fe.name + "' has shape [" + a + "] but the stage needs [" + b + "]";
    return nullptr;
  }
  if (t->dtype == st::OTHER) { *why = "tensor '" + fe.name + "' has dtype " + t->dtype_name + " (need F32/F16/BF16)"; return nullptr; }
  return t;
}

static float host_f16(uint16_t v) {
  const uint32_t sgn = (uint32_t)(v >> 15) << 31, ex = (v >> 10) & 31, man = v & 1023;
  uint32_t bits;
  if (ex == 31) bits = sgn | 0x7F800000u | (man << 13);
  else if (ex) bits = sgn | ((ex + 112) << 23) | (man << 13);
  else if (!man) bits = sgn;
  else {  // subnormal: exact in fp32
    float f = (float)man * 5.9604644775390625e-8f;  // 2^-24
    std::memcpy(&bits, &f, 4);
    bits |= sgn;
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

static int init_stage(const bs_stage_desc* desc, bs_stage** out, const st::Checkpoint* ck);

extern "C" int bs_init_stage(const bs_stage_desc* desc, bs_stage** out) { return init_stage(desc, out, nullptr); }

extern "C" int bs_init_stage_file(const bs_stage_desc* desc, const char* path, bs_stage** out) {
  if (!out) return fail(BS_ERR_INVALID, "out is NULL");
  *out = nullptr;
  if (!path) return fail(BS_ERR_INVALID, "path is NULL");
  int rc = validate(desc, true);
  if (rc) return rc;
  st::Checkpoint ck;
  std::string err;
  if (!ck.open(path, &err)) return fail(BS_ERR_INVALID, err);
  for (const auto& fe : file_entries(desc))  // every tensor present and shaped right before any allocation
    if (!find_entry(ck, fe, &err)) return fail(BS_ERR_INVALID, err);
  return init_stage(desc, out, &ck);
}

extern "C" int bs_weights_file_probe(const char* path, int32_t* hidden, int32_t* n_layer, int32_t* vocab) {
  if (!path) return fail(BS_ERR_INVALID, "path is NULL");
  st::Checkpoint ck;
  std::string err;
  if (!ck.open(path, &err)) return fail(BS_ERR_INVALID, err);
  const st::Tensor* e = ck.find("word_embeddings.weight");
  if (!e) e = ck.find("lm_head.weight");
  int32_t hid = -1, nl = 0, V = -1;
  if (e && e->shape.size() == 2) { V = (int32_t)e->shape[0]; hid = (int32_t)e->shape[1]; }
  for (const auto& kv : ck.tensors()) {  // layers: 1 + the highest h.<i>. present
    const std::string& n = kv.first;
    auto ends = [&](const std::string& x) { return n.size() >= x.size() && !n.compare(n.size() - x.size(), x.size(), x); };
    if (hid < 0 && (ends("layernorm.weight") || ends("ln_f.weight")) && kv.second.shape.size() == 1)
      hid = (int32_t)kv.second.shape[0];  // any LayerNorm gives the width
    size_t p = n.rfind("h.", 0) == 0 ? 2 : (n.rfind("transformer.h.", 0) == 0 ? 14 : std::string::npos);
    if (p == std::string::npos) continue;
    long i = 0;
    size_t q = p;
    while (q < n.size() && n[q] >= '0' && n[q] <= '9' && i < 1000000) i = i * 10 + (n[q++] - '0');
    if (q > p && q < n.size() && n[q] == '.') nl = std::max(nl, (int32_t)i + 1);
  }
  if (hidden) *hidden = hid;
  if (n_layer) *n_layer = nl;
  if (vocab) *vocab = V;
  return BS_OK;
}

static int init_stage(const bs_stage_desc* desc, bs_stage** out, const st::Checkpoint* ck) {
  if (!out) return fail(BS_ERR_INVALID, "out is NULL");
  *out = nullptr;
  int rc = validate(desc, ck != nullptr);
  if (rc) return rc;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (desc->device < 0 || desc->device >= ndev) return fail(BS_ERR_INVALID, "device ordinal out of range");
  HIP_TRY(hipSetDevice(desc->device));

  bs_stage* s = new bs_stage();
  s->d = *desc;
  if (s->d.max_tokens <= 0) s->d.max_tokens = s->d.max_batch * 128;
  s->bf16 = desc->dtype == BS_DT_BFLOAT16;
  s->q8 = (desc->flags & BS_FLAG_INT8_WEIGHTS) != 0;
  s->esz = s->bf16 ? 2 : 4;
  s->n_labels = (desc->flags & BS_FLAG_CLASSIFIER) ? desc->n_labels : 0;
  s->hd = desc->hidden / desc->n_head;
  s->L = desc->layer_end - desc->layer_begin;
  const size_t h = desc->hidden, V = desc->vocab, T = s->d.max_tokens;

  auto cleanup = [&](int code) { free_stage(s); return code; };
  if (hipStreamCreateWithFlags(&s->own, hipStreamNonBlocking) != hipSuccess)
    return cleanup(fail(BS_ERR_DEVICE, "hipStreamCreate failed"));

  // ---- weight arena: every tensor 256-B aligned
  std::vector<std::pair<void**, size_t>> plan;  // (slot, elements)
  size_t off = 0;
  std::vector<size_t> offs;
  auto add = [&](size_t n) { offs.push_back(off); off = align_up(off + n * s->esz, 256); };
  auto addb = [&](size_t bytes) { offs.push_back(off); off = align_up(off + bytes, 256); };
  const bool own_emb = desc->is_first || (desc->is_last && !s->n_labels);
  if (own_emb) add(V * h);
  if (desc->is_first) { add(h); add(h); }
  size_t lsz[T_NLAYER];
  layer_sizes(h, lsz);
  for (int l = 0; l < s->L; l++)
    for (int t = 0; t < T_NLAYER; t++) {
      if (s->q8 && is_matrix(t)) {
        addb(lsz[t]);                                               // int8 [N][K]
        addb((t == T_FC1_W ? 4 * h : (t == T_QKV_W ? 3 * h : h)) * 4);  // fp32 scale [N]
      } else {
        add(lsz[t]);
      }
    }
  if (desc->is_last) { add(h); add(h); }
  if (s->n_labels) add((size_t)s->n_labels * h);
  const bool slice = desc->head_vocab_end > desc->head_vocab_begin;
  s->hv0 = desc->head_vocab_begin;
  s->hv1 = desc->head_vocab_end;
  const size_t hrows = (size_t)(s->hv1 - s->hv0);
  if (slice && !desc->is_first && !desc->is_last) add(hrows * h);
  if (slice && !desc->is_last) { add(h); add(h); }
  s->wbytes = off;
  if (hipMalloc(&s->wbase, s->wbytes ? s->wbytes : 256) != hipSuccess)
    return cleanup(fail(BS_ERR_OOM, "weight allocation failed (" + std::to_string(s->wbytes) + " B)"));
  size_t oi = 0;
  if (own_emb) s->wemb = s->wbase + offs[oi++];
  if (desc->is_first) { s->emb_g = s->wbase + offs[oi++]; s->emb_b = s->wbase + offs[oi++]; }
  s->layers.resize(s->L);
  for (int l = 0; l < s->L; l++)
    for (int t = 0; t < T_NLAYER; t++) {
      s->layers[l].t[t] = s->wbase + offs[oi++];
      s->layers[l].sc[t] = (s->q8 && is_matrix(t)) ? (float*)(s->wbase + offs[oi++]) : nullptr;
    }
  if (desc->is_last) { s->lnf_g = s->wbase + offs[oi++]; s->lnf_b = s->wbase + offs[oi++]; }
  if (s->n_labels) s->score = s->wbase + offs[oi++];
  if (slice) {
    if (s->wemb) s->hw = (char*)s->wemb + (size_t)s->hv0 * h * s->esz;
    else s->hw = s->wbase + offs[oi++];
    if (!desc->is_last) { s->lnf_g = s->wbase + offs[oi++]; s->lnf_b = s->wbase + offs[oi++]; }
  } else if (desc->is_last && !s->n_labels) {
    s->hw = s->wemb; s->hv0 = 0; s->hv1 = desc->vocab;  // the last stage's full head
  }
  if (s->wemb) s->order.push_back({s->wemb, V * h});
  if (s->emb_g) { s->order.push_back({s->emb_g, h}); s->order.push_back({s->emb_b, h}); }
  for (int l = 0; l < s->L; l++)
    for (int t = 0; t < T_NLAYER; t++) s->order.push_back({s->layers[l].t[t], lsz[t]});
  if (desc->is_last) { s->order.push_back({s->lnf_g, h}); s->order.push_back({s->lnf_b, h}); }
  if (s->score) s->order.push_back({s->score, (size_t)s->n_labels * h});
  if (slice && !desc->is_first && !desc->is_last) s->order.push_back({s->hw, hrows * h});
  if (slice && !desc->is_last) { s->order.push_back({s->lnf_g, h}); s->order.push_back({s->lnf_b, h}); }
  s->order_q8.assign(s->order.size(), {nullptr, 0});
  if (s->q8) {
    for (size_t i = 0; i < s->order.size(); i++)
      for (int l = 0; l < s->L; l++)
        for (int t = 0; t < T_NLAYER; t++)
          if (s->layers[l].sc[t] && s->order[i].first == s->layers[l].t[t])
            s->order_q8[i] = {s->layers[l].sc[t], (int)(t == T_FC2_W ? 4 * h : h)};
    if (hipMalloc(&s->wtmp, 4 * h * h * 2) != hipSuccess) return cleanup(fail(BS_ERR_OOM, "int8 staging allocation failed"));
  }
  // int8 matrices are produced in bf16 in the staging buffer, then quantized into the arena
  auto quantize = [&](size_t i) {
    const int K = s->order_q8[i].second, N = (int)(s->order[i].second / K);
    launch_quantize_rows(s->wtmp, (int8_t*)s->order[i].first, (float*)s->order_q8[i].first, N, K, s->own);
  };

  // ---- weights
  if (ck) {
    // Straight from the file mapping: matching dtypes are copied as they are, others widen to fp32 on
    // the host (exact) and take the BS_WEIGHTS_HOST conversion, so a file of fp32 weights loads
    // bit-identical to the same weights passed as a host buffer.
    const std::vector<FileEntry> fes = file_entries(desc);
    if (fes.size() != s->order.size()) return cleanup(fail(BS_ERR_STATE, "checkpoint entry list out of step"));
    const size_t chunk = 16u << 20;
    std::vector<float> wide(chunk);
    float* bounce = nullptr;
    if (hipMalloc(&bounce, chunk * sizeof(float)) != hipSuccess) return cleanup(fail(BS_ERR_OOM, "bounce alloc"));
    std::string why;
    for (size_t oi2 = 0; oi2 < s->order.size(); oi2++) {
      const auto& o = s->order[oi2];
      const bool q = s->order_q8[oi2].first != nullptr;
      char* dst = (char*)(q ? s->wtmp : o.first);
      const st::Tensor* t = find_entry(*ck, fes[oi2], &why);
      if (!t || fes[oi2].first + o.second > t->numel()) {
        hipFree(bounce);
        return cleanup(fail(BS_ERR_INVALID, t ? "head slice outside the checkpoint's embedding" : why));
      }
      const bool same = (s->bf16 && t->dtype == st::BF16) || (!s->bf16 && t->dtype == st::F32);
      const size_t tes = t->dtype == st::F32 ? 4 : 2;
      const uint8_t* src = t->data + fes[oi2].first * tes;
      bool ok = true;
      if (same) {
        ok = hipMemcpyAsync(dst, src, o.second * s->esz, hipMemcpyHostToDevice, s->own) == hipSuccess;
      } else {
        for (size_t i = 0; ok && i < o.second; i += chunk) {
          const size_t n = std::min(chunk, o.second - i);
          const uint8_t* p = src + i * tes;
          if (t->dtype == st::F32) {
            std::memcpy(wide.data(), p, n * 4);
          } else {
            for (size_t j = 0; j < n; j++) {
              uint16_t v;
              std::memcpy(&v, p + 2 * j, 2);
              if (t->dtype == st::BF16) {
                const uint32_t b = (uint32_t)v << 16;
                std::memcpy(&wide[j], &b, 4);
              } else {
                wide[j] = host_f16(v);
              }
            }
          }
          ok = hipMemcpyAsync(bounce, wide.data(), n * sizeof(float), hipMemcpyHostToDevice, s->own) == hipSuccess;
          if (ok) launch_convert_f32(dst + i * s->esz, s->bf16, bounce, n, s->own);
          ok = ok && hipStreamSynchronize(s->own) == hipSuccess;  // `wide` is refilled next round
        }
      }
      if (ok && q) quantize(oi2);
      if (!ok) {
        hipFree(bounce);
        return cleanup(fail(BS_ERR_DEVICE, "weight upload failed"));
      }
    }
    const bool synced = hipStreamSynchronize(s->own) == hipSuccess;  // the mapping goes away after init
    hipFree(bounce);
    if (!synced) return cleanup(fail(BS_ERR_DEVICE, "weight upload failed"));
  } else if (desc->weight_source == BS_WEIGHTS_SYNTHETIC) {
    const uint64_t seed = desc->seed;
    if (s->wemb) launch_gen_fill(s->wemb, s->bf16, V * h, tensor_key(seed, -1, M_WEMB), 0, s->own);
    if (s->emb_g) launch_gen_fill(s->emb_g, s->bf16, h, tensor_key(seed, -1, M_EMB_G), 2, s->own);
    if (s->emb_b) launch_gen_fill(s->emb_b, s->bf16, h, tensor_key(seed, -1, M_EMB_B), 3, s->own);
    for (int l = 0; l < s->L; l++)
      for (int t = 0; t < T_NLAYER; t++) {
        const bool q = s->layers[l].sc[t] != nullptr;
        launch_gen_fill(q ? s->wtmp : s->layers[l].t[t], s->bf16, lsz[t], tensor_key(seed, desc->layer_begin + l, t),
                        layer_kind(t), s->own);
        if (q) {
          for (size_t i = 0; i < s->order.size(); i++)
            if (s->order[i].first == s->layers[l].t[t]) quantize(i);
        }
      }
    if (slice && !s->wemb)
      launch_gen_fill(s->hw, s->bf16, hrows * h, tensor_key(seed, -1, M_WEMB), 0, s->own, (uint64_t)s->hv0 * h);
    if (s->lnf_g) launch_gen_fill(s->lnf_g, s->bf16, h, tensor_key(seed, -1, M_LNF_G), 2, s->own);
    if (s->lnf_b) launch_gen_fill(s->lnf_b, s->bf16, h, tensor_key(seed, -1, M_LNF_B), 3, s->own);
    if (s->score) launch_gen_fill(s->score, s->bf16, (size_t)s->n_labels * h, tensor_key(seed, -1, M_SCORE), 0, s->own);
  } else {
    const uint64_t need = bs_stage_weight_count(desc);
    if (!desc->host_weights || desc->host_weight_count != need)
      return cleanup(fail(BS_ERR_INVALID, "host_weights count mismatch: need " + std::to_string(need)));
    // canonical order == arena order; upload through an fp32 bounce buffer
    const size_t chunk = 16u << 20;
    float* bounce = nullptr;
    if (hipMalloc(&bounce, chunk * sizeof(float)) != hipSuccess) return cleanup(fail(BS_ERR_OOM, "bounce alloc"));
    const float* src = desc->host_weights;
    for (size_t oi2 = 0; oi2 < s->order.size(); oi2++) {
      const auto& o = s->order[oi2];
      const bool q = s->order_q8[oi2].first != nullptr;
      for (size_t i = 0; i < o.second; i += chunk) {
        const size_t n = std::min(chunk, o.second - i);
        if (hipMemcpyAsync(bounce, src + i, n * sizeof(float), hipMemcpyHostToDevice, s->own) != hipSuccess) {
          hipFree(bounce);
          return cleanup(fail(BS_ERR_DEVICE, "weight upload failed"));
        }
        launch_convert_f32((char*)(q ? s->wtmp : o.first) + i * s->esz, s->bf16, bounce, n, s->own);
      }
      if (q) quantize(oi2);
      src += o.second;
    }
    hipStreamSynchronize(s->own);
    hipFree(bounce);
  }

  // ---- KV cache
  s->kv_half = (size_t)desc->max_batch * desc->n_head * desc->max_ctx * s->hd * s->esz;
  s->kv_layer_stride = 2 * s->kv_half;
  s->kvbytes = s->kv_layer_stride * (s->L > 0 ? s->L : 0);
  if (s->kvbytes) {
    if (hipMalloc(&s->kv, s->kvbytes) != hipSuccess)
      return cleanup(fail(BS_ERR_OOM, "KV cache allocation failed (" + std::to_string(s->kvbytes) + " B)"));
    if (hipMemsetAsync(s->kv, 0, s->kvbytes, s->own) != hipSuccess) return cleanup(fail(BS_ERR_DEVICE, "kv memset"));
  }

  // ---- workspace
  const size_t attn_f = attention_workspace_floats(desc->max_batch, desc->n_head, s->hd, desc->max_ctx, &s->max_chunks,
                                                   &s->chunk);
  std::vector<size_t> wo;
  size_t woff = 0;
  auto wadd = [&](size_t bytes) { wo.push_back(woff); woff = align_up(woff + bytes, 256); };
  wadd(T * h * 4);       // xa
  wadd(T * h * 4);       // xb
  wadd(T * h * 4);       // attn
  wadd(T * h * 4);       // q
  wadd(T * h * s->esz);  // xn
  wadd(T * h * s->esz);  // ctx
  wadd(T * 4 * h * s->esz);  // g
  wadd(attn_f * 4);      // partials
  wadd(desc->n_head * 4);
  wadd((size_t)desc->max_batch * (V / 16) * 8);
  wadd((size_t)desc->max_batch * 4);
  wadd(T * 4);
  wadd((size_t)desc->max_batch * 4);                 // per-row past_len (device copy)
  wadd((size_t)desc->max_batch * desc->n_head * 4);  // attention split-merge tickets
  wadd(kSkCap * 4);                                  // batched-GEMV split-K partials
  wadd(kSkTickets * 4);                              // and their tickets
  s->wsbytes = woff;
  if (hipMalloc(&s->ws, s->wsbytes) != hipSuccess) return cleanup(fail(BS_ERR_OOM, "workspace allocation failed"));
  int wi = 0;
  s->xa = (float*)(s->ws + wo[wi++]);
  s->xb = (float*)(s->ws + wo[wi++]);
  s->attn = (float*)(s->ws + wo[wi++]);
  s->q = s->ws + wo[wi++];
  s->xn = s->ws + wo[wi++];
  s->ctx = s->ws + wo[wi++];
  s->g = s->ws + wo[wi++];
  s->part_acc = (float*)(s->ws + wo[wi++]);
  s->part_ml = s->part_acc + (size_t)desc->max_batch * desc->n_head * s->max_chunks * s->hd;
  s->slopes = (float*)(s->ws + wo[wi++]);
  s->keys = (unsigned long long*)(s->ws + wo[wi++]);
  s->tok = (int*)(s->ws + wo[wi++]);
  s->ids = (int*)(s->ws + wo[wi++]);
  s->past_dev = (int*)(s->ws + wo[wi++]);
  s->att_tickets = (unsigned*)(s->ws + wo[wi++]);
  s->sk_ws = (float*)(s->ws + wo[wi++]);
  s->sk_tickets = (unsigned*)(s->ws + wo[wi++]);
  HIP_TRY(hipMemsetAsync(s->ws, 0, s->wsbytes, s->own));
  std::vector<float> sl(desc->n_head);
  alibi_slopes(desc->n_head, sl.data());
  HIP_TRY(hipMemcpyAsync(s->slopes, sl.data(), sl.size() * 4, hipMemcpyHostToDevice, s->own));
  hipError_t e = hipStreamSynchronize(s->own);
  if (e != hipSuccess) return cleanup(fail(BS_ERR_DEVICE, std::string("init sync: ") + hipGetErrorString(e)));
  e = hipGetLastError();
  if (e != hipSuccess) return cleanup(fail(BS_ERR_DEVICE, std::string("init kernels: ") + hipGetErrorString(e)));
  *out = s;
  return BS_OK;
}

extern "C" void bs_release(bs_stage* s) { free_stage(s); }

extern "C" int bs_stage_info(const bs_stage* s, bs_stage_desc* d, uint64_t* wb, uint64_t* kvb, uint64_t* wsb) {
  if (!s) return fail(BS_ERR_INVALID, "stage is NULL");
  if (d) *d = s->d;
  if (wb) *wb = s->wbytes;
  if (kvb) *kvb = s->kvbytes;
  if (wsb) *wsb = s->wsbytes;
  return BS_OK;
}

extern "C" int bs_read_weights(const bs_stage* s, uint64_t offset, uint64_t count, float* out) {
  if (!s || (count && !out)) return fail(BS_ERR_INVALID, "stage/out is NULL");
  HIP_TRY(hipSetDevice(s->d.device));
  HIP_TRY(hipStreamSynchronize(s->own));
  uint64_t base = 0, done = 0;
  std::vector<uint16_t> tmp;
  std::vector<int8_t> qtmp;
  std::vector<float> stmp;
  for (size_t oi = 0; oi < s->order.size(); oi++) {
    const auto& o = s->order[oi];
    const uint64_t b = base, e = base + o.second;
    base = e;
    if (e <= offset || b >= offset + count) continue;
    const uint64_t lo = std::max<uint64_t>(b, offset), hi = std::min<uint64_t>(e, offset + count);
    const uint64_t n = hi - lo;
    const char* src = (const char*)o.first + (lo - b) * s->esz;
    float* dst = out + (lo - offset);
    if (s->order_q8[oi].first) {  // int8 matrix: dequantized values Q * scale
      const int K = s->order_q8[oi].second;
      const uint64_t r0 = (lo - b) / K, r1 = (hi - b - 1) / K;
      qtmp.resize(n);
      stmp.resize(r1 - r0 + 1);
      HIP_TRY(hipMemcpy(qtmp.data(), (const int8_t*)o.first + (lo - b), n, hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy(stmp.data(), s->order_q8[oi].first + r0, stmp.size() * 4, hipMemcpyDeviceToHost));
      for (uint64_t i = 0; i < n; i++) dst[i] = (float)qtmp[i] * stmp[(lo - b + i) / K - r0];
    } else if (s->bf16) {
      tmp.resize(n);
      HIP_TRY(hipMemcpy(tmp.data(), src, n * 2, hipMemcpyDeviceToHost));
      for (uint64_t i = 0; i < n; i++) {
        uint32_t u = (uint32_t)tmp[i] << 16;
        std::memcpy(&dst[i], &u, 4);
      }
    } else {
      HIP_TRY(hipMemcpy(dst, src, n * 4, hipMemcpyDeviceToHost));
    }
    done += n;
  }
  if (done != count) return fail(BS_ERR_INVALID, "read range outside the stage weights");
  return BS_OK;
}

extern "C" int bs_read_kv(const bs_stage* s, int32_t layer, int32_t slot, int32_t pos0, int32_t npos, float* out) {
  if (!s || !out) return fail(BS_ERR_INVALID, "stage/out is NULL");
  if (layer < 0 || layer >= s->L) return fail(BS_ERR_INVALID, "layer outside the stage");
  if (slot < 0 || slot >= s->d.max_batch) return fail(BS_ERR_INVALID, "slot out of range");
  if (pos0 < 0 || npos < 0 || pos0 + npos > s->d.max_ctx) return fail(BS_ERR_INVALID, "positions outside max_ctx");
  HIP_TRY(hipSetDevice(s->d.device));
  HIP_TRY(hipStreamSynchronize(s->own));
  const int nh = s->d.n_head, hd = s->hd;
  const size_t run = (size_t)npos * hd;  // contiguous elements of one (K|V, head)
  std::vector<uint16_t> tmp(s->bf16 ? run : 0);
  for (int w = 0; w < 2; w++)
    for (int hh = 0; hh < nh; hh++) {
      const size_t e0 = (((size_t)slot * nh + hh) * s->d.max_ctx + pos0) * hd;
      const char* src = s->kv + layer * s->kv_layer_stride + w * s->kv_half + e0 * s->esz;
      float* dst = out + ((size_t)w * nh + hh) * run;
      if (s->bf16) {
        HIP_TRY(hipMemcpy(tmp.data(), src, run * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < run; i++) {
          const uint32_t u = (uint32_t)tmp[i] << 16;
          std::memcpy(&dst[i], &u, 4);
        }
      } else {
        HIP_TRY(hipMemcpy(dst, src, run * 4, hipMemcpyDeviceToHost));
      }
    }
  return BS_OK;
}

extern "C" int bs_reset_kv(bs_stage* s, int32_t slot) {
  if (!s) return fail(BS_ERR_INVALID, "stage is NULL");
  if (slot >= s->d.max_batch) return fail(BS_ERR_INVALID, "slot out of range");
  HIP_TRY(hipSetDevice(s->d.device));
  // Cached positions are addressed by past_len, so forgetting is bookkeeping only; zero the
  // rows anyway so stale data can never be read by a caller that reuses past_len wrongly.
  const size_t row = (size_t)s->d.n_head * s->d.max_ctx * s->hd * s->esz;
  for (int l = 0; l < s->L; l++)
    for (int w = 0; w < 2; w++) {
      char* base = s->kv + l * s->kv_layer_stride + w * s->kv_half;
      if (slot < 0) HIP_TRY(hipMemsetAsync(base, 0, s->kv_half, s->own));
      else HIP_TRY(hipMemsetAsync(base + (size_t)slot * row, 0, row, s->own));
    }
  HIP_TRY(hipStreamSynchronize(s->own));
  return BS_OK;
}

// ---- profiling
extern "C" int bs_profile_enable(bs_stage* s, int32_t cls) {
  if (!s) return fail(BS_ERR_INVALID, "stage is NULL");
  s->prof.cls = cls;
  s->prof.used = 0;
  s->prof.algo = 0.0;
  return BS_OK;
}

static hipEvent_t prof_event(bs_stage* s) {
  if (s->prof.used >= s->prof.ev.size()) {
    // no system-scope fence on the timing markers: a fenced record writes back L2 between the
    // timed kernels and stretches each ~5 us launch by ~2 us against the kernel trace
    hipEvent_t e;
    hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    s->prof.ev.push_back(e);
  }
  return s->prof.ev[s->prof.used++];
}

extern "C" int bs_profile_read(bs_stage* s, double* total_ms, uint64_t* launches, double* algo) {
  if (!s) return fail(BS_ERR_INVALID, "stage is NULL");
  double tot = 0.0;
  for (size_t i = 0; i + 1 < s->prof.used; i += 2) {
    HIP_TRY(hipEventSynchronize(s->prof.ev[i + 1]));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, s->prof.ev[i], s->prof.ev[i + 1]));
    tot += ms;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = s->prof.used / 2;
  if (algo) *algo = s->prof.algo;
  return BS_OK;
}

// s_memrealtime ticks at 100 MHz; the spin is bounded by its argument
__global__ void stream_delay_kernel(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

extern "C" int bs_stream_delay(void* stream, int32_t microseconds) {
  if (microseconds < 0 || microseconds > 100000) return fail(BS_ERR_INVALID, "delay must be in [0, 100000] us");
  stream_delay_kernel<<<1, 1, 0, (hipStream_t)stream>>>((long long)microseconds * 100);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(BS_ERR_DEVICE, std::string("stream delay: ") + hipGetErrorString(e));
  return BS_OK;
}

// ---- HBM probe (bench.py "hbm_measured"): STREAM-like read and copy rates of this device.
typedef unsigned int probe_u4 __attribute__((ext_vector_type(4)));
// Every thread keeps 8 16-B loads in flight (a 32 KB tile per 256-thread block and step), grid-stride
// over tiles: enough bytes in flight per CU to hide HBM latency at the full rate.
constexpr int kProbeU = 8;
__global__ __launch_bounds__(256) void probe_read_kernel(const probe_u4* __restrict__ p, size_t n, probe_u4* sink) {
  probe_u4 acc = {0u, 0u, 0u, 0u};
  const size_t tile = (size_t)blockDim.x * kProbeU;
  for (size_t t = (size_t)blockIdx.x * tile; t + tile <= n; t += (size_t)gridDim.x * tile) {
    probe_u4 v[kProbeU];
#pragma unroll
    for (int u = 0; u < kProbeU; u++) v[u] = __builtin_nontemporal_load(p + t + u * blockDim.x + threadIdx.x);
#pragma unroll
    for (int u = 0; u < kProbeU; u++) acc ^= v[u];
  }
  if ((acc.x & acc.y & acc.z & acc.w) == 0xFFFFFFFFu) sink[0] = acc;  // never in practice; keeps the loads
}
__global__ __launch_bounds__(256) void probe_copy_kernel(const probe_u4* __restrict__ p, probe_u4* __restrict__ q, size_t n) {
  const size_t tile = (size_t)blockDim.x * kProbeU;
  for (size_t t = (size_t)blockIdx.x * tile; t + tile <= n; t += (size_t)gridDim.x * tile) {
    probe_u4 v[kProbeU];
#pragma unroll
    for (int u = 0; u < kProbeU; u++) v[u] = __builtin_nontemporal_load(p + t + u * blockDim.x + threadIdx.x);
#pragma unroll
    for (int u = 0; u < kProbeU; u++) __builtin_nontemporal_store(v[u], q + t + u * blockDim.x + threadIdx.x);
  }
}

// Probe resources released on every exit path; every HIP call's status is checked.
namespace {
struct ProbeRes {
  void* buf[2] = {nullptr, nullptr};
  hipStream_t st = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  ~ProbeRes() {
    if (st) hipStreamSynchronize(st);
    for (auto e : ev) if (e) hipEventDestroy(e);
    if (st) hipStreamDestroy(st);
    for (auto b : buf) if (b) hipFree(b);
  }
  int init(size_t bytes, int nbuf) {
    for (int i = 0; i < nbuf; i++)
      if (hipMalloc(&buf[i], bytes) != hipSuccess) return fail(BS_ERR_OOM, "probe allocation failed");
    HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&ev[0]));
    HIP_TRY(hipEventCreate(&ev[1]));
    return BS_OK;
  }
  // Time one launch (enqueued by `launch`) with the event pair; ms < 0 never escapes (status instead).
  template <typename F>
  int timed(F&& launch, float* ms) {
    HIP_TRY(hipEventRecord(ev[0], st));
    launch();
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev[1], st));
    HIP_TRY(hipEventSynchronize(ev[1]));
    HIP_TRY(hipEventElapsedTime(ms, ev[0], ev[1]));
    if (!(*ms > 0.f)) return fail(BS_ERR_DEVICE, "probe: non-positive event time");
    return BS_OK;
  }
};
}  // namespace

extern "C" int bs_hbm_probe(int32_t device, uint64_t bytes, double* read_gbps, double* copy_gbps) {
  if (bytes < (1u << 20) || bytes % (1u << 20)) return fail(BS_ERR_INVALID, "probe bytes must be a positive multiple of 1 MiB");
  HIP_TRY(hipSetDevice(device));
  ProbeRes p;
  int rc = p.init(bytes, 2);
  if (rc) return rc;
  HIP_TRY(hipMemsetAsync(p.buf[0], 1, bytes, p.st));
  const size_t n = bytes / 16;
  const unsigned grid = 256 * 8;  // 8 blocks per CU
  const probe_u4* a = (const probe_u4*)p.buf[0];
  probe_u4* b = (probe_u4*)p.buf[1];
  float best_r = 1e30f, best_c = 1e30f;
  for (int it = 0; it < 12; it++) {
    float ms = 0.f;
    if ((rc = p.timed([&] { probe_read_kernel<<<grid, 256, 0, p.st>>>(a, n, b); }, &ms))) return rc;
    if (it >= 2) best_r = std::min(best_r, ms);
    if ((rc = p.timed([&] { probe_copy_kernel<<<grid, 256, 0, p.st>>>(a, b, n); }, &ms))) return rc;
    if (it >= 2) best_c = std::min(best_c, ms);
  }
  if (read_gbps) *read_gbps = (double)bytes / (best_r * 1e-3) / 1e9;
  if (copy_gbps) *copy_gbps = 2.0 * (double)bytes / (best_c * 1e-3) / 1e9;
  return BS_OK;
}

// ---- MFMA probe (bench.py "mfma_measured"): dense bf16 matrix-core rate of this device.
// Every wave keeps 8 independent accumulator chains of v_mfma_f32_32x32x16_bf16 (16x16x32 for
// shape = 1) on register operands, 2 waves per SIMD (8 per CU) on a 4-block-per-CU grid: issue-bound
// on the matrix pipes, no memory traffic.  The result is stored only if it equals a value it never
// takes, which keeps the chains live.
typedef float f32x16 __attribute__((ext_vector_type(16)));
template <int SHAPE>
__global__ __launch_bounds__(128) void probe_mfma_kernel(int iters, float* sink) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    a[j] = (bf16)(1.0f + 0.001f * (float)((lane + j) & 7));
    b[j] = (bf16)(0.5f - 0.001f * (float)((lane * 3 + j) & 7));
  }
  float tot = 0.f;
  if constexpr (SHAPE == 0) {
    f32x16 acc[8];
#pragma unroll
    for (int c = 0; c < 8; c++) acc[c] = (f32x16){};
    for (int i = 0; i < iters; i++)
#pragma unroll
      for (int c = 0; c < 8; c++) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
#pragma unroll
    for (int c = 0; c < 8; c++)
#pragma unroll
      for (int j = 0; j < 16; j++) tot += acc[c][j];
  } else {
    f32x4 acc[8];
#pragma unroll
    for (int c = 0; c < 8; c++) acc[c] = (f32x4){};
    for (int i = 0; i < iters; i++)
#pragma unroll
      for (int c = 0; c < 8; c++) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[c], 0, 0, 0);
#pragma unroll
    for (int c = 0; c < 8; c++)
#pragma unroll
      for (int j = 0; j < 4; j++) tot += acc[c][j];
  }
  if (tot == -1.2345f) sink[blockIdx.x] = tot;
}

extern "C" int bs_mfma_probe(int32_t device, double* tflops_32x32x16, double* tflops_16x16x32) {
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  ProbeRes p;
  int rc = p.init(1u << 20, 1);
  if (rc) return rc;
  const int iters = 4096, blocks = prop.multiProcessorCount * 4;
  const double flops_per_iter[2] = {2.0 * 32 * 32 * 16, 2.0 * 16 * 16 * 32};  // per MFMA instruction
  double best[2] = {0.0, 0.0};
  for (int shape = 0; shape < 2; shape++) {
    for (int it = 0; it < 6; it++) {
      float ms = 0.f;
      rc = p.timed([&] {
        if (shape == 0) probe_mfma_kernel<0><<<blocks, 128, 0, p.st>>>(iters, (float*)p.buf[0]);
        else probe_mfma_kernel<1><<<blocks, 128, 0, p.st>>>(iters, (float*)p.buf[0]);
      }, &ms);
      if (rc) return rc;
      const double fl = (double)blocks * 2 /* waves */ * iters * 8 /* chains */ * flops_per_iter[shape];
      if (it >= 1) best[shape] = std::max(best[shape], fl / (ms * 1e-3) / 1e12);
    }
  }
  if (tflops_32x32x16) *tflops_32x32x16 = best[0];
  if (tflops_16x16x32) *tflops_16x16x32 = best[1];
  return BS_OK;
}

namespace {
struct ProfScope {
  bs_stage* s;
  hipStream_t st;
  bool on;
  ProfScope(bs_stage* s_, hipStream_t st_, int cls, double units) : s(s_), st(st_), on(s_->prof.cls == cls && cls) {
    if (on) {
      hipEventRecord(prof_event(s), st);
      s->prof.algo += units;
    }
  }
  ~ProfScope() {
    if (on) hipEventRecord(prof_event(s), st);
  }
};
}  // namespace

// Algorithmic bytes of one weight GEMV launch (decode): weights + bias + activations in/out.
static double gemv_bytes(const bs_stage* s, int M, int N, int K, int out_bytes) {
  return (double)N * K * s->esz + (double)N * s->esz + (double)M * K * s->esz + (double)M * N * out_bytes;
}

// The forward's GEMVs may split K through the stage's workspace (see kSkCap).
static Epi with_splitk(const bs_stage* s, const Epi& ep) {
  Epi e = ep;
  e.sk_ws = s->sk_ws; e.sk_tickets = s->sk_tickets; e.sk_cap = kSkCap; e.sk_ntickets = kSkTickets;
  return e;
}

static void linear(bs_stage* s, hipStream_t st, const void* X, const void* W, int M, int N, int K, const Epi& ep,
                   int out_bytes) {
  const bool decode = M <= 32 && s->bf16;
  if (decode) {
    ProfScope p(s, st, 1, gemv_bytes(s, M, N, K, out_bytes));
    launch_linear(s->bf16, X, W, M, N, K, ep, st);
  } else {
    ProfScope p(s, st, 2, 2.0 * M * N * K);
    launch_linear(s->bf16, X, W, M, N, K, ep, st);
  }
}

static void linear_ln(bs_stage* s, hipStream_t st, const float* x, int row_stride, int row_offset, const void* g,
                      const void* b, const void* W, int M, int N, int K, const Epi& ep, int out_bytes) {
  const bool decode = M <= 32 && s->bf16;
  if (decode) {
    ProfScope p(s, st, 1, gemv_bytes(s, M, N, K, out_bytes));
    launch_linear_ln(s->bf16, x, row_stride, row_offset, g, b, s->d.ln_eps, s->xn, W, M, N, K, ep, st);
  } else {
    ProfScope p(s, st, 2, 2.0 * M * N * K);
    launch_linear_ln(s->bf16, x, row_stride, row_offset, g, b, s->d.ln_eps, s->xn, W, M, N, K, ep, st);
  }
}

// Algorithmic bytes of one int8 weight GEMV launch: int8 weights + row scales + bias + activations.
static double gemv_bytes_q8(const bs_stage* s, int M, int N, int K, int out_bytes) {
  return (double)N * K + (double)N * 4 + (double)N * s->esz + (double)M * K * s->esz + (double)M * N * out_bytes;
}

// Block matrix t of a layer: int8 stages stream the int8 weights (launch_linear_q8).
static void wlinear(bs_stage* s, hipStream_t st, const void* X, const Layer& w, int t, int M, int N, int K,
                    const Epi& ep, int out_bytes) {
  if (!w.sc[t]) {
    linear(s, st, X, w.t[t], M, N, K, ep, out_bytes);
  } else if (M <= 32) {  // int8 GEMV / batched tile GEMV: weight-stream bound
    ProfScope p(s, st, 1, gemv_bytes_q8(s, M, N, K, out_bytes));
    launch_linear_q8(X, (const int8_t*)w.t[t], w.sc[t], s->wtmp, M, N, K, ep, st);
  } else {
    ProfScope p(s, st, 2, 2.0 * M * N * K);
    launch_linear_q8(X, (const int8_t*)w.t[t], w.sc[t], s->wtmp, M, N, K, ep, st);
  }
}

static void wlinear_ln(bs_stage* s, hipStream_t st, const float* x, const void* g, const void* b, const Layer& w,
                       int t, int M, int N, int K, const Epi& ep, int out_bytes) {
  if (!w.sc[t]) {
    linear_ln(s, st, x, 1, 0, g, b, w.t[t], M, N, K, ep, out_bytes);
    return;
  }
  if (linear_q8_ln_fused(M, K)) {
    ProfScope p(s, st, 1, gemv_bytes_q8(s, M, N, K, out_bytes));
    launch_linear_q8_ln(x, 1, 0, g, b, s->d.ln_eps, (const int8_t*)w.t[t], w.sc[t], M, N, K, ep, st);
    return;
  }
  launch_ln_rows(x, 1, 0, g, b, s->d.ln_eps, s->xn, M, K, st);
  wlinear(s, st, s->xn, w, t, M, N, K, ep, out_bytes);
}

// Device staging for logits requested with host I/O: one buffer per stage, grown on demand (a
// stream-ordered hipMallocAsync/hipFreeAsync pair per call handed blocks across the streams of
// two stages and returned zeros on ROCm 7.2; this is also cheaper).
static int logits_staging(bs_stage* s, size_t bytes, hipStream_t st, float** out) {
  if (bytes > s->logit_cap) {
    HIP_TRY(hipStreamSynchronize(st));
    if (s->logit_buf) HIP_TRY(hipFree(s->logit_buf));
    s->logit_buf = nullptr;
    s->logit_cap = 0;
    if (hipMalloc((void**)&s->logit_buf, bytes) != hipSuccess) return fail(BS_ERR_OOM, "logits staging allocation failed");
    s->logit_cap = bytes;
  }
  *out = s->logit_buf;
  return BS_OK;
}

// Enqueue one forward on `st`.  The kernels read each row's past_len from past_dev (device [B],
// written ahead of the forward or of the graph replay); `pasts` is the host copy (profiling bytes).
static int enqueue_forward(bs_stage* s, const bs_step* step, const void* in, void* out, float* logits, hipStream_t st,
                           const int* past_dev, const std::vector<int>& pasts) {
  const bs_stage_desc& d = s->d;
  const int B = step->batch, S = step->seq, slot = step->slot, past = pasts[0];
  double ctx_sum = 0.0;
  for (int b = 0; b < B; b++) ctx_sum += (double)pasts[b] + S;
  const int M = B * S;
  const bool want_logits = (step->flags & BS_STEP_LOGITS) != 0;
  const bool host_io = (step->flags & BS_STEP_HOST_IO) != 0;
  const int h = d.hidden, V = d.vocab, hd = s->hd, nh = d.n_head;

  // ---- input
  const float* cur = nullptr;
  const int* ids = nullptr;
  // bf16 decode of <= 2 rows: the embedding gather and its LayerNorm run in layer 0's LN + QKV kernel
  const bool emb_fused = d.is_first && s->bf16 && !s->q8 && M <= 2 && s->L > 0;
  if (d.is_first) {
    ids = (const int*)in;
    if (host_io) {
      HIP_TRY(hipMemcpyAsync(s->ids, ids, (size_t)M * 4, hipMemcpyHostToDevice, st));
      ids = s->ids;
    }
    if (!emb_fused) launch_layernorm(s->bf16, s->wemb, ids, 0, 0, s->emb_g, s->emb_b, s->xa, 1, M, h, d.ln_eps, st);
    cur = s->xa;
  } else if (host_io) {
    HIP_TRY(hipMemcpyAsync(s->xa, in, (size_t)M * h * 4, hipMemcpyHostToDevice, st));
    cur = s->xa;
  } else {
    cur = (const float*)in;
  }

  // ---- decoder blocks
  const float inv_norm = 1.0f / std::sqrt((float)hd);
  for (int l = 0; l < s->L; l++) {
    const Layer& w = s->layers[l];
    char* kbase = s->kv + l * s->kv_layer_stride;
    // x1 = LN_in(x); fused QKV (+bias) -> q, K/V cache
    Epi e{};
    e.kind = EPI_QKV; e.bias = w.t[T_QKV_B]; e.q_out = s->q; e.k_cache = kbase; e.v_cache = kbase + s->kv_half;
    e.hidden = h; e.head_dim = hd; e.max_ctx = d.max_ctx; e.n_head = nh; e.seq = S; e.slot = slot; e.past = past;
    e.past_dev = past_dev; e.ldo = 3 * h;
    bool done = false;
    if (l == 0 && emb_fused) {
      ProfScope p(s, st, 1, gemv_bytes(s, M, 3 * h, h, 4) + (double)M * h * (s->esz + 4));
      done = launch_linear_emb(ids, s->wemb, s->emb_g, s->emb_b, s->xa, w.t[T_LN1_G], w.t[T_LN1_B], d.ln_eps,
                               w.t[T_QKV_W], M, 3 * h, h, with_splitk(s, e), st);
      if (!done) launch_layernorm(s->bf16, s->wemb, ids, 0, 0, s->emb_g, s->emb_b, s->xa, 1, M, h, d.ln_eps, st);
    }
    if (!done) wlinear_ln(s, st, cur, w.t[T_LN1_G], w.t[T_LN1_B], w, T_QKV_W, M, 3 * h, h, with_splitk(s, e), 4);
    // attention
    AttnArgs a{};
    a.q = s->q; a.k_cache = kbase; a.v_cache = kbase + s->kv_half; a.ctx_out = s->ctx; a.slopes = s->slopes;
    a.B = B; a.S = S; a.slot = slot; a.past = past; a.past_dev = past_dev; a.n_head = nh; a.head_dim = hd;
    a.max_ctx = d.max_ctx; a.hidden = h; a.inv_norm = inv_norm; a.part_acc = s->part_acc; a.part_ml = s->part_ml;
    a.max_chunks = s->max_chunks; a.chunk = s->chunk; a.tickets = s->att_tickets;
    // prefill: the long query tiles' keys split over blocks of 4 key tiles, partials in the GEMM split-K
    // workspace (free between the QKV GEMM and the dense GEMM on this stream)
    a.pf_tiles = 4; a.pf_ws = s->sk_ws; a.pf_cap = kSkCap; a.pf_tickets = s->sk_tickets; a.pf_ntickets = kSkTickets;
    a.pf_past_max = *std::max_element(pasts.begin(), pasts.end());
    // a split decode context merges in the dense GEMV's prologue when that kernel can take it
    const int nsplit = S == 1 ? attention_decode_splits(B, nh, s->max_chunks) : 1;
    a.defer_merge = s->bf16 && nsplit > 1 &&
                    (w.sc[T_DENSE_W] ? linear_q8_parts_supported(M, h, hd, nsplit)
                                     : linear_parts_supported(M, h, hd, nsplit));
    // a = x + dense(ctx)
    Epi e2{};
    e2.kind = EPI_RESID; e2.bias = w.t[T_DENSE_B]; e2.out_f32 = s->attn; e2.resid = cur; e2.ldo = h;
    {
      ProfScope p(s, st, 3, ctx_sum * nh * hd * 2 * s->esz);
      launch_attention(s->bf16, a, st);
    }
    if (a.defer_merge) {
      const AttnParts parts{s->part_acc, s->part_ml, nsplit, nh, hd, s->max_chunks, slot};
      ProfScope p(s, st, 1, w.sc[T_DENSE_W] ? gemv_bytes_q8(s, M, h, h, 4) : gemv_bytes(s, M, h, h, 4));
      if (w.sc[T_DENSE_W]) launch_linear_q8_parts(parts, (const int8_t*)w.t[T_DENSE_W], w.sc[T_DENSE_W], M, h, h, e2, st);
      else launch_linear_parts(parts, w.t[T_DENSE_W], M, h, h, e2, st);
    } else {
      wlinear(s, st, s->ctx, w, T_DENSE_W, M, h, h, with_splitk(s, e2), 4);
    }
    // x2 = LN_post(a); g = gelu(x2 W1 + b1)
    Epi e3{};
    e3.kind = EPI_GELU; e3.bias = w.t[T_FC1_B]; e3.out_act = s->g; e3.ldo = 4 * h;
    wlinear_ln(s, st, s->attn, w.t[T_LN2_G], w.t[T_LN2_B], w, T_FC1_W, M, 4 * h, h, with_splitk(s, e3), (int)s->esz);
    // x = a + g W2 + b2
    float* nxt = (!d.is_last && !host_io && l == s->L - 1) ? (float*)out : (cur == s->xa ? s->xb : s->xa);
    Epi e4{};
    e4.kind = EPI_RESID; e4.bias = w.t[T_FC2_B]; e4.out_f32 = nxt; e4.resid = s->attn; e4.ldo = h;
    wlinear(s, st, s->g, w, T_FC2_W, M, h, 4 * h, with_splitk(s, e4), 4);
    cur = nxt;
  }

  // ---- output
  if (d.is_last && s->n_labels) {
    // sequence-classification tail (run_inference_with_binary_classification, inference.cpp:220-270): ln_f on each
    // row's last position, score, first maximal class; the class kernel is the step's last (advances past_dev)
    float* dev_logits = want_logits && !host_io ? logits : nullptr;
    if (want_logits && host_io) {
      int rc = logits_staging(s, (size_t)B * s->n_labels * 4, st, &dev_logits);
      if (rc != BS_OK) return rc;
    }
    launch_layernorm(s->bf16, cur, nullptr, S, S - 1, s->lnf_g, s->lnf_b, s->xn, 0, B, h, d.ln_eps, st);
    int* cls_out = host_io ? s->tok : (int*)out;
    launch_classify(s->bf16, s->xn, s->score, B, s->n_labels, h, dev_logits, cls_out, s->past_dev, S, st);
    if (host_io) {
      HIP_TRY(hipMemcpyAsync(out, s->tok, (size_t)B * 4, hipMemcpyDeviceToHost, st));
      if (dev_logits)
        HIP_TRY(hipMemcpyAsync(logits, dev_logits, (size_t)B * s->n_labels * 4, hipMemcpyDeviceToHost, st));
    }
  } else if (d.is_last) {
    // ln_f on each row's last position, tied lm_head, token pick (greedy argmax or top-k sample)
    const bool sample = s->top_k > 1;
    Epi e{};
    e.kind = EPI_ARGMAX; e.keys = s->keys; e.logits = want_logits && !host_io ? logits : nullptr; e.ldo = V;
    e.key_hi_index = sample ? 1 : 0;  // sampling ranks equal logits by the higher index (decoding.cpp:44-45)
    float* dev_logits = nullptr;
    if (want_logits && host_io) {
      int rc = logits_staging(s, (size_t)B * V * 4, st, &dev_logits);
      if (rc != BS_OK) return rc;
      e.logits = dev_logits;
    }
    if (sample && !e.logits) e.logits = s->sample_logits;
    linear_ln(s, st, cur, S, S - 1, s->lnf_g, s->lnf_b, s->wemb, B, V, h, with_splitk(s, e), 0);
    int* tok_out = host_io ? s->tok : (int*)out;
    // the pick is the step's last kernel: it advances the device copy of every row's past_len by S
    if (sample)
      launch_topk_sample(s->keys, V / 16, e.logits, V, B, s->top_k, 1.0f / s->temperature, s->sample_seed, slot,
                         past_dev, S, tok_out, st, s->past_dev);
    else
      launch_argmax_finalize(s->keys, B, V / 16, nullptr, nullptr, tok_out, st, s->past_dev, S);
    if (host_io) {
      HIP_TRY(hipMemcpyAsync(out, s->tok, (size_t)B * 4, hipMemcpyDeviceToHost, st));
      if (dev_logits) HIP_TRY(hipMemcpyAsync(logits, dev_logits, (size_t)B * V * 4, hipMemcpyDeviceToHost, st));
    }
  } else if (host_io) {
    HIP_TRY(hipMemcpyAsync(out, cur, (size_t)M * h * 4, hipMemcpyDeviceToHost, st));
  } else if (s->L == 0) {
    HIP_TRY(hipMemcpyAsync(out, cur, (size_t)M * h * 4, hipMemcpyDeviceToDevice, st));
  }
  return BS_OK;
}

extern "C" int bs_head_norm(bs_stage* s, const float* hidden, int32_t B, int32_t S, void* xn, void* stream) {
  if (!s || !hidden || !xn) return fail(BS_ERR_INVALID, "stage/hidden/xn is NULL");
  if (!s->lnf_g) return fail(BS_ERR_STATE, "stage has no ln_f (needs is_last or a head slice)");
  if (B <= 0 || S <= 0 || B > s->d.max_batch) return fail(BS_ERR_INVALID, "bad batch/seq");
  HIP_TRY(hipSetDevice(s->d.device));
  hipStream_t st = stream ? (hipStream_t)stream : s->own;
  launch_layernorm(s->bf16, hidden, nullptr, S, S - 1, s->lnf_g, s->lnf_b, xn, 0, B, s->d.hidden, s->d.ln_eps, st);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return fail(BS_ERR_DEVICE, std::string("head_norm: ") + hipGetErrorString(err));
  return BS_OK;
}

extern "C" int bs_head_slice(bs_stage* s, const void* xn, int32_t B, const uint64_t* keys_in, uint64_t* keys_out,
                             int32_t* tokens, void* stream) {
  if (!s || !xn) return fail(BS_ERR_INVALID, "stage/xn is NULL");
  if (!s->hw || s->hv1 <= s->hv0) return fail(BS_ERR_STATE, "stage has no head slice");
  if (B <= 0 || B > s->d.max_batch) return fail(BS_ERR_INVALID, "bad batch");
  HIP_TRY(hipSetDevice(s->d.device));
  hipStream_t st = stream ? (hipStream_t)stream : s->own;
  const int n = s->hv1 - s->hv0;
  Epi e{};
  e.kind = EPI_ARGMAX; e.keys = s->keys; e.ldo = n; e.col_offset = s->hv0;
  linear(s, st, xn, s->hw, B, n, s->d.hidden, e, 0);
  launch_argmax_finalize(s->keys, B, n / 16, (const unsigned long long*)keys_in, (unsigned long long*)keys_out,
                         tokens, st);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return fail(BS_ERR_DEVICE, std::string("head_slice: ") + hipGetErrorString(err));
  return BS_OK;
}

extern "C" int bs_set_sampling(bs_stage* s, int32_t top_k, float temperature, uint64_t seed) {
  if (!s) return fail(BS_ERR_INVALID, "stage is NULL");
  if (top_k > 16) return fail(BS_ERR_UNSUPPORTED, "top_k must be <= 16");
  if (top_k > 1 && (!s->d.is_last || s->n_labels))
    return fail(BS_ERR_UNSUPPORTED, "sampling needs the last stage of a generation model (whole lm_head)");
  if (top_k > 1 && !(temperature > 0.f)) return fail(BS_ERR_INVALID, "temperature must be positive");
  HIP_TRY(hipSetDevice(s->d.device));
  if (top_k > 1 && !s->sample_logits) {
    HIP_TRY(hipStreamSynchronize(s->own));
    if (hipMalloc((void**)&s->sample_logits, (size_t)s->d.max_batch * s->d.vocab * 4) != hipSuccess)
      return fail(BS_ERR_OOM, "sampling logits allocation failed");
  }
  s->top_k = top_k < 1 ? 1 : top_k;
  s->temperature = top_k > 1 ? temperature : 1.f;
  s->sample_seed = seed;
  // captured decode graphs hold the old pick as kernel arguments
  HIP_TRY(hipDeviceSynchronize());
  for (auto& g : s->graphs) hipGraphExecDestroy(g.second);
  s->graphs.clear();
  return BS_OK;
}

extern "C" int bs_set_graphs(bs_stage* s, int32_t on) {
  if (!s) return fail(BS_ERR_INVALID, "stage is NULL");
  HIP_TRY(hipSetDevice(s->d.device));
  HIP_TRY(hipDeviceSynchronize());
  for (auto& g : s->graphs) hipGraphExecDestroy(g.second);
  s->graphs.clear();
  s->graphs_on = on ? 1 : 0;
  return BS_OK;
}

extern "C" int bs_forward(bs_stage* s, const bs_step* step, const void* in, void* out, float* logits, void* stream) {
  if (!s || !step) return fail(BS_ERR_INVALID, "stage/step is NULL");
  const bs_stage_desc& d = s->d;
  const int B = step->batch, S = step->seq, slot = step->slot;
  const int M = B * S;
  if (B <= 0 || S <= 0) return fail(BS_ERR_INVALID, "batch and seq must be positive");
  if (slot < 0 || slot + B > d.max_batch) return fail(BS_ERR_INVALID, "slot range outside max_batch");
  std::vector<int> pasts(B);
  for (int b = 0; b < B; b++) {
    pasts[b] = step->past_lens ? step->past_lens[b] : step->past_len;
    if (pasts[b] < 0 || pasts[b] + S > d.max_ctx) return fail(BS_ERR_INVALID, "past_len + seq exceeds max_ctx");
  }
  if (M > d.max_tokens) return fail(BS_ERR_INVALID, "batch*seq exceeds max_tokens");
  if (!in || !out) return fail(BS_ERR_INVALID, "in/out is NULL");
  const bool want_logits = (step->flags & BS_STEP_LOGITS) != 0;
  if (want_logits && (!d.is_last || !logits)) return fail(BS_ERR_INVALID, "logits requested on a non-last stage or NULL");
  const bool host_io = (step->flags & BS_STEP_HOST_IO) != 0;
  if (d.is_first && host_io) {
    const int* ids = (const int*)in;
    for (int i = 0; i < M; i++)
      if (ids[i] < 0 || ids[i] >= d.vocab) return fail(BS_ERR_INVALID, "token id out of range");
  }
  BS_TRACE("B=%d S=%d slot=%d flags=%u stream=%p hipSetDevice", B, S, slot, (unsigned)step->flags, stream);
  HIP_TRY(hipSetDevice(d.device));
  hipStream_t st = stream ? (hipStream_t)stream : s->own;

  // Decode steps on device buffers replay a captured hipGraph: the kernels read past_len from
  // device memory, set by one small kernel ahead of the replay -- unless the last forward (a last
  // stage's, whose token pick advances past_dev by its seq) already left exactly these values there,
  // on this same stream: a forward on another stream is not ordered behind that advance, so it always
  // writes its own positions.
  const bool past_matches = s->past_next_valid && s->past_stream == st && (int)s->past_next.size() == B &&
                            std::equal(pasts.begin(), pasts.end(), s->past_next.begin());
  s->past_next_valid = false;  // until this forward is enqueued
  const bool graph = S == 1 && !host_io && s->prof.cls == 0 && s->graphs_on;
  if (graph) {
    GraphKey key{B, slot, step->flags, in, out, logits, st};
    hipGraphExec_t exec = nullptr;
    for (auto& g : s->graphs)
      if (g.first == key) { exec = g.second; break; }
    if (!exec) {
      hipGraph_t gr = nullptr;
      BS_TRACE("hipStreamBeginCapture");
      HIP_TRY(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
      BS_TRACE("enqueue_forward (capturing)");
      int rc = enqueue_forward(s, step, in, out, logits, st, s->past_dev, pasts);
      BS_TRACE("hipStreamEndCapture");
      hipError_t ce = hipStreamEndCapture(st, &gr);
      if (rc != BS_OK) { if (gr) hipGraphDestroy(gr); return rc; }
      if (ce != hipSuccess) return fail(BS_ERR_DEVICE, std::string("graph capture: ") + hipGetErrorString(ce));
      BS_TRACE("hipGraphInstantiate");
      hipError_t ie = hipGraphInstantiate(&exec, gr, nullptr, nullptr, 0);
      BS_TRACE("hipGraphDestroy");
      hipGraphDestroy(gr);
      if (ie != hipSuccess) return fail(BS_ERR_DEVICE, std::string("graph instantiate: ") + hipGetErrorString(ie));
      if (s->graphs.size() >= 64) {
        hipGraphExecDestroy(s->graphs.front().second);
        s->graphs.erase(s->graphs.begin());
      }
      s->graphs.push_back({key, exec});
    }
    if (!past_matches) {
      BS_TRACE("set_past launch");
      launch_set_past(s->past_dev, pasts.data(), B, st);
    }
    BS_TRACE("hipGraphLaunch");
    HIP_TRY(hipGraphLaunch(exec, st));
  } else {
    if (!past_matches) {
      BS_TRACE("set_past launch");
      launch_set_past(s->past_dev, pasts.data(), B, st);
    }
    BS_TRACE("enqueue_forward (eager)");
    int rc = enqueue_forward(s, step, in, out, logits, st, s->past_dev, pasts);
    if (rc != BS_OK) return rc;
  }
  BS_TRACE("hipGetLastError");
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return fail(BS_ERR_DEVICE, std::string("kernel launch: ") + hipGetErrorString(err));
  if (d.is_last) {  // the last kernel advanced past_dev[0..B) by S (stream-ordered before the next forward)
    s->past_next.assign(pasts.begin(), pasts.end());
    for (int& p : s->past_next) p += S;
    s->past_next_valid = true;
    s->past_stream = st;
  }
  if (host_io) {
    BS_TRACE("hipStreamSynchronize");
    HIP_TRY(hipStreamSynchronize(st));
  }
  BS_TRACE("done");
  return BS_OK;
}
