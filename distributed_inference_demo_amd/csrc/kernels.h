// kernels.h — host-side launch wrappers for the stage kernels (implemented in kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Epilogue of every weight GEMM/GEMV: y[m][n] = sum_k X[m][k] * W[n][k] (+ what `kind` says).
enum EpiKind : int {
  EPI_QKV = 0,     // + bias; q -> q_out (T) [M][h]; k,v -> KV cache (T) at (slot+b, past+t)
  EPI_RESID = 1,   // out_f32[m][n] = (y + bias) + resid[m][n]
  EPI_GELU = 2,    // out_act[m][n] = T(gelu(y + bias))
  EPI_ARGMAX = 3,  // no bias; 64-bit atomicMax of (order(y), ~n) into keys[m]; optional logits
};

struct Epi {
  int kind;
  const void* bias;       // T [N]
  float* out_f32;         // EPI_RESID output [M][ldo]
  void* out_act;          // EPI_GELU output (T) [M][ldo]
  const float* resid;     // EPI_RESID residual [M][ldo]
  int ldo;                // leading dim of out/resid (= N)
  // EPI_QKV
  void* q_out;            // T [M][hidden]
  void* k_cache;          // T, layer base of K: [max_batch][heads][max_ctx][hd]
  void* v_cache;
  int hidden, head_dim, max_ctx, n_head;
  int seq, slot;
  const int* past_dev;    // device past_len per row b = m / seq (graph-replayable); used when non-null
  int past;               // host past_len of every row otherwise
  // EPI_ARGMAX
  unsigned long long* keys;  // [M][N/16]: max over each 16-column tile
  float* logits;          // optional [M][ldo]
  int col_offset;         // vocabulary index of column 0 (head slices)
  int key_hi_index;       // 0: keys rank equal logits by the LOWER index (greedy, torch.argmax);
                          // 1: by the HIGHER index (top-k sampling, decoding.cpp:44-45 std::greater)
  // split-K workspace of the batched GEMV (gemv_tiles): fp32 partials [ks][M][N] (capacity in
  // floats) and one arrival ticket per 16-column tile (zero between launches).  Null: no split-K.
  float* sk_ws;
  unsigned* sk_tickets;
  size_t sk_cap;
  int sk_ntickets;
  // int8 weights: y[m][n] *= col_scale[n] before the epilogue (the weight operand held Q, not
  // Q * scale).  Null otherwise.  Not applied by EPI_ARGMAX.
  const float* col_scale;
};

// dtype tag: 0 = fp32, 1 = bf16
void launch_gen_fill(void* dst, int is_bf16, uint64_t n, uint64_t key, int kind, hipStream_t s,
                     uint64_t index_offset = 0);
void launch_convert_f32(void* dst, int is_bf16, const float* src, uint64_t n, hipStream_t s);

// LayerNorm rows: out[m] (T, or fp32 when out_f32) = LN(x[m*row_stride + row_offset]) with
// gamma/beta (T); x is fp32 [.][K].  If ids != null, row m is instead gathered from the
// embedding table `x` (T) [vocab][K] at ids[m] (word_embeddings + word_embeddings_layernorm).
void launch_layernorm(int is_bf16, const void* x, const int* ids, int row_stride, int row_offset,
                      const void* gamma, const void* beta, void* out, int out_f32, int M, int K,
                      float eps, hipStream_t s);

// Weight GEMM: X (T) [M][K] x W (T) [N][K]^T with epilogue.
void launch_linear(int is_bf16, const void* X, const void* W, int M, int N, int K, const Epi& ep,
                   hipStream_t s);

// LayerNorm(x rows) followed by a weight GEMM; fused into one kernel on the bf16 decode path.
void launch_linear_ln(int is_bf16, const float* x, int row_stride, int row_offset, const void* gamma,
                      const void* beta, float eps, void* xn_scratch, const void* W, int M, int N, int K,
                      const Epi& ep, hipStream_t s);

// The first stage's layer 0 at M <= 2 (bf16): word_embeddings[ids] -> word_embeddings_layernorm (fp32,
// stored to x_out: the residual stream) -> LN_in -> weight GEMV, one kernel.  False: not launched.
bool launch_linear_emb(const int* ids, const void* wemb, const void* emb_g, const void* emb_b, float* x_out,
                       const void* gamma, const void* beta, float eps, const void* W, int M, int N, int K,
                       const Epi& ep, hipStream_t s);

// Attention over the KV cache for B rows x S new queries per row (causal, ALiBi).
struct AttnArgs {
  const void* q;       // T [B*S][hidden]
  const void* k_cache; // T layer base
  const void* v_cache;
  void* ctx_out;       // T [B*S][hidden]
  const float* slopes; // [n_head]
  int B, S, slot;
  const int* past_dev; // device past_len per row [B] (graph-replayable) or null
  int past;
  int n_head, head_dim, max_ctx, hidden;
  float inv_norm;
  float* part_acc;     // workspace [max_batch][n_head][max_chunks][head_dim] (row = slot + b)
  float* part_ml;      // workspace [max_batch][n_head][max_chunks][2]
  int max_chunks;
  int chunk;           // positions per chunk (decode) = 64
  unsigned* tickets;   // [max_batch][n_head] split-merge tickets (zero between launches)
  int defer_merge;     // decode split > 1: leave the partials for the consumer (launch_linear_parts)
  // prefill (S > 1) split-KV: key tiles of a 64-query tile spread over blocks of `pf_tiles` 64-key
  // tiles each (0: no split); partials [item][split][64 queries][4 + head_dim] in pf_ws (pf_cap floats), one
  // ticket per (row, head, query tile) in pf_tickets (zero between launches, pf_ntickets of them)
  int pf_tiles;
  float* pf_ws;
  size_t pf_cap;
  unsigned* pf_tickets;
  int pf_ntickets;
  int pf_past_max;     // largest past_len of the call's rows (sizes the split grid)
};
void launch_attention(int is_bf16, const AttnArgs& a, hipStream_t s);
// S > 1, bf16, head_dim <= 128 (attn_prefill.hip): NSTG LDS stages (2 or 3), split-KV over blocks of pf_tiles key tiles
// (-1: a.pf_tiles) when the grid has fewer than max_units blocks; kgroups key groups per block (1 or 2; -1: by shape);
// qgroups query groups of 16 per wave (1 or 2 = 128-query blocks, no key split; -1: by shape).
void attn_prefill_tr_launch(const AttnArgs& a, hipStream_t s, int nstg = 2, int pf_tiles = -1, int max_units = 256,
                            int kgroups = -1, int qgroups = -1);
size_t attention_workspace_floats(int B, int n_head, int head_dim, int max_ctx, int* max_chunks, int* chunk);
// Context splits per (row, head) of a decode attention launch (1 = the block writes ctx itself).
int attention_decode_splits(int B, int n_head, int max_chunks);

// Split-attention partials as the consumer reads them (attn_merge.h).
struct AttnParts {
  const float* acc;  // AttnArgs::part_acc
  const float* ml;   // AttnArgs::part_ml
  int nsplit, n_head, head_dim, max_chunks, slot;
};
// Can launch_linear_parts run M rows of a K-wide ctx split `nsplit` ways?
bool linear_parts_supported(int M, int K, int head_dim, int nsplit);
// Weight GEMV on ctx = merge(partials) (bf16): the dense projection after a deferred-merge attention.
void launch_linear_parts(const AttnParts& p, const void* W, int M, int N, int K, const Epi& ep, hipStream_t s);

// keys -> token ids
// Reduce the per-tile keys of each row (and keys_in[m] if given) -> keys_out[m] / tokens[m] (either optional).
// past_adv (optional): past_adv[m] += seq for every row (the decode step's last kernel advances the
// device copy of the cached lengths; stage.hip skips set_past when the host's next step matches it).
void launch_argmax_finalize(const unsigned long long* keys, int M, int ntiles, const unsigned long long* keys_in,
                            unsigned long long* keys_out, int* tokens, hipStream_t s, int* past_adv = nullptr,
                            int seq = 0);
// Sequence-classification head: xn (T) [M][K] . score (T) [n_labels][K] -> logits fp32 [M][n_labels] (optional),
// cls[m] = first maximal label (inference.cpp:57-69); past_adv[m] += seq (optional).  n_labels <= 64, K % 8 == 0.
void launch_classify(int is_bf16, const void* xn, const void* score, int M, int n_labels, int K, float* logits,
                     int* cls, int* past_adv, int seq, hipStream_t s);
// past_dev[0..n) = values[0..n) (host), stream ordered, by kernel arguments (graph-capturable).
// Seeded top-k sampling (include/bloomstage.h bs_set_sampling; decoding.cpp:24-66) of M rows from the
// per-16-column tile keys (key_hi_index = 1) and the logits they came from ([M][ldl], column = vocab index).
// Row b's draw is keyed by (seed, KV row slot + b, position past_dev[b] + seq).
void launch_topk_sample(const unsigned long long* keys, int ntiles, const float* logits, int ldl, int M, int k,
                        float inv_temp, uint64_t seed, int slot, const int* past_dev, int seq, int* tokens,
                        hipStream_t s, int* past_adv = nullptr);
void launch_set_past(int* past_dev, const int* values, int n, hipStream_t s);

// ---- Weight-only int8 (bf16 stages with BS_FLAG_INT8_WEIGHTS; kernels.hip "Weight-only int8") ----
// Q[n][k] = rne(W[n][k] / scale[n]), scale[n] = max_k |W[n][k]| / 127 (1 for a zero row); W bf16 [N][K].
void launch_quantize_rows(const void* W_bf16, int8_t* Q, float* scale, int N, int K, hipStream_t s);
// out bf16 [N][K] = Q * scale (row-wise).
void launch_dequant_rows(const int8_t* Q, const float* scale, void* out_bf16, int N, int K, hipStream_t s);
// Does launch_linear_q8 run M rows of a K-wide GEMV straight from the int8 weights?
bool linear_q8_gemv(int M, int K);
// X bf16 [M][K] x (Q * scale)^T with epilogue (not EPI_ARGMAX).  M <= 8: int8 GEMV; otherwise Q is
// dequantized into w_scratch (bf16, N*K) and the bf16 GEMM runs on it.
void launch_linear_q8(const void* X, const int8_t* Q, const float* scale, void* w_scratch, int M, int N, int K,
                      const Epi& ep, hipStream_t s);
// The int8 dense GEMV on ctx = merge(split-attention partials) (M <= 2): the int8 counterpart of
// launch_linear_parts.
bool linear_q8_parts_supported(int M, int K, int head_dim, int nsplit);
void launch_linear_q8_parts(const AttnParts& p, const int8_t* Q, const float* scale, int M, int N, int K,
                            const Epi& ep, hipStream_t s);
// M <= 4, K <= 4096: LayerNorm(x rows) fused into the int8 GEMV prologue (rows normalised to LDS).
bool linear_q8_ln_fused(int M, int K);
void launch_linear_q8_ln(const float* x, int row_stride, int row_offset, const void* gamma, const void* beta,
                         float eps, const int8_t* Q, const float* scale, int M, int N, int K, const Epi& ep,
                         hipStream_t s);
// LayerNorm of M fp32 rows -> bf16 (register-resident one-block-per-row kernel when K <= 4096).
void launch_ln_rows(const float* x, int row_stride, int row_offset, const void* gamma, const void* beta, float eps,
                    void* out_bf16, int M, int K, hipStream_t s);
