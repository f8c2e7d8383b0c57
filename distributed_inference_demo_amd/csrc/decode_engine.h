// decode_engine.h — persistent single-launch decode step of one pipeline stage (gfx950).
//
// One workgroup (512 threads) per CU walks the whole stage for a decode step (S = 1, B <= 4):
// for every layer  LN_in+QKV -> attention -> dense(+res) -> LN_post+fc1(+GELU) -> fc2(+res),
// then (last stage) ln_f + lm_head + argmax.  Each GEMV phase gives every workgroup a fixed
// slice of weight rows; the slice of the NEXT phase is requested into registers before the
// workgroup waits for the phase's input, so the weight stream runs through every dependency
// wait.  Inputs cross workgroups through write-through (sc1) stores + agent-scope counters
// (MI355X_MICROARCH.md, Guideline 16 row 1); no grid barrier, no fences, no atomics on data.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;

struct DeLayer {
  const bf16 *ln1_g, *ln1_b, *wqkv, *bqkv, *wo, *bo, *ln2_g, *ln2_b, *w1, *b1, *w2, *b2;
  bf16* kc;  // K cache base of the layer: [max_batch][n_head][max_ctx][head_dim]
  bf16* vc;
};

struct DeArgs {
  const DeLayer* layers;  // device array [L]
  int L, M, h, nh, hd, max_ctx, slot, past;
  unsigned kv_half_bytes;  // vc - kc of every layer (V cache follows K)
  float eps, inv_norm;
  const float* slopes;
  // input: first stage -> token ids (+ embedding table and its LayerNorm), else fp32 hidden [M][h]
  const int* ids;
  const bf16 *wemb, *emb_g, *emb_b;
  const float* x_in;
  float* x_out;  // non-last stage: fp32 hidden [M][h] out (may be null -> workspace)
  // workspace
  float *xb0, *xb1, *attn, *x0;  // fp32 [M][h]
  bf16 *q, *ctx, *g;             // [M][h], [M][h], [M][4h]
  float* part;                   // attention partials [units][hd + 2]
  // head (last stage or head slice)
  int has_head;
  const bf16 *lnf_g, *lnf_b, *whead;
  int head_rows, col_offset;
  unsigned long long* wgkeys;          // [grid][4]
  const unsigned long long* keys_in;   // [M] or null
  unsigned long long* keys_out;        // [M] or null
  int* tokens;                         // [M] or null
  float* logits;                       // [M][ldl] or null
  int ldl;
  // in-launch synchronisation state (zero between launches; the last workgroup re-zeroes it)
  unsigned* ctr;  // edge counters [L*5][8 shards][16 words]
  int n_ctr_words;
  unsigned* tick;  // attention merge tickets [L][4][n_head]
  int n_tick_words;
  unsigned* fin;   // final ticket (16 words)
  unsigned* err;      // abort flag of the running launch (re-zeroed by its last workgroup)
  unsigned* err_log;  // sticky give-up codes, read and cleared by the host (bs_engine_status)
  // diagnostics: per-workgroup s_memrealtime stamps at phase boundaries (null = off)
  unsigned long long* trace;
  int trace_stride;
  // LDS carve (bytes)
  int lds_res, lds_scr, maxrows;
};

// Host side.  engine_prepare: kernel attributes + residency check for `lds` bytes of LDS;
// returns the workgroup count to launch (one per CU) or 0 when the engine cannot run.
int engine_prepare(int mm, size_t lds, int device);
size_t engine_lds_bytes(int mm, int h, int maxrows);
void engine_launch(const DeArgs& a, int mm, int grid, size_t lds, hipStream_t s);
