/*
 * oracle/gen.h — TEST INFRASTRUCTURE (CPU checker only; never linked into the product).
 *
 * Deterministic synthetic-weight generator, C restatement.  This is the repo's data
 * spec (DESIGN.md §"Synthetic weights"), implemented three times independently:
 *   - here (C, used by the oracle stage forward and the CPU baseline),
 *   - oracle/gen_np.py (numpy, used to build HF golden fixtures),
 *   - distributed_inference_demo_amd/csrc/gen.hip (device, the product path).
 * The tests check that all three agree bit for bit.
 *
 * Distribution choices follow SURVEY.md §8(d) "Synthetic inputs" (Linear/Embedding ~
 * N(0,0.02) i.e. HF initializer_range, biases ~ U(-0.02,0.02), LN gamma ~ 1+U(-0.1,0.1),
 * beta ~ U(-0.1,0.1)).  "Normal" is an Irwin-Hall sum of four 16-bit uniforms so every
 * implementation is exact integer arithmetic + one float rounding.
 * Compile with -ffp-contract=off (gamma = 1 + t must not fuse).
 */
#ifndef BS_ORACLE_GEN_H
#define BS_ORACLE_GEN_H
#include <stdint.h>

#define GEN_NSC 0x1.1bc77ap-22f  /* 0.02 / sd(2*sum4(u16) - 4*65535) */
#define GEN_U002 0x1.47ae14p-30f /* 0.02 / 2^24 */
#define GEN_U010 0x1.99999ap-28f /* 0.1  / 2^24 */

/* tensor ids, model level (layer = -1) */
enum { GT_WEMB = 0, GT_EMB_G = 1, GT_EMB_B = 2, GT_LNF_G = 3, GT_LNF_B = 4, GT_SCORE = 5, GT_PROMPT = 255 };
/* tensor ids, per layer */
enum {
  GT_LN1_G = 0, GT_LN1_B, GT_QKV_W, GT_QKV_B, GT_DENSE_W, GT_DENSE_B,
  GT_LN2_G, GT_LN2_B, GT_FC1_W, GT_FC1_B, GT_FC2_W, GT_FC2_B, GT_NUM_LAYER_TENSORS
};

static inline uint64_t gen_sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
static inline uint32_t gen_lb32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
static inline uint64_t gen_tensor_key(uint64_t seed, int layer, uint32_t tid) {
  return gen_sm64(seed ^ gen_sm64(((uint64_t)(uint32_t)(layer + 1) << 8) | tid));
}
static inline uint32_t gen_bits(uint64_t key, uint32_t i) {
  return gen_lb32((uint32_t)key ^ gen_lb32(i + (uint32_t)(key >> 32)));
}
/* approx N(0, 0.02) */
static inline float gen_normal(uint64_t key, uint32_t i) {
  uint32_t h1 = gen_bits(key, i), h2 = gen_bits(gen_sm64(key), i);
  int32_t s = 2 * (int32_t)((h1 & 0xFFFFu) + (h1 >> 16) + (h2 & 0xFFFFu) + (h2 >> 16)) - 4 * 65535;
  return (float)s * GEN_NSC;
}
/* U(-a, a) with scale = a / 2^24 */
static inline float gen_uniform(uint64_t key, uint32_t i, float scale) {
  int32_t s = 2 * (int32_t)(gen_bits(key, i) >> 8) - 16777215;
  return (float)s * scale;
}
/* kind: 0 normal(0.02), 1 bias U(0.02), 2 gamma 1+U(0.1), 3 beta U(0.1) */
static inline float gen_value(int kind, uint64_t key, uint32_t i) {
  switch (kind) {
    case 0: return gen_normal(key, i);
    case 1: return gen_uniform(key, i, GEN_U002);
    case 2: { float t = gen_uniform(key, i, GEN_U010); return 1.0f + t; }
    default: return gen_uniform(key, i, GEN_U010);
  }
}
static inline int gen_layer_kind(int tid) {
  switch (tid) {
    case GT_LN1_G: case GT_LN2_G: return 2;
    case GT_LN1_B: case GT_LN2_B: return 3;
    case GT_QKV_W: case GT_DENSE_W: case GT_FC1_W: case GT_FC2_W: return 0;
    default: return 1;
  }
}
static inline int gen_model_kind(int tid) {
  switch (tid) {
    case GT_WEMB: case GT_SCORE: return 0;
    case GT_EMB_G: case GT_LNF_G: return 2;
    default: return 3;
  }
}
static inline uint32_t gen_prompt_id(uint64_t seed, uint32_t i, uint32_t vocab) {
  return gen_bits(gen_tensor_key(seed, -1, GT_PROMPT), i) % vocab;
}
static inline float gen_bf16_round(float f) {
  union { float f; uint32_t u; } v; v.f = f;
  v.u = (v.u + 0x7FFFu + ((v.u >> 16) & 1u)) & 0xFFFF0000u;
  return v.f;
}
#endif
