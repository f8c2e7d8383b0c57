"""oracle/gen_np.py — TEST INFRASTRUCTURE (checker side only).

numpy restatement of the repo's deterministic synthetic-weight generator (spec in
DESIGN.md "Synthetic weights"; C twin: oracle/gen.h; device twin:
distributed_inference_demo_amd/csrc/gen.hip).  Used to build the HF-BLOOM golden
fixtures (tests/golden/make_golden.py) and by the CPU tests that check the C and
numpy generators agree bit for bit.
"""
import numpy as np

NSC = np.float32(float.fromhex("0x1.1bc77ap-22"))
U002 = np.float32(float.fromhex("0x1.47ae14p-30"))
U010 = np.float32(float.fromhex("0x1.99999ap-28"))

GT_WEMB, GT_EMB_G, GT_EMB_B, GT_LNF_G, GT_LNF_B, GT_SCORE, GT_PROMPT = 0, 1, 2, 3, 4, 5, 255
(GT_LN1_G, GT_LN1_B, GT_QKV_W, GT_QKV_B, GT_DENSE_W, GT_DENSE_B,
 GT_LN2_G, GT_LN2_B, GT_FC1_W, GT_FC1_B, GT_FC2_W, GT_FC2_B) = range(12)

M64 = (1 << 64) - 1


def sm64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def tensor_key(seed: int, layer: int, tid: int) -> int:
    return sm64(seed ^ sm64((((layer + 1) & 0xFFFFFFFF) << 8) | tid))


def _lb32(x):
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7feb352d)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846ca68b)
    x ^= x >> np.uint32(16)
    return x


def gen_bits(key: int, idx) -> np.ndarray:
    idx = np.asarray(idx, dtype=np.uint32)
    with np.errstate(over="ignore"):
        inner = _lb32(idx + np.uint32((key >> 32) & 0xFFFFFFFF))
        return _lb32(np.uint32(key & 0xFFFFFFFF) ^ inner)


def gen_normal(key: int, idx) -> np.ndarray:
    h1 = gen_bits(key, idx).astype(np.int64)
    h2 = gen_bits(sm64(key), idx).astype(np.int64)
    s = 2 * ((h1 & 0xFFFF) + (h1 >> 16) + (h2 & 0xFFFF) + (h2 >> 16)) - 4 * 65535
    return s.astype(np.float32) * NSC


def gen_uniform(key: int, idx, scale) -> np.ndarray:
    s = 2 * (gen_bits(key, idx).astype(np.int64) >> 8) - 16777215
    return s.astype(np.float32) * scale


def gen_value(kind: int, key: int, idx) -> np.ndarray:
    if kind == 0:
        return gen_normal(key, idx)
    if kind == 1:
        return gen_uniform(key, idx, U002)
    if kind == 2:
        return np.float32(1.0) + gen_uniform(key, idx, U010)
    return gen_uniform(key, idx, U010)


def layer_kind(tid: int) -> int:
    if tid in (GT_LN1_G, GT_LN2_G):
        return 2
    if tid in (GT_LN1_B, GT_LN2_B):
        return 3
    if tid in (GT_QKV_W, GT_DENSE_W, GT_FC1_W, GT_FC2_W):
        return 0
    return 1


def model_kind(tid: int) -> int:
    return {GT_WEMB: 0, GT_SCORE: 0, GT_EMB_G: 2, GT_LNF_G: 2}.get(tid, 3)


def tensor(seed: int, layer: int, tid: int, shape, chunk=1 << 24) -> np.ndarray:
    """One weight tensor, flat index = row-major index in HF's [out][in] layout."""
    n = int(np.prod(shape))
    kind = model_kind(tid) if layer < 0 else layer_kind(tid)
    key = tensor_key(seed, layer, tid)
    out = np.empty(n, dtype=np.float32)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        out[s:e] = gen_value(kind, key, np.arange(s, e, dtype=np.uint32))
    return out.reshape(shape)


def prompt_ids(seed: int, batch: int, seq: int, vocab: int) -> np.ndarray:
    key = tensor_key(seed, -1, GT_PROMPT)
    b = gen_bits(key, np.arange(batch * seq, dtype=np.uint32))
    return (b % np.uint32(vocab)).astype(np.int64).reshape(batch, seq)


def bf16_round(x: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return u.view(np.float32)


def layer_shapes(h: int):
    return {
        GT_LN1_G: (h,), GT_LN1_B: (h,), GT_QKV_W: (3 * h, h), GT_QKV_B: (3 * h,),
        GT_DENSE_W: (h, h), GT_DENSE_B: (h,), GT_LN2_G: (h,), GT_LN2_B: (h,),
        GT_FC1_W: (4 * h, h), GT_FC1_B: (4 * h,), GT_FC2_W: (h, 4 * h), GT_FC2_B: (h,),
    }


def hf_state_dict(seed: int, hidden: int, n_layer: int, vocab: int, bf16: bool = False, n_labels: int = 0):
    """State dict for transformers' BloomForCausalLM built from the generator; with n_labels > 0 also the
    sequence-classification head "score.weight" [n_labels][hidden] (BloomForSequenceClassification)."""
    rnd = bf16_round if bf16 else (lambda a: a)
    sd = {
        "transformer.word_embeddings.weight": rnd(tensor(seed, -1, GT_WEMB, (vocab, hidden))),
        "transformer.word_embeddings_layernorm.weight": rnd(tensor(seed, -1, GT_EMB_G, (hidden,))),
        "transformer.word_embeddings_layernorm.bias": rnd(tensor(seed, -1, GT_EMB_B, (hidden,))),
        "transformer.ln_f.weight": rnd(tensor(seed, -1, GT_LNF_G, (hidden,))),
        "transformer.ln_f.bias": rnd(tensor(seed, -1, GT_LNF_B, (hidden,))),
    }
    names = {
        GT_LN1_G: "input_layernorm.weight", GT_LN1_B: "input_layernorm.bias",
        GT_QKV_W: "self_attention.query_key_value.weight", GT_QKV_B: "self_attention.query_key_value.bias",
        GT_DENSE_W: "self_attention.dense.weight", GT_DENSE_B: "self_attention.dense.bias",
        GT_LN2_G: "post_attention_layernorm.weight", GT_LN2_B: "post_attention_layernorm.bias",
        GT_FC1_W: "mlp.dense_h_to_4h.weight", GT_FC1_B: "mlp.dense_h_to_4h.bias",
        GT_FC2_W: "mlp.dense_4h_to_h.weight", GT_FC2_B: "mlp.dense_4h_to_h.bias",
    }
    for l in range(n_layer):
        for tid, shape in layer_shapes(hidden).items():
            sd[f"transformer.h.{l}.{names[tid]}"] = rnd(tensor(seed, l, tid, shape))
    sd["lm_head.weight"] = sd["transformer.word_embeddings.weight"]
    if n_labels:
        sd["score.weight"] = rnd(tensor(seed, -1, GT_SCORE, (n_labels, hidden)))
    return sd


def int8_rows(w: np.ndarray):
    """Weight-only int8 rule of BS_FLAG_INT8_WEIGHTS (include/bloomstage.h), numpy restatement of
    oracle/bloom_oracle.c quantize_rows: per row scale = max|w| / 127 (1 for a zero row),
    q = rint(w / scale) clamped to [-127, 127].  w: fp32 [N][K] (the bf16-rounded weight).
    Returns (q int8 [N][K], scale fp32 [N])."""
    w = np.asarray(w, dtype=np.float32)
    amax = np.abs(w).max(axis=1)
    scale = np.where(amax > 0, amax / np.float32(127.0), np.float32(1.0)).astype(np.float32)
    q = np.clip(np.rint(w / scale[:, None]), -127, 127).astype(np.int8)
    return q, scale
