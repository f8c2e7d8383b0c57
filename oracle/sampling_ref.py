"""oracle/sampling_ref.py — TEST INFRASTRUCTURE: restatement of the tail token pick, the checker
for bs_set_sampling (include/bloomstage.h) / topk_sample_kernel (csrc/kernels.hip).

Reference: decoding::StaticDecoding (decoding.cpp:24-66):
  * the (value, index) pairs of the last position are partially sorted with
    std::greater<std::pair<float, int>> (:37-45): larger value first, and on equal values the
    HIGHER index first;
  * the k values are normalised by their sum (:48-57) -- the ONNX tail emits probabilities, so on
    logits that is softmax restricted to the top k: w_i = exp(l_i - l_0) (temperature 1; the
    reference never applies its temperature, :51-52);
  * an index is drawn from that distribution (:59-65) with an unseeded mt19937; here the draw u is
    the repo's counter generator keyed by (seed, KV row, position), and the pick is the first rank i
    whose running fp32 sum of w exceeds u * sum(w) (the last rank if rounding leaves none).
"""
import numpy as np

from .gen_np import M64, gen_bits, sm64


def order_key(v):
    """fp32 -> uint32, monotone (the device's f32_order_key)."""
    u = np.asarray(v, np.float32).view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)


def topk_reference_order(logits, k):
    """Indices of the top k of one row in std::greater<pair<float,int>> order."""
    logits = np.asarray(logits, np.float32).reshape(-1)
    idx = np.arange(logits.size, dtype=np.uint64)
    keys = (order_key(logits) << np.uint64(32)) | idx
    top = np.argsort(keys)[::-1][:k]  # keys are unique (the index is in the low bits)
    return top.astype(np.int64)


def sample_u(seed, row, pos):
    key = sm64((seed ^ sm64(0x5A4D504C00000000 | (row & 0xFFFFFFFF))) & M64)
    bits = int(gen_bits(key, np.uint32(pos & 0xFFFFFFFF)))
    return np.float32(bits >> 8) * np.float32(2.0 ** -24)


def sample_pick(logits, k, seed, row, pos, temperature=1.0):
    """(picked vocab index, ranked indices, weights, u) of one row."""
    logits = np.asarray(logits, np.float32).reshape(-1)
    ranked = topk_reference_order(logits, k)
    inv_t = np.float32(1.0) / np.float32(temperature)
    w = np.exp((logits[ranked] - logits[ranked[0]]) * inv_t).astype(np.float32)
    total = np.float32(0.0)
    for x in w:
        total = np.float32(total + x)
    u = sample_u(seed, row, pos)
    target = np.float32(u * total)
    run, sel = np.float32(0.0), k - 1
    for i, x in enumerate(w):
        run = np.float32(run + x)
        if run > target:
            sel = i
            break
    return int(ranked[sel]), ranked, w, u
