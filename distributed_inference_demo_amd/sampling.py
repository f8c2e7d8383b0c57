"""Tail token pick alternatives to greedy argmax.

Reference: decoding::StaticDecoding (decoding.cpp:24-66) takes the top-k of the last
position's row, normalises those k values by their sum and samples with an mt19937 seeded
from std::random_device (non-deterministic).  The ONNX tail module is inferred to emit
probabilities.  Here the stage emits raw logits, so the k values are
turned into probabilities with a temperature softmax first; the generator is seeded so runs
are reproducible.  Temperature is plumbed (the reference receives it but never applies it,
decoding.cpp:51-52).
"""
import numpy as np


def top_k_sample(logits: np.ndarray, k: int, temperature: float = 1.0, seed: int = 0) -> int:
    logits = np.asarray(logits, dtype=np.float64).reshape(-1)
    k = max(1, min(int(k), logits.size))
    idx = np.argpartition(-logits, k - 1)[:k]
    idx = idx[np.lexsort((idx, -logits[idx]))]  # descending value, ascending index on ties
    z = logits[idx] / max(float(temperature), 1e-6)
    p = np.exp(z - z.max())
    p /= p.sum()
    return int(idx[np.random.default_rng(seed).choice(k, p=p)])
