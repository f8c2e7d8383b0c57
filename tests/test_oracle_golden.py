"""The CPU checker (oracle/bloom_oracle.c) pinned against HF BLOOM fp32 golden fixtures
(tests/golden/make_golden.py).  No GPU needed."""
import os

import numpy as np
import pytest

from oracle import gen_np
from oracle.oracle import OracleStage, alibi_slopes, gen_tensor, prompt_ids

G = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    return np.load(os.path.join(G, name))


def test_generator_c_matches_numpy():
    for layer, tid, n in [(-1, gen_np.GT_WEMB, 4096), (-1, gen_np.GT_EMB_G, 512), (-1, gen_np.GT_LNF_B, 512),
                          (0, gen_np.GT_QKV_W, 9000), (5, gen_np.GT_FC1_B, 777), (2, gen_np.GT_LN2_G, 300),
                          (29, gen_np.GT_FC2_W, 5000)]:
        a = gen_tensor(123, layer, tid, n)
        kind = gen_np.model_kind(tid) if layer < 0 else gen_np.layer_kind(tid)
        b = gen_np.gen_value(kind, gen_np.tensor_key(123, layer, tid), np.arange(n, dtype=np.uint32))
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (layer, tid)


def test_generator_statistics():
    w = gen_np.tensor(1, 0, gen_np.GT_FC1_W, (4096, 256))
    assert abs(float(w.std()) - 0.02) < 5e-4 and abs(float(w.mean())) < 2e-4
    g = gen_np.tensor(1, 0, gen_np.GT_LN1_G, (4096,))
    assert g.min() >= 0.9 and g.max() <= 1.1


def test_prompt_ids_match():
    assert np.array_equal(prompt_ids(1234, 3, 17, 250880), gen_np.prompt_ids(1234, 3, 17, 250880))


def test_bf16_round_matches_rne():
    x = np.array([1.0, 1.00390625, 1.005859375, -3.14159, 1e-20, 65504.0], np.float32)
    import torch
    ref = torch.from_numpy(x).to(torch.bfloat16).float().numpy()
    assert np.array_equal(gen_np.bf16_round(x), ref)


def test_alibi_slopes_match_hf():
    a = _load("alibi.npz")
    for nh in (16, 32, 12):
        np.testing.assert_allclose(alibi_slopes(nh), a[f"slopes_{nh}"], rtol=1e-6, atol=0)


def test_tiny_logits_and_greedy_match_hf():
    g = _load("tiny_e2e.npz")
    h, nh, L, V, seed, B, S = (int(v) for v in g["config"])
    st = OracleStage(h, nh, L, V, 0, L, max_batch=B, max_ctx=S + 128, seed=seed)
    tok, lg = st.forward(g["ids"], B, S, want_logits=True)
    np.testing.assert_allclose(lg, g["logits"], atol=2e-6 * np.abs(g["logits"]).max(), rtol=0)
    toks = [tok]
    for i in range(127):
        tok = st.forward(tok.reshape(B, 1), B, 1, past_len=S + i)
        toks.append(tok)
    assert np.array_equal(np.stack(toks, 1), g["greedy"])


@pytest.mark.parametrize("split", [1, 2, 3])
def test_tiny_stage_boundaries_match_hf(split):
    g = _load("tiny_e2e.npz")
    h, nh, L, V, seed, B, S = (int(v) for v in g["config"])
    s0 = OracleStage(h, nh, L, V, 0, split, max_batch=B, max_ctx=S, seed=seed)
    hid = s0.forward(g["ids"], B, S)
    np.testing.assert_allclose(hid, g["layer_out"][split - 1], atol=2e-6, rtol=0)
    s1 = OracleStage(h, nh, L, V, split, L, max_batch=B, max_ctx=S, seed=seed)
    tok, lg = s1.forward(hid, B, S, want_logits=True)
    np.testing.assert_allclose(lg, g["logits"], atol=2e-6 * np.abs(g["logits"]).max(), rtol=0)


def test_nonpow2_heads_match_hf():
    g = _load("tiny_nonpow2.npz")
    h, nh, L, V, seed, B, S = (int(v) for v in g["config"])
    st = OracleStage(h, nh, L, V, 0, L, max_batch=B, max_ctx=S, seed=seed)
    _, lg = st.forward(g["ids"], B, S, want_logits=True)
    np.testing.assert_allclose(lg, g["logits"], atol=2e-6 * np.abs(g["logits"]).max(), rtol=0)


@pytest.mark.parametrize("fam", ["560m", "1b1", "3b", "7b1"])
def test_family_block_matches_hf(fam):
    f = _load("family_blocks.npz")
    h, nh, _, V, seed = (int(v) for v in f[fam + "_config"])
    st = OracleStage(h, nh, 1, V, 0, 1, max_batch=1, max_ctx=64, seed=seed, is_last=False)
    ref = f[fam + "_out64"]
    tol = 4e-6 * np.abs(ref).max()
    np.testing.assert_allclose(st.forward(f[fam + "_ids64"], 1, 64), ref, atol=tol, rtol=0)
    ids = f[fam + "_ids23"]
    st.forward(ids[:, :15], 1, 15)
    np.testing.assert_allclose(st.forward(ids[:, 15:22], 1, 7, past_len=15), f[fam + "_out7"], atol=tol, rtol=0)
    np.testing.assert_allclose(st.forward(ids[:, 22:23], 1, 1, past_len=22), f[fam + "_out1"], atol=tol, rtol=0)


def test_kv_cached_decode_equals_full_recompute():
    """the parity target is full-context decode; cached == recompute."""
    g = _load("tiny_e2e.npz")
    h, nh, L, V, seed, B, S = (int(v) for v in g["config"])
    full = np.concatenate([g["ids"], g["greedy"][:, :-1]], axis=1)
    st = OracleStage(h, nh, L, V, 0, L, max_batch=B, max_ctx=full.shape[1], seed=seed)
    _, lg = st.forward(full, B, full.shape[1], want_logits=True)
    np.testing.assert_allclose(lg, g["full_recompute_logits"], atol=5e-6 * np.abs(lg).max(), rtol=0)


def test_bf16_noise_floor_of_the_checker():
    """Two fp32 accumulation orders of the same bf16-emulated block: the spread the GPU-vs-oracle
    bf16 tolerance must admit (see tests/test_gpu_parity.py header)."""
    from oracle.oracle import lib
    f = _load("family_blocks.npz")
    h, nh, _, V, seed = (int(v) for v in f["7b1_config"])
    outs = []
    try:
        for dbl in (0, 1):
            lib().or_set_accum_double(dbl)
            st = OracleStage(h, nh, 1, V, 0, 1, bf16=True, max_ctx=64, seed=seed, is_last=False)
            outs.append(st.forward(f["7b1_ids64"], 1, 64))
            st.close()
    finally:
        lib().or_set_accum_double(0)
    d = float(np.abs(outs[0] - outs[1]).max())
    scale = float(np.abs(outs[1]).max())
    assert 1e-3 < d < 2.5e-3 * scale, (d, scale)


@pytest.mark.parametrize("n_labels", [2, 3])
@pytest.mark.parametrize("split", [0, 1])
def test_classifier_tail_matches_hf(n_labels, split):
    """Sequence-classification tail (or_set_classifier) against BloomForSequenceClassification's pooled logits,
    as one stage and as a 1 + 1 layer split; the class is the first maximal index (inference.cpp:57-69)."""
    g = _load("tiny_classify.npz")
    h, nh, L, V, seed, B, S = (int(v) for v in g["config"])
    x = g["ids"]
    if split:
        x = OracleStage(h, nh, L, V, 0, split, max_batch=B, max_ctx=S, seed=seed).forward(x, B, S)
    st = OracleStage(h, nh, L, V, split, L, max_batch=B, max_ctx=S, seed=seed, n_labels=n_labels)
    cls, lg = st.forward(x, B, S, want_logits=True)
    ref = g[f"logits{n_labels}"]
    assert lg.shape == (B, n_labels)
    np.testing.assert_allclose(lg, ref, atol=2e-6 * np.abs(ref).max(), rtol=0)
    assert np.array_equal(cls, g[f"class{n_labels}"])


def test_classifier_one_label():
    """n_labels = 1 (a regression-style head): logits [B][1], every row's class 0."""
    st = OracleStage(64, 4, 1, 512, 0, 1, max_batch=2, max_ctx=4, seed=1, n_labels=1)
    cls, lg = st.forward(np.array([[5, 6], [7, 8]]), 2, 2, want_logits=True)
    assert lg.shape == (2, 1) and np.array_equal(cls, [0, 0])
