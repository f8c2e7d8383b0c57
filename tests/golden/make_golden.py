"""tests/golden/make_golden.py — builds the committed golden fixtures (run in the dev container only).

Why this oracle: the reference's stage arithmetic is ONNX Runtime executing BLOOM sub-graphs
exported from HF transformers.  Neither ORT nor the ONNX files exist here,
so the arithmetic is pinned on the locally installed transformers BloomForCausalLM (fp32,
CPU), built from a hand-written BloomConfig (no from_pretrained, no network) with weights
from the repo's deterministic generator (oracle/gen_np.py).  The C checker
(oracle/bloom_oracle.c) is validated against these fixtures by tests/test_oracle_golden.py;
the device path is then validated against the C checker on the GPU.

Usage:  python tests/golden/make_golden.py      (writes tests/golden/*.npz)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle import gen_np  # noqa: E402

from transformers import BloomConfig, BloomForCausalLM, BloomForSequenceClassification  # noqa: E402
from transformers.models.bloom.modeling_bloom import build_alibi_tensor  # noqa: E402

torch.set_grad_enabled(False)
torch.manual_seed(0)


def build(hidden, n_head, n_layer, vocab, seed):
    cfg = BloomConfig(vocab_size=vocab, hidden_size=hidden, n_layer=n_layer, n_head=n_head,
                      layer_norm_epsilon=1e-5, apply_residual_connection_post_layernorm=False,
                      hidden_dropout=0.0, attention_dropout=0.0, use_cache=True)
    m = BloomForCausalLM(cfg).eval().float()
    sd = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in
          gen_np.hf_state_dict(seed, hidden, n_layer, vocab).items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all("lm_head" in k for k in missing), missing
    m.tie_weights()
    assert torch.equal(m.lm_head.weight, m.transformer.word_embeddings.weight)
    return m


def layer_outputs(model, ids, past=None):
    """Outputs of every decoder block (pre ln_f) + logits + cache."""
    outs = []
    hooks = [blk.register_forward_hook(lambda mod, i, o: outs.append(o[0].clone()))
             for blk in model.transformer.h]
    r = model(input_ids=torch.from_numpy(ids), past_key_values=past, use_cache=True)
    for hk in hooks:
        hk.remove()
    return [o.numpy() for o in outs], r.logits[:, -1, :].numpy(), r.past_key_values


def tiny_e2e():
    """(1) tiny config end to end: per-layer outputs, last-position logits, 128 greedy ids."""
    h, nh, L, V, seed, B, S = 64, 4, 4, 512, 0, 2, 8
    m = build(h, nh, L, V, seed)
    ids = gen_np.prompt_ids(1234, B, S, V)
    layers, logits, past = layer_outputs(m, ids)
    toks, margins = [], []
    cur = logits
    for _ in range(128):
        nxt = cur.argmax(-1)
        srt = np.sort(cur, axis=-1)
        margins.append(srt[:, -1] - srt[:, -2])
        toks.append(nxt)
        r = m(input_ids=torch.from_numpy(nxt[:, None].astype(np.int64)), past_key_values=past, use_cache=True)
        past, cur = r.past_key_values, r.logits[:, -1, :].numpy()
    # full-recompute check of the KV-cached decode
    full = np.concatenate([ids, np.stack(toks, 1)[:, :-1]], axis=1)
    full_logits = m(input_ids=torch.from_numpy(full), use_cache=False).logits[:, -1, :].numpy()
    np.savez_compressed(os.path.join(HERE, "tiny_e2e.npz"),
                        config=np.array([h, nh, L, V, seed, B, S]), ids=ids.astype(np.int32),
                        layer_out=np.stack(layers), logits=logits,
                        greedy=np.stack(toks, 1).astype(np.int32), margins=np.stack(margins, 1),
                        full_recompute_logits=full_logits)
    print("tiny_e2e ok; cached-vs-full max|d| =", np.abs(full_logits - cur).max())


def tiny_nonpow2():
    """(3b) non-power-of-2 head count exercises the ALiBi extra-slope branch."""
    h, nh, L, V, seed, B, S = 96, 12, 2, 256, 5, 1, 9
    m = build(h, nh, L, V, seed)
    ids = gen_np.prompt_ids(99, B, S, V)
    layers, logits, _ = layer_outputs(m, ids)
    np.savez_compressed(os.path.join(HERE, "tiny_nonpow2.npz"),
                        config=np.array([h, nh, L, V, seed, B, S]), ids=ids.astype(np.int32),
                        layer_out=np.stack(layers), logits=logits)
    print("tiny_nonpow2 ok")


FAMILIES = {"560m": (1024, 16), "1b1": (1536, 16), "3b": (2560, 32), "7b1": (4096, 32)}


def family_blocks():
    """(2) one real-dimension block per family: S=64 from empty cache; S=7 after 15 cached; S=1 after 22."""
    V, seed = 1024, 11
    out = {}
    for name, (h, nh) in FAMILIES.items():
        m = build(h, nh, 1, V, seed)
        ids64 = gen_np.prompt_ids(2024, 1, 64, V)
        l64, _, _ = layer_outputs(m, ids64)
        ids22 = gen_np.prompt_ids(77, 1, 23, V)
        _, _, past = layer_outputs(m, ids22[:, :15])
        l7, _, past = layer_outputs(m, ids22[:, 15:22], past)
        l1, _, _ = layer_outputs(m, ids22[:, 22:23], past)
        out[f"{name}_config"] = np.array([h, nh, 1, V, seed])
        out[f"{name}_ids64"] = ids64.astype(np.int32)
        out[f"{name}_out64"] = l64[0]
        out[f"{name}_ids23"] = ids22.astype(np.int32)
        out[f"{name}_out7"] = l7[0]
        out[f"{name}_out1"] = l1[0]
        print("family", name, "ok")
    np.savez_compressed(os.path.join(HERE, "family_blocks.npz"), **out)


def tiny_classify():
    """(4) sequence-classification tail: BloomForSequenceClassification's pooled logits (the row's last
    non-pad token; no prompt holds the pad id) and their argmax, for 2 labels (what the reference's
    binary_classify reads, inference.cpp:57-69) and 3 labels."""
    h, nh, L, V, seed, B, S = 64, 4, 2, 512, 3, 3, 9
    ids = gen_np.prompt_ids(4321, B, S, V)
    out = {"config": np.array([h, nh, L, V, seed, B, S]), "ids": ids.astype(np.int32)}
    for nl in (2, 3):
        pad = next(p for p in range(V) if not (ids == p).any())
        cfg = BloomConfig(vocab_size=V, hidden_size=h, n_layer=L, n_head=nh, layer_norm_epsilon=1e-5,
                          hidden_dropout=0.0, attention_dropout=0.0, num_labels=nl, pad_token_id=pad)
        m = BloomForSequenceClassification(cfg).eval().float()
        sd = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in
              gen_np.hf_state_dict(seed, h, L, V, n_labels=nl).items() if k != "lm_head.weight"}
        m.load_state_dict(sd, strict=True)
        lg = m(input_ids=torch.from_numpy(ids)).logits.numpy()
        out[f"logits{nl}"] = lg
        out[f"class{nl}"] = lg.argmax(-1).astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "tiny_classify.npz"), **out)
    print("tiny_classify ok")


def alibi():
    """(3) ALiBi slopes from HF build_alibi_tensor for 16, 32 and 12 heads."""
    res = {}
    for nh in (16, 32, 12):
        t = build_alibi_tensor(torch.ones(1, 2), nh, torch.float32).reshape(nh, 2)
        res[f"slopes_{nh}"] = t[:, 1].numpy()
    np.savez_compressed(os.path.join(HERE, "alibi.npz"), **res)
    print("alibi ok")


if __name__ == "__main__":
    alibi()
    tiny_e2e()
    tiny_nonpow2()
    family_blocks()
    tiny_classify()
