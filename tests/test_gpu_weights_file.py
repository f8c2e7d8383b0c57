"""Stages created from checkpoint files (bs_init_stage_file, the createSession(model_path) entry of
native-lib.cpp:671-678) on the GPU: the weights land bit-identical to the host-buffer and
synthetic paths, dtype conversions round as documented, head slices and int8 read the right rows,
and a checkpoint written by transformers' own save_pretrained (sharded) reproduces the HF golden
greedy ids through the JNI-mirror loopback."""
import os

import numpy as np
import pytest
import torch
from safetensors.torch import save_file

from distributed_inference_demo_amd.config import BloomDims
from distributed_inference_demo_amd.stage import (Stage, create_session, deserialize_int, run_inference_master_residual,
                                                  run_inference_worker_residual_last_generation)
from oracle import gen_np
from tests.test_gpu_parity import canonical_weights
from tests.test_weights_file import H, L, NH, V, hf_tensors, write_sharded

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.parametrize("lb,le", [(0, L), (1, 3), (2, L)])
def test_fp32_file_equals_host_buffer(tmp_path, lb, le):
    f = str(tmp_path / "m.safetensors")
    save_file(hf_tensors(seed=4), f)
    a = Stage(H, NH, L, V, lb, le, dtype="fp32", max_ctx=16, weights_file=f)
    b = Stage(H, NH, L, V, lb, le, dtype="fp32", max_ctx=16,
              host_weights=canonical_weights(4, H, L, V, lb, le, first=lb == 0, last=le == L))
    assert np.array_equal(_bits(a.read_weights()), _bits(b.read_weights()))
    if lb == 0:
        x = gen_np.prompt_ids(1, 1, 6, V).astype(np.int32)
    else:
        x = np.random.default_rng(0).standard_normal((1, 6, H)).astype(np.float32)
    if le == L:
        ya, la = a.forward_host(x, 1, 6, want_logits=True)
        yb, lb_ = b.forward_host(x, 1, 6, want_logits=True)
        assert np.array_equal(la, lb_)
    else:
        ya, yb = a.forward_host(x, 1, 6), b.forward_host(x, 1, 6)
    assert np.array_equal(ya, yb)


@pytest.mark.parametrize("src", ["BF16", "F32"])
def test_bf16_stage_from_file_equals_synthetic(tmp_path, src):
    """bf16 checkpoint bits are copied as they are; fp32 ones round to nearest even on the device,
    exactly like the synthetic generator's own rounding."""
    t = hf_tensors(seed=4)
    if src == "BF16":
        t = {k: v.to(torch.bfloat16) for k, v in t.items()}
    f = str(tmp_path / "m.safetensors")
    save_file(t, f)
    a = Stage(H, NH, L, V, 0, L, dtype="bf16", max_ctx=16, weights_file=f)
    b = Stage(H, NH, L, V, 0, L, dtype="bf16", max_ctx=16, seed=4)
    assert np.array_equal(_bits(a.read_weights()), _bits(b.read_weights()))
    x = gen_np.prompt_ids(2, 1, 9, V).astype(np.int32)
    _, la = a.forward_host(x, 1, 9, want_logits=True)
    _, lb = b.forward_host(x, 1, 9, want_logits=True)
    assert np.array_equal(la, lb)


def test_f16_file_widens_exactly(tmp_path):
    t = {k: v.to(torch.float16) for k, v in hf_tensors(seed=4).items()}
    f = str(tmp_path / "m.safetensors")
    save_file(t, f)
    a = Stage(H, NH, L, V, 1, 3, dtype="fp32", max_ctx=8, weights_file=f, is_first=False, is_last=False)
    want = canonical_weights(4, H, L, V, 1, 3, first=False, last=False).astype(np.float16).astype(np.float32)
    assert np.array_equal(_bits(a.read_weights()), _bits(want))


def test_head_slice_and_int8_from_sharded_index(tmp_path):
    """A middle stage holding a vocabulary slice reads rows [128, 256) of the embedding; an int8
    stage quantizes the file's weights exactly as it quantizes synthetic ones."""
    idx = write_sharded(tmp_path, hf_tensors(seed=4), n_shards=3)
    kw = dict(max_ctx=8, is_first=False, is_last=False, head_slice=(128, 256))
    a = Stage(H, NH, L, V, 1, 3, dtype="fp32", weights_file=idx, **kw)
    b = Stage(H, NH, L, V, 1, 3, dtype="fp32", seed=4, **kw)
    assert np.array_equal(_bits(a.read_weights()), _bits(b.read_weights()))
    q = Stage(H, NH, L, V, 0, L, dtype="bf16", max_ctx=8, weights_file=idx, int8_weights=True)
    r = Stage(H, NH, L, V, 0, L, dtype="bf16", max_ctx=8, seed=4, int8_weights=True)
    assert np.array_equal(_bits(q.read_weights()), _bits(r.read_weights()))


def test_save_pretrained_checkpoint_reproduces_hf_greedy(tmp_path):
    """transformers writes the checkpoint (its own names, tied head dropped, sharded with an index);
    the two-stage JNI-mirror loopback over it yields the HF golden greedy ids."""
    transformers = pytest.importorskip("transformers")
    m = BloomDims("tiny", 64, 4, 4, vocab=512)
    cfg = transformers.BloomConfig(vocab_size=m.vocab, hidden_size=m.hidden, n_layer=m.n_layer, n_head=m.n_head,
                                   layer_norm_epsilon=1e-5, hidden_dropout=0.0, attention_dropout=0.0)
    model = transformers.BloomForCausalLM(cfg).eval().float()
    sd = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in gen_np.hf_state_dict(0, m.hidden, m.n_layer,
                                                                                         m.vocab).items()}
    model.load_state_dict(sd, strict=False)
    model.tie_weights()
    model.save_pretrained(str(tmp_path), safe_serialization=True, max_shard_size="200KB")
    idx = os.path.join(str(tmp_path), "model.safetensors.index.json")
    assert os.path.exists(idx), os.listdir(str(tmp_path))
    g = np.load(os.path.join(G, "tiny_e2e.npz"))
    head = create_session(m, 0, 2, dtype="fp32", max_ctx=64, weights_file=idx)
    tail = create_session(m, 2, 4, dtype="fp32", max_ctx=64, weights_file=idx)
    seq, res = run_inference_master_residual(head, list(g["ids"][0]))
    toks = []
    for _ in range(8):
        tok = deserialize_int(run_inference_worker_residual_last_generation(tail, seq, res, k=1))
        toks.append(tok)
        seq, res = run_inference_master_residual(head, [tok])
    assert toks == list(g["greedy"][0][:8])
