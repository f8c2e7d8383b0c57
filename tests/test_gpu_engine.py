"""GPU parity of the persistent decode engine (decode_engine.hip): one launch per decode step.

A stage runs it on eligible decode steps (bf16, S = 1, B <= 4, hidden % 512 == 0) after
bs_set_engine(BS_ENGINE_PERSISTENT).  These tests pin it three ways: against the bf16 CPU checker (oracle/bloom_oracle.c,
same storage roundings; tolerance of tests/test_gpu_parity.py), against the multi-launch engine of
the same library on the same weights (bs_set_engine), and across many consecutive launches (the
in-launch counters are re-zeroed by each launch's last workgroup).
"""
import numpy as np
import pytest

from distributed_inference_demo_amd.stage import BloomStageError, Stage
from oracle import gen_np
from oracle.oracle import OracleStage

from test_gpu_parity import check_close

pytestmark = pytest.mark.gpu


def stages(h, nh, L, V, lb, le, seed, max_batch, max_ctx, is_first=None, is_last=None):
    kw = dict(dtype="bf16", max_batch=max_batch, max_ctx=max_ctx, max_tokens=max_batch * max_ctx, seed=seed,
              is_first=is_first, is_last=is_last)
    pe = Stage(h, nh, L, V, lb, le, **kw)
    pe.set_engine("persistent")
    ln = Stage(h, nh, L, V, lb, le, **kw)
    ln.set_engine("launches")
    o = OracleStage(h, nh, L, V, lb, le, bf16=True, max_batch=max_batch, max_ctx=max_ctx, seed=seed,
                    is_first=is_first, is_last=is_last)
    return pe, ln, o


@pytest.mark.parametrize("B", [1, 2, 3, 4])
def test_engine_full_model_decode_matches_oracle_and_launches(B):
    h, nh, L, V, P = 512, 8, 3, 4096, 9
    pe, ln, o = stages(h, nh, L, V, 0, L, seed=11, max_batch=4, max_ctx=64)
    assert pe.engine(B) == "persistent" and ln.engine(B) == "launches"
    ids = gen_np.prompt_ids(2, B, P, V).astype(np.int32)
    tp, _ = pe.forward_host(ids, B, P, slot=4 - B, want_logits=True)
    ln.forward_host(ids, B, P, slot=4 - B)
    to, _ = o.forward(ids, B, P, slot=4 - B, want_logits=True)
    for step in range(12):
        x = to.reshape(B, 1)  # teacher-force the checker's tokens
        tp, lp = pe.forward_host(x, B, 1, slot=4 - B, past_len=P + step, want_logits=True)
        tl, ll = ln.forward_host(x, B, 1, slot=4 - B, past_len=P + step, want_logits=True)
        to, lo = o.forward(x, B, 1, slot=4 - B, past_len=P + step, want_logits=True)
        check_close(lp, lo, "bf16", f"B={B} step {step}: engine vs checker")
        check_close(lp, ll, "bf16", f"B={B} step {step}: engine vs launches")
        # greedy ids: equal unless the checker's top-2 margin is inside the tolerance
        for b in range(B):
            if tp[b] != to[b]:
                top2 = np.sort(lo[b])[-2:]
                assert top2[1] - top2[0] < 2e-2, (step, b, tp[b], to[b], top2)


@pytest.mark.parametrize("first,last", [(True, False), (False, False), (False, True)])
def test_engine_stage_roles(first, last):
    """Header (embedding in-launch), middle (hidden in/out) and tail (head + argmax) stages."""
    h, nh, L, V, B, P = 1024, 16, 4, 2048, 2, 6
    lb, le = (0, 2) if first else ((1, 3) if not last else (2, 4))
    pe, ln, o = stages(h, nh, L, V, lb, le, seed=5, max_batch=B, max_ctx=32, is_first=first, is_last=last)
    if first:
        x = gen_np.prompt_ids(3, B, P, V).astype(np.int32)
        x1 = gen_np.prompt_ids(4, B, 1, V).astype(np.int32)
    else:
        rng = np.random.default_rng(1)
        x = rng.standard_normal((B, P, h)).astype(np.float32)
        x1 = rng.standard_normal((B, 1, h)).astype(np.float32)
    for s_ in (pe, ln):
        s_.forward_host(x, B, P)
    o.forward(x, B, P)
    if last:
        tp, lp = pe.forward_host(x1, B, 1, past_len=P, want_logits=True)
        tl, ll = ln.forward_host(x1, B, 1, past_len=P, want_logits=True)
        to, lo = o.forward(x1, B, 1, past_len=P, want_logits=True)
        check_close(lp, lo, "bf16", "tail logits")
        check_close(lp, ll, "bf16", "tail logits vs launches")
        assert np.array_equal(tp, np.argmax(lp, axis=1))  # in-launch argmax == argmax of its logits
    else:
        hp = pe.forward_host(x1, B, 1, past_len=P)
        hl = ln.forward_host(x1, B, 1, past_len=P)
        ho = o.forward(x1, B, 1, past_len=P)
        check_close(hp, ho, "bf16", "hidden vs checker")
        check_close(hp, hl, "bf16", "hidden vs launches")


def test_engine_long_context_split_merge():
    """Context 700-760 over 8 heads: every (row, head) splits its KV over many workgroups and the
    last arriving split merges (ticket), across 60 consecutive launches."""
    import torch
    h, nh, L, V, B, P = 512, 8, 2, 1024, 1, 700
    pe, ln, o = stages(h, nh, L, V, 0, L, seed=7, max_batch=B, max_ctx=800)
    ids = gen_np.prompt_ids(9, B, P, V).astype(np.int32)
    to, _ = o.forward(ids, B, P, want_logits=True)
    dev = torch.device("cuda", 0)
    cs = torch.cuda.Stream()
    with torch.cuda.stream(cs):
        tin = torch.from_numpy(ids).to(dev)
        tok = torch.empty(B, dtype=torch.int32, device=dev)
        lg = torch.empty((B, V), dtype=torch.float32, device=dev)
        pe.forward(tin, tok, B, P, past_len=0, stream=cs.cuda_stream)
        for step in range(60):
            tok.copy_(torch.from_numpy(to))
            pe.forward(tok, tok, B, 1, past_len=P + step, logits=lg, stream=cs.cuda_stream)
            to, lo = o.forward(to.reshape(B, 1), B, 1, past_len=P + step, want_logits=True)
            if step % 7 == 0 or step == 59:
                torch.cuda.synchronize()
                check_close(lg.cpu().numpy(), lo, "bf16", f"decode step {step} (ctx {P + step + 1})")


def test_engine_real_dims_one_block_per_family():
    """One real-dimension middle layer per BLOOM family (h 1024/1536/2560/4096, 16/16/32/32 heads)."""
    for h, nh in ((1024, 16), (1536, 16), (2560, 32), (4096, 32)):
        pe, ln, o = stages(h, nh, 3, 1024, 1, 2, seed=h, max_batch=1, max_ctx=40, is_first=False, is_last=False)
        rng = np.random.default_rng(h)
        x = rng.standard_normal((1, 20, h)).astype(np.float32)
        for s_ in (pe, ln):
            s_.forward_host(x, 1, 20)
        o.forward(x, 1, 20)
        for p in range(20, 24):
            x1 = rng.standard_normal((1, 1, h)).astype(np.float32)
            check_close(pe.forward_host(x1, 1, 1, past_len=p), o.forward(x1, 1, 1, past_len=p), "bf16", f"h={h} p={p}")
            ln.forward_host(x1, 1, 1, past_len=p)


def test_engine_selection_rules():
    st = Stage(512, 8, 2, 1024, 0, 2, dtype="bf16", max_batch=8, max_ctx=16)
    st.set_engine("persistent")
    assert st.engine(1) == "persistent" and st.engine(4) == "persistent" and st.engine(5) == "launches"
    st.set_engine("launches")
    assert st.engine(1) == "launches"
    st.set_engine("persistent")
    with pytest.raises(BloomStageError, match="not eligible"):
        st.forward_host(np.zeros((5, 1), np.int32), 5, 1)
    small = Stage(256, 4, 2, 1024, 0, 2, dtype="bf16", max_ctx=16)  # hidden % 512 != 0
    assert small.engine(1) == "launches"
    with pytest.raises(BloomStageError, match="unavailable"):
        small.set_engine("persistent")
    f32 = Stage(512, 8, 2, 1024, 0, 2, dtype="fp32", max_ctx=16)
    assert f32.engine(1) == "launches"
