"""Split decode attention and the dense GEMV in one launch (kernels.hip attn_dense_kernel, B <= 2, bf16).

The fused launch runs the same attention block body, the same partial merge and the same dense rows
body as the two separate launches (BS_ATTN_DENSE=0), only with the hand-off inside the launch: its
outputs must be BIT-identical to theirs at every step, across 1..3 context splits (each split covers
256 positions), and both must match the CPU checker within the bf16 logits bound.
"""
import numpy as np
import pytest

from distributed_inference_demo_amd.stage import Stage
from oracle import gen_np
from oracle.oracle import OracleStage

pytestmark = pytest.mark.gpu
BF16_TOL = 2e-2


def _stage(monkeypatch, fused, h, nh, L, V, B, max_ctx, seed):
    monkeypatch.setenv("BS_ATTN_DENSE", "1" if fused else "0")
    return Stage(h, nh, L, V, 0, L, dtype="bf16", max_batch=B, max_ctx=max_ctx, max_tokens=B * max_ctx, seed=seed)


@pytest.mark.parametrize("h,nh,B,P", [(1536, 16, 1, 200), (1024, 16, 1, 530), (1024, 16, 2, 250)])
def test_attn_dense_fused_bitwise_equals_separate_launches(monkeypatch, h, nh, B, P):
    import torch
    L, V, max_ctx, seed = 2, 1024, 700, 17
    sf = _stage(monkeypatch, True, h, nh, L, V, B, max_ctx, seed)
    su = _stage(monkeypatch, False, h, nh, L, V, B, max_ctx, seed)
    ids = gen_np.prompt_ids(8, B, P, V).astype(np.int32)
    lf = sf.forward_host(ids, B, P, past_len=0)
    lu = su.forward_host(ids, B, P, past_len=0)
    np.testing.assert_array_equal(lf, lu)
    dev = torch.device("cuda", 0)
    cs = torch.cuda.Stream()
    steps = 300 if P < 256 else 120  # crosses split boundaries at 256 and 512 positions
    with torch.cuda.stream(cs):
        tf = torch.from_numpy(ids[:, -1].copy()).to(dev)
        tu = tf.clone()
        gf = torch.empty((B, V), dtype=torch.float32, device=dev)
        gu = torch.empty_like(gf)
        for step in range(steps):
            past = P + step
            sf.forward(tf, tf, B, 1, past_len=past, logits=gf, stream=cs.cuda_stream)
            su.forward(tu, tu, B, 1, past_len=past, logits=gu, stream=cs.cuda_stream)
            if step % 16 == 0 or step == steps - 1:
                cs.synchronize()
                assert torch.equal(gf, gu), f"step {step} (ctx {past + 1}): fused logits differ"
                assert torch.equal(tf, tu), f"step {step}: fused tokens differ"


def test_attn_dense_fused_matches_oracle_three_splits(monkeypatch):
    """560m width (hd 64), one layer, a 530-token prompt: decode at contexts 531..540 runs three splits;
    greedy tokens and logits against the checker, teacher forced."""
    import torch
    h, nh, L, V, B, P, seed = 1024, 16, 1, 1024, 1, 530, 23
    sf = _stage(monkeypatch, True, h, nh, L, V, B, 560, seed)
    o = OracleStage(h, nh, L, V, 0, L, bf16=True, max_batch=B, max_ctx=560, seed=seed)
    ids = gen_np.prompt_ids(9, B, P, V).astype(np.int32)
    sf.forward_host(ids, B, P, past_len=0)
    to, _ = o.forward(ids, B, P, past_len=0, want_logits=True)
    dev = torch.device("cuda", 0)
    cs = torch.cuda.Stream()
    with torch.cuda.stream(cs):
        tok = torch.empty(B, dtype=torch.int32, device=dev)
        lg = torch.empty((B, V), dtype=torch.float32, device=dev)
        for step in range(10):
            past = P + step
            tok.copy_(torch.from_numpy(np.asarray(to, dtype=np.int32).reshape(B)))
            sf.forward(tok, tok, B, 1, past_len=past, logits=lg, stream=cs.cuda_stream)
            to, lo = o.forward(np.asarray(to, dtype=np.int32).reshape(B, 1), B, 1, past_len=past, want_logits=True)
            cs.synchronize()
            got = lg.cpu().numpy()
            err = float(np.abs(got - lo).max())
            assert err <= BF16_TOL, f"step {step}: logits max err {err}"
