"""GPU parity of three boundary features, through the C-ABI:

  * per-row positions (bs_step.past_lens, SURVEY.md §8b ctx_lens): the reference keeps
    core_pool_size samples in flight, each at its own position (Communication.java:418-464,
    :621-651).  Rows of one bs_forward call sit at different positions and are checked row by row
    against the CPU checker decoding each row alone;
  * the seeded top-k tail pick (bs_set_sampling) against its restatement oracle/sampling_ref.py of
    decoding::StaticDecoding (decoding.cpp:24-66): the ranked index set bit-exact (ties: higher
    index first), the draw equal;
  * the vocabulary-parallel head (bs_head_norm / bs_head_slice) against the checker's
    or_head_norm / or_head_slice.
"""
import numpy as np
import pytest

from distributed_inference_demo_amd.stage import BloomStageError, Stage
from oracle import gen_np
from oracle.oracle import OracleStage
from oracle.sampling_ref import sample_pick, topk_reference_order

from test_gpu_parity import BF16_TOL, assert_ids_match, canonical_weights, check_close, check_logits

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_rows_at_different_positions_match_per_row_checker(dtype):
    """4 rows, prompts of 3/9/1/6 tokens prefilled one row at a time, then batched steps where
    every row sits at its own position: an S = 5 chunk (prefill attention + QKV epilogue with
    per-row positions), then 12 S = 1 decode steps (eager host I/O), row by row vs the checker."""
    h, nh, L, V, B = 256, 4, 2, 1024, 4
    lens = [3, 9, 1, 6]
    g = Stage(h, nh, L, V, 0, L, dtype=dtype, max_batch=B, max_ctx=40, max_tokens=B * 8, seed=41)
    o = OracleStage(h, nh, L, V, 0, L, bf16=dtype == "bf16", max_batch=B, max_ctx=40, seed=41)
    toks = []
    for r, n in enumerate(lens):
        ids = gen_np.prompt_ids(100 + r, 1, n, V).astype(np.int32)
        g.forward_host(ids, 1, n, slot=r, past_len=0)
        toks.append(o.forward(ids, 1, n, slot=r, past_len=0))
    past = list(lens)
    chunk = gen_np.prompt_ids(7, B, 5, V).astype(np.int32)
    tg, lg = g.forward_host(chunk, B, 5, slot=0, past_len=past, want_logits=True)
    for r in range(B):
        to, lo = o.forward(chunk[r:r + 1], 1, 5, slot=r, past_len=past[r], want_logits=True)
        check_logits(lg[r:r + 1], lo, dtype, f"row {r} chunk at position {past[r]}")
        assert_ids_match(tg[r:r + 1], to, lo, f"row {r} chunk")
        toks[r] = to
    past = [p + 5 for p in past]
    for step in range(12):
        x = np.concatenate(toks).reshape(B, 1)
        tg, lg = g.forward_host(x, B, 1, slot=0, past_len=past, want_logits=True)
        for r in range(B):
            to, lo = o.forward(x[r:r + 1], 1, 1, slot=r, past_len=past[r], want_logits=True)
            check_logits(lg[r:r + 1], lo, dtype, f"step {step} row {r} (position {past[r]})")
            assert_ids_match(tg[r:r + 1], to, lo, f"step {step} row {r}")
            toks[r] = to
        past = [p + 1 for p in past]
    with pytest.raises(BloomStageError, match="max_ctx"):
        g.forward_host(np.zeros((B, 1), np.int32), B, 1, past_len=[0, 39, 0, 40])


def test_rows_at_different_positions_graph_replay():
    """Device-I/O decode (captured hipGraph, per-row positions written ahead of every replay) over
    rows ~150 positions apart: the split-context attention (2 splits at this cache size) reads each
    row's own length."""
    import torch
    h, nh, L, V, B = 512, 8, 2, 2048, 3
    lens = [5, 150, 300]
    g = Stage(h, nh, L, V, 0, L, dtype="bf16", max_batch=B, max_ctx=400, max_tokens=300, seed=43)
    o = OracleStage(h, nh, L, V, 0, L, bf16=True, max_batch=B, max_ctx=400, seed=43)
    toks = []
    for r, n in enumerate(lens):
        ids = gen_np.prompt_ids(200 + r, 1, n, V).astype(np.int32)
        g.forward_host(ids, 1, n, slot=r, past_len=0)
        toks.append(o.forward(ids, 1, n, slot=r, past_len=0))
    dev = torch.device("cuda", 0)
    cs = torch.cuda.Stream()
    past = list(lens)
    with torch.cuda.stream(cs):
        tok = torch.empty(B, dtype=torch.int32, device=dev)
        lg = torch.empty((B, V), dtype=torch.float32, device=dev)
        for step in range(40):
            x = np.concatenate(toks).astype(np.int32)
            tok.copy_(torch.from_numpy(x))
            g.forward(tok, tok, B, 1, slot=0, past_len=past, logits=lg, stream=cs.cuda_stream)
            torch.cuda.synchronize()
            gl, gt = lg.cpu().numpy(), tok.cpu().numpy()
            for r in range(B):
                to, lo = o.forward(x[r:r + 1].reshape(1, 1), 1, 1, slot=r, past_len=past[r], want_logits=True)
                if step % 6 == 0 or step == 39:
                    check_logits(gl[r:r + 1], lo, "bf16", f"graph step {step} row {r}")
                assert_ids_match(gt[r:r + 1], to, lo, f"graph step {step} row {r}")
                toks[r] = to
            past = [p + 1 for p in past]


def _tied_head_stage(h, nh, V, top_rows, token, seed=4):
    """A layer-free first+last stage (embedding -> emb LN -> ln_f -> tied lm_head), so the head's
    input depends on the input token only.  Its tied embedding rows `top_rows` are one identical
    row along that input (xn of `token`): their logits tie exactly at ~5, far above the rest."""
    w = canonical_weights(seed, h, 2, V, 0, 0, first=True, last=True)
    emb = w[:V * h].reshape(V, h)
    eg, eb = w[V * h:V * h + h], w[V * h + h:V * h + 2 * h]
    fg, fb = w[V * h + 2 * h:V * h + 3 * h], w[V * h + 3 * h:]

    def ln(x, g, b):
        x = x.astype(np.float64)
        return (x - x.mean()) / np.sqrt(x.var() + 1e-5) * g + b
    xn = ln(ln(emb[token], eg, eb), fg, fb)
    emb[list(top_rows)] = (xn * (5.0 / float(xn @ xn))).astype(np.float32)
    return Stage(h, nh, 2, V, 0, 0, dtype="fp32", max_batch=1, max_ctx=80, host_weights=w, is_first=True,
                 is_last=True)


@pytest.mark.parametrize("k", [2, 7, 16])
def test_topk_sampling_matches_restatement(k):
    """Free-running sampled decode: every step's pick equals the restatement applied to the
    stage's own logits at (seed, row, position); the ranked top-k set is reproduced bit for bit."""
    h, nh, L, V, B = 256, 4, 2, 2048, 3
    g = Stage(h, nh, L, V, 0, L, dtype="bf16", max_batch=B, max_ctx=48, max_tokens=B * 8, seed=9)
    g.set_sampling(k, 1.0, seed=1234)
    x = gen_np.prompt_ids(5, B, 8, V).astype(np.int32)
    past, picks = 0, []
    for step in range(24):
        S = x.shape[1]
        tg, lg = g.forward_host(x, B, S, slot=0, past_len=past, want_logits=True)
        for r in range(B):
            want, ranked, w, u = sample_pick(lg[r], k, 1234, r, past + S)
            assert len(set(ranked.tolist())) == k
            if tg[r] != want:  # only a draw on a rounding boundary may differ
                cum = np.cumsum(w.astype(np.float64))
                assert np.min(np.abs(cum - float(u) * cum[-1])) < 1e-5 * cum[-1], (step, r, tg[r], want)
            assert tg[r] in ranked
            picks.append(int(tg[r]))
        past += S
        x = tg.reshape(B, 1)
    assert len(set(picks)) > 1  # a fresh draw per step (the position keys the generator)


def test_topk_sampling_ties_rank_higher_index_first():
    """Eight exactly tied, dominant logits (identical tied-embedding rows): std::greater ranks the
    higher index first (decoding.cpp:44-45), so k = 7 draws only from the 7 highest of the 8."""
    h, nh, V = 128, 4, 1024
    top = [40, 300, 301, 555, 700, 701, 900, 1000]
    g = _tied_head_stage(h, nh, V, top, token=3)
    g.set_sampling(7, 1.0, seed=77)
    seen = set()
    x = np.array([[3]], np.int32)
    for step in range(60):
        tg, lg = g.forward_host(x, 1, 1, slot=0, past_len=step, want_logits=True)
        assert np.all(lg[0][top] == lg[0][top[0]]) and lg[0][top[0]] > 4.0
        ranked = topk_reference_order(lg[0], 7)
        assert sorted(ranked.tolist()) == sorted(top[1:]), ranked  # index 40 (the lowest) is out
        want, _, _, _ = sample_pick(lg[0], 7, 77, 0, step + 1)
        assert int(tg[0]) == want
        seen.add(int(tg[0]))
        x = np.array([[3]], np.int32)
    assert seen <= set(top[1:]) and len(seen) >= 4
    g.set_sampling(1)  # back to greedy: lowest index among the ties (torch.argmax)
    tg = g.forward_host(x, 1, 1, slot=0, past_len=60)
    assert int(tg[0]) == top[0]


def test_sampling_rejected_on_non_last_stage():
    g = Stage(128, 4, 2, 512, 0, 1, dtype="bf16", max_ctx=8)
    with pytest.raises(BloomStageError, match="last stage"):
        g.set_sampling(7, 1.0, 1)
    t = Stage(128, 4, 2, 512, 1, 2, dtype="bf16", max_ctx=8)
    with pytest.raises(BloomStageError, match="top_k"):
        t.set_sampling(17, 1.0, 1)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_head_norm_and_slice_match_checker(dtype):
    """bs_head_norm (ln_f of each row's last position) and bs_head_slice (argmax keys of a 16-aligned
    vocabulary slice, merged with incoming keys) on a middle stage that holds a slice of the tied
    head, against or_head_norm / or_head_slice; then the slices of a 3-way split merged in ring
    order give the whole-vocabulary greedy token."""
    import torch
    h, nh, L, V, B, S = 512, 8, 4, 4096, 3, 5
    slices = [(0, 1376), (1376, 2752), (2752, 4096)]
    dev = torch.device("cuda", 0)
    o = OracleStage(h, nh, L, V, 0, 0, bf16=dtype == "bf16", max_batch=B, max_ctx=8, seed=6, is_first=False,
                    is_last=True)
    rng = np.random.default_rng(3)
    hidden = rng.standard_normal((B, S, h)).astype(np.float32)
    xo = o.head_norm(hidden, B, S)
    keys = None
    act = torch.bfloat16 if dtype == "bf16" else torch.float32
    for i, (v0, v1) in enumerate(slices):
        st = Stage(h, nh, L, V, 1 + i, 2 + i, dtype=dtype, max_batch=B, max_ctx=8, seed=6, is_first=False,
                   is_last=False, head_slice=(v0, v1))
        hid = torch.from_numpy(hidden).to(dev).reshape(-1)
        xn = torch.empty((B, h), dtype=act, device=dev)
        st.head_norm(hid, B, S, xn)
        torch.cuda.synchronize()
        check_close(xn.float().cpu().numpy(), xo, dtype, f"head_norm slice {i}")
        kin = None if keys is None else torch.from_numpy(keys.view(np.int64)).to(dev)
        kout = torch.empty(B, dtype=torch.int64, device=dev)
        tk = torch.empty(B, dtype=torch.int32, device=dev)
        st.head_slice(xn, B, kin, kout, tk)
        torch.cuda.synchronize()
        want_keys, want_tok = o.head_slice(xo, B, v0, v1, keys_in=keys)
        got_keys = kout.cpu().numpy().view(np.uint64)
        # the key's high word is the order-preserving image of the winning logit
        gv = _key_value(got_keys)
        wv = _key_value(want_keys)
        check_logits(gv, wv, dtype, f"head_slice {i} max logit")
        keys = want_keys  # the ring carries the checker's keys on (each hop checked on its own)
    _, full = o.forward(hidden, B, S, want_logits=True)
    assert_ids_match(tk.cpu().numpy(), np.argmax(full, axis=1), full, "ring token", tol=BF16_TOL)


def _key_value(keys):
    hi = (np.asarray(keys, np.uint64) >> np.uint64(32)).astype(np.uint32)
    u = np.where(hi & 0x80000000, hi & 0x7FFFFFFF, ~hi)
    return u.astype(np.uint32).view(np.float32)
