"""Weight-only int8 stages (BS_FLAG_INT8_WEIGHTS; SURVEY.md §8f row 4, the reference's bloom*-int8
variants, server.py:796-799) against the oracle with the same quantization (oracle/bloom_oracle.c
or_quantize_int8).  The reference's int8 ONNX modules come from the absent model_card export, so
the quantization rule is the build's own: parity is against the oracle restatement ("parity
unpinned" against the reference).  Tolerances as bf16 (tests/test_gpu_parity.py check_close):
the device GEMV applies the row scale after the reduction, the oracle per weight."""
import numpy as np
import pytest

from distributed_inference_demo_amd.stage import Stage
from oracle import gen_np
from oracle.oracle import OracleStage

from test_gpu_parity import assert_ids_match, canonical_weights, check_close, check_logits

pytestmark = pytest.mark.gpu


def pair8(h, nh, L, V, lb, le, seed=0, max_batch=1, max_ctx=128, max_tokens=0, is_first=None, is_last=None):
    g = Stage(h, nh, L, V, lb, le, dtype="bf16", max_batch=max_batch, max_ctx=max_ctx, max_tokens=max_tokens,
              seed=seed, is_first=is_first, is_last=is_last, int8_weights=True)
    o = OracleStage(h, nh, L, V, lb, le, bf16=True, max_batch=max_batch, max_ctx=max_ctx, seed=seed,
                    is_first=is_first, is_last=is_last, int8=True)
    return g, o


def test_device_quantization_is_bit_exact():
    """Device Q * scale (bs_read_weights) == the numpy rule applied to the bf16 weights, bit for bit;
    everything that is not a block matrix stays the bf16 weight."""
    h, nh, L, V = 128, 4, 2, 512
    w = gen_np.bf16_round(canonical_weights(4, h, L, V))
    st = Stage(h, nh, L, V, 0, L, dtype="bf16", max_ctx=8, seed=4, int8_weights=True)
    got = st.read_weights()
    want = w.copy()
    off = V * h + 2 * h
    sizes = [h, h, 3 * h * h, 3 * h, h * h, h, h, h, 4 * h * h, 4 * h, 4 * h * h, h]
    kdim = {2: h, 4: h, 8: h, 10: 4 * h}
    for _ in range(L):
        for t, n in enumerate(sizes):
            if t in kdim:
                K = kdim[t]
                q, sc = gen_np.int8_rows(w[off:off + n].reshape(-1, K))
                want[off:off + n] = (q.astype(np.float32) * sc[:, None]).reshape(-1)
            off += n
    bad = np.flatnonzero(got.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, (bad[:10], got[bad[:5]], want[bad[:5]])


def test_host_weights_int8_equal_synthetic():
    h, nh, L, V = 128, 4, 2, 512
    w = canonical_weights(4, h, L, V)
    ids = gen_np.prompt_ids(1, 1, 6, V).astype(np.int32)
    a = Stage(h, nh, L, V, 0, L, dtype="bf16", max_ctx=8, seed=4, int8_weights=True)
    b = Stage(h, nh, L, V, 0, L, dtype="bf16", max_ctx=8, host_weights=w, int8_weights=True)
    assert np.array_equal(a.read_weights().view(np.uint32), b.read_weights().view(np.uint32))
    _, la = a.forward_host(ids, 1, 6, want_logits=True)
    _, lb = b.forward_host(ids, 1, 6, want_logits=True)
    assert np.array_equal(la, lb)


@pytest.mark.parametrize("fam", ["560m", "1b1", "3b", "7b1"])
def test_int8_family_block_prefill_and_decode(fam):
    """One block at each family's real width: S=64 prefill (dequantized operand + bf16 GEMM), S=7
    after 15 cached (int8 GEMV, 7 rows), S=1 after 22 cached (int8 GEMV, 1 row)."""
    import os
    f = np.load(os.path.join(os.path.dirname(__file__), "golden", "family_blocks.npz"))
    h, nh, _, V, seed = (int(v) for v in f[fam + "_config"])
    gs, os_ = pair8(h, nh, 1, V, 0, 1, seed, max_ctx=64, max_tokens=64, is_last=False)
    check_close(gs.forward_host(f[fam + "_ids64"], 1, 64), os_.forward(f[fam + "_ids64"], 1, 64), "bf16",
                f"{fam} int8 S=64")
    ids = f[fam + "_ids23"]
    gs.forward_host(ids[:, :15], 1, 15, past_len=0)
    os_.forward(ids[:, :15], 1, 15, past_len=0)
    check_close(gs.forward_host(ids[:, 15:22], 1, 7, past_len=15), os_.forward(ids[:, 15:22], 1, 7, past_len=15),
                "bf16", f"{fam} int8 S=7 past=15")
    check_close(gs.forward_host(ids[:, 22:23], 1, 1, past_len=22), os_.forward(ids[:, 22:23], 1, 1, past_len=22),
                "bf16", f"{fam} int8 S=1 past=22")


@pytest.mark.parametrize("B", [1, 2, 4, 8, 20])
def test_int8_batched_greedy_decode(B):
    """Whole model (embedding .. argmax head), B rows at a slot offset: int8 GEMVs for B <= 8, the
    dequantized operand + batched bf16 GEMV above; logits within the bf16 bound, tokens agree."""
    h, nh, L, V = 512, 8, 3, 2048
    gs, os_ = pair8(h, nh, L, V, 0, L, seed=7, max_batch=B + 1, max_ctx=40, max_tokens=B * 8)
    ids = gen_np.prompt_ids(9, B, 8, V).astype(np.int32)
    tg, lg = gs.forward_host(ids, B, 8, slot=1, past_len=0, want_logits=True)
    to, lo = os_.forward(ids, B, 8, slot=1, past_len=0, want_logits=True)
    check_logits(lg, lo, "bf16", f"B={B} int8 prefill")
    assert_ids_match(tg, to, lo, f"B={B} int8 prefill")
    for step in range(6):
        tg, lg = gs.forward_host(to.reshape(B, 1), B, 1, slot=1, past_len=8 + step, want_logits=True)
        to, lo = os_.forward(to.reshape(B, 1), B, 1, slot=1, past_len=8 + step, want_logits=True)
        check_logits(lg, lo, "bf16", f"B={B} int8 decode step {step}")
        assert_ids_match(tg, to, lo, f"B={B} int8 decode step {step}")


def test_int8_long_context_graph_decode():
    """Graph-replayed S=1 decode (device I/O, hipGraph) of a 1b1-width stage over a context long
    enough for split attention (merged by the attention kernel: the int8 dense GEMV reads ctx)."""
    import torch
    h, nh, L, V, P = 1536, 16, 2, 1024, 1000
    gs, os_ = pair8(h, nh, L, V, 0, L, seed=5, max_ctx=P + 40, max_tokens=P)
    ids = gen_np.prompt_ids(3, 1, P, V).astype(np.int32)
    dev = torch.device("cuda", 0)
    cs = torch.cuda.Stream()
    with torch.cuda.stream(cs):
        tin = torch.from_numpy(ids).to(dev)
        tok = torch.empty(1, dtype=torch.int32, device=dev)
        lg = torch.empty((1, V), dtype=torch.float32, device=dev)
        gs.forward(tin, tok, 1, P, slot=0, past_len=0, logits=lg, stream=cs.cuda_stream)
        to, lo = os_.forward(ids, 1, P, want_logits=True)
        torch.cuda.synchronize()
        check_logits(lg.cpu().numpy(), lo, "bf16", "int8 prefill logits")
        for step in range(24):
            tok.copy_(torch.from_numpy(to))
            gs.forward(tok, tok, 1, 1, slot=0, past_len=P + step, logits=lg, stream=cs.cuda_stream)
            to, lo = os_.forward(to.reshape(1, 1), 1, 1, past_len=P + step, want_logits=True)
            if step % 5 == 0 or step == 23:
                torch.cuda.synchronize()
                check_logits(lg.cpu().numpy(), lo, "bf16", f"int8 graph decode step {step}")


def test_serve_run_int8_on_gpu_matches_oracle():
    """serve.py lifecycle on one GPU with an int8 model (bf16 stage, BS_FLAG_INT8_WEIGHTS): 4 samples,
    2 in flight; each sample's greedy ids against the int8 oracle decoding it alone, teacher-forced
    with the served ids: every id equal unless the oracle's top-2 margin at that step is < 2e-2."""
    import torch
    from distributed_inference_demo_amd.config import BloomDims
    from distributed_inference_demo_amd.serve import RunConfig, run_rank, synthetic_prompts
    model = BloomDims("tinygpu-int8", 256, 2, 4, vocab=1024, int8_weights=True)
    cfg = RunConfig(model=model, num_sample=4, max_length=8, core_pool_size=2, prompt_len=9, dtype="bf16", seed=13)
    res = run_rank(cfg, 0, 1, torch.device("cuda", 0))
    for got, p in zip(res["samples"], synthetic_prompts(cfg, model.vocab)):
        o = OracleStage(256, 4, 2, 1024, 0, 2, bf16=True, max_batch=1, max_ctx=32, seed=13, int8=True)
        tok, lo = o.forward(np.array(p, np.int32).reshape(1, -1), 1, len(p), want_logits=True)
        assert_ids_match([got[0]], tok, lo, "int8 serve first id")
        for i in range(cfg.max_length - 1):
            tok, lo = o.forward(np.array([[got[i]]], np.int32), 1, 1, past_len=len(p) + i,  # teacher-forced
                                want_logits=True)
            assert_ids_match([got[i + 1]], tok, lo, f"int8 serve id {i + 1}")
