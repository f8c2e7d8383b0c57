"""GPU parity tests: libbloomstage.so (HIP, gfx950) through its C-ABI against the CPU checker
(oracle/bloom_oracle.c, itself pinned to HF BLOOM by test_oracle_golden.py) and the HF golden
fixtures.

Tolerances (BASELINE.json north_star):
  fp32 mode: max|gpu - ref| <= 1e-3 * max|ref| (relative 1e-3), and identical greedy ids.
  bf16 mode: logits max|gpu - ref| <= 2e-2 (north_star) where |logits| <= 8; hidden states
             max|gpu - ref| <= 2e-2 + 2^-9 * max|ref| (ref = oracle with the same bf16 storage
             roundings): the north-star 2e-2 plus half a bf16 ulp of the largest output.  The extra
             term matters only for wide blocks (bloom-3b/7b1, outputs up to 13): there every
             intermediate rounded to bf16 (LayerNorm out, q/K/V, attention context, GELU out) flips with
             the accumulation order of the sums that produce it, and the flips spread over the whole
             row.  A float64 restatement of the same rounded math lands 0.011 max / 0.0021 mean from
             the fp32 checker on a bloom-7b1-width block and the GPU 0.017 / 0.0034 (tools/diag_parity.py,
             DESIGN.md section 2): the error is the rounding noise of the format, not of the kernels.
"""
import json
import os

import numpy as np
import pytest

from distributed_inference_demo_amd.stage import (BloomStageError, Stage, create_session, deserialize_int,
                                                  deserialize_tensors,
                                                  run_inference_master_residual, run_inference_worker_residual,
                                                  run_inference_worker_residual_last_generation)
from distributed_inference_demo_amd.config import BloomDims
from oracle import gen_np
from oracle.oracle import EMUL_DEVICE, OracleStage

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
BF16_TOL = 2e-2
FP32_REL = 1e-3
# bf16 against the checker that also emulates the device's P.V staging (TwinChecker), relative to max|ref| of the
# checked tensor (logits or hidden states).  Applied where no bf16 rounding flips occur (small dimensions, few rows:
# smoke, tiny splits, B <= 4 decode); there the round-6 measurement is <= 1.2e-5 relative, against 6e-4 for the
# default-order checker (profiles/r06_parity_errors.jsonl "tight" records).  At real widths
# the flips dominate both checkers alike; tests/test_gpu_attention_exact.py pins the attention kernels there.
TIGHT_REL = 5e-5


def pair(h, nh, L, V, lb, le, dtype, seed=0, max_batch=1, max_ctx=128, max_tokens=0, is_first=None, is_last=None,
         twin=False):
    """Device stage + checker; twin (bf16): the checker is a TwinChecker (default + emulating)."""
    g = Stage(h, nh, L, V, lb, le, dtype=dtype, max_batch=max_batch, max_ctx=max_ctx, max_tokens=max_tokens,
              seed=seed, is_first=is_first, is_last=is_last)
    mk = TwinChecker if (twin and dtype == "bf16") else OracleStage
    o = mk(h, nh, L, V, lb, le, bf16=(dtype == "bf16"), max_batch=max_batch, max_ctx=max_ctx, seed=seed,
           is_first=is_first, is_last=is_last)
    return g, o


class TwinChecker:
    """The bf16 checker twice, fed the same inputs: in its default order (what the format-noise bounds compare
    against) and emulating the device's P.V staging (oracle EMUL_DEVICE: bf16 hi + lo P against bf16 V, normalised
    after the product, in the prefill kernel; fp32 unnormalised P in the decode kernel).  forward() returns the
    default checker's result; the emulating twin's is kept in .tight (logits when the stage is last, else the
    hidden states) for check_tight."""

    def __init__(self, *a, **k):
        self.o = OracleStage(*a, **k)
        self.t = OracleStage(*a, emul_pv=EMUL_DEVICE, **k)
        self.tight = None

    def forward(self, x, B, S, slot=0, past_len=0, want_logits=False):
        r = self.o.forward(x, B, S, slot=slot, past_len=past_len, want_logits=want_logits)
        t = self.t.forward(x, B, S, slot=slot, past_len=past_len, want_logits=want_logits)
        self.tight = t[1] if want_logits else t
        return r

    def close(self):
        self.o.close()
        self.t.close()


def check_tight(got, ref, what="", rel=TIGHT_REL):
    """bf16 device against the emulating checker (TwinChecker.tight): max-abs <= rel * max|ref|."""
    bound = rel * float(np.abs(ref).max())
    err = record_error(what + " [emulating checker]", got, ref, bound, "tight bf16")
    assert err <= bound, f"{what}: max-abs {err} > {bound} against the emulating checker"
    return err


def record_error(what, got, ref, bound, kind):
    """Append this check's achieved error and its bound to the parity log (JSON lines, the file $BS_PARITY_LOG
    names; nothing is written when it is unset), so the margin to every bound is on record, not only pass/fail."""
    d = np.abs(np.asarray(got, np.float64) - np.asarray(ref, np.float64))
    rec = {"test": os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0], "check": what, "kind": kind,
           "max_abs": float(d.max()) if d.size else 0.0, "mean_abs": float(d.mean()) if d.size else 0.0,
           "max_ref": float(np.abs(ref).max()) if np.size(ref) else 0.0, "bound": float(bound)}
    path = os.environ.get("BS_PARITY_LOG")
    if not path:
        return rec["max_abs"]
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")
    except OSError:
        pass
    return rec["max_abs"]


def check_close(got, ref, dtype, what=""):
    if dtype == "bf16":
        tol = BF16_TOL + 2.0 ** -9 * float(np.abs(ref).max())
    else:
        tol = FP32_REL * float(np.abs(ref).max())
    err = record_error(what, got, ref, tol, f"hidden {dtype}")
    assert err <= tol, f"{what}: max-abs {err} > {tol}"
    return err


def check_bf16_stored(got, ref, what=""):
    """Values the device STORES in bf16 (the K/V cache): the hidden-state bound plus one bf16 ulp of the
    largest |ref|.  Two correct paths whose fp32 pre-rounding values straddle a rounding boundary store
    adjacent bf16 numbers, a full ulp apart (2^-7 relative: 0.03125 for a cached value in [4, 8), which
    the first bloom-7b1-width prefill measured), so the half-ulp term of check_close is one flip short."""
    mx = float(np.abs(ref).max())
    ulp = 2.0 ** (np.floor(np.log2(mx)) - 7) if mx > 0 else 0.0
    tol = BF16_TOL + 2.0 ** -9 * mx + ulp
    err = record_error(what, got, ref, tol, "kv bf16")
    assert err <= tol, f"{what}: max-abs {err} > {tol}"
    return err


def check_logits(got, ref, dtype, what=""):
    """Logits: north_star's flat 2e-2 max-abs in bf16 (relative 1e-3 in fp32)."""
    tol = BF16_TOL if dtype == "bf16" else FP32_REL * float(np.abs(ref).max())
    err = record_error(what, got, ref, tol, f"logits {dtype}")
    assert err <= tol, f"{what}: logits max-abs {err} > {tol}"
    return err


def assert_ids_match(got, ref_ids, ref_logits, what="", tol=BF16_TOL):
    """Greedy ids equal to the checker's, except rows whose checker top-2 logit margin is < tol
    (a near-tie inside the bf16 tolerance may legitimately pick either token)."""
    got, ref_ids = np.asarray(got).reshape(-1), np.asarray(ref_ids).reshape(-1)
    ref_logits = np.asarray(ref_logits).reshape(len(ref_ids), -1)
    for b in np.flatnonzero(got != ref_ids):
        top2 = np.sort(ref_logits[b])[-2:]
        assert top2[1] - top2[0] < tol, f"{what}: row {b} id {got[b]} != {ref_ids[b]}, checker top-2 {top2}"


def test_tiny_fp32_matches_hf_golden_and_greedy_128():
    g = np.load(os.path.join(G, "tiny_e2e.npz"))
    h, nh, L, V, seed, B, S = (int(v) for v in g["config"])
    st = Stage(h, nh, L, V, 0, L, dtype="fp32", max_batch=B, max_ctx=S + 128, seed=seed)
    tok, lg = st.forward_host(g["ids"], B, S, want_logits=True)
    check_logits(lg, g["logits"], "fp32", "tiny logits vs HF")
    toks = [tok]
    for i in range(127):
        toks.append(st.forward_host(toks[-1].reshape(B, 1), B, 1))
    assert np.array_equal(np.stack(toks, 1), g["greedy"])


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_tiny_stage_splits_match_oracle(dtype):
    g = np.load(os.path.join(G, "tiny_e2e.npz"))
    h, nh, L, V, seed, B, S = (int(v) for v in g["config"])
    tw = dtype == "bf16"
    for split in (1, 2, 3):
        g0, o0 = pair(h, nh, L, V, 0, split, dtype, seed, max_batch=B, max_ctx=32, twin=tw)
        g1, o1 = pair(h, nh, L, V, split, L, dtype, seed, max_batch=B, max_ctx=32, twin=tw)
        hid_g = g0.forward_host(g["ids"], B, S)
        hid_o = o0.forward(g["ids"], B, S)
        check_close(hid_g, hid_o, dtype, f"stage0 [0,{split})")
        if tw:
            check_tight(hid_g, o0.tight, f"stage0 [0,{split})")
        if dtype == "fp32":
            check_close(hid_g, g["layer_out"][split - 1], dtype, "stage0 vs HF")
        tg, lg = g1.forward_host(hid_o, B, S, want_logits=True)
        to, lo = o1.forward(hid_o, B, S, want_logits=True)
        check_logits(lg, lo, dtype, "stage1 logits")
        if tw:
            check_tight(lg, o1.tight, f"stage1 [{split},{L}) logits")
        assert np.array_equal(tg, to)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("fam", ["560m", "1b1", "3b", "7b1"])
def test_family_block_prefill_and_decode(fam, dtype):
    f = np.load(os.path.join(G, "family_blocks.npz"))
    h, nh, _, V, seed = (int(v) for v in f[fam + "_config"])
    gs, os_ = pair(h, nh, 1, V, 0, 1, dtype, seed, max_ctx=64, max_tokens=64, is_last=False)
    out_g = gs.forward_host(f[fam + "_ids64"], 1, 64)
    out_o = os_.forward(f[fam + "_ids64"], 1, 64)
    check_close(out_g, out_o, dtype, f"{fam} S=64")
    if dtype == "fp32":
        check_close(out_g, f[fam + "_out64"], dtype, f"{fam} S=64 vs HF")
    ids = f[fam + "_ids23"]
    gs.forward_host(ids[:, :15], 1, 15, past_len=0)
    os_.forward(ids[:, :15], 1, 15, past_len=0)
    o7g = gs.forward_host(ids[:, 15:22], 1, 7, past_len=15)
    o7o = os_.forward(ids[:, 15:22], 1, 7, past_len=15)
    check_close(o7g, o7o, dtype, f"{fam} S=7 past=15")
    o1g = gs.forward_host(ids[:, 22:23], 1, 1, past_len=22)
    o1o = os_.forward(ids[:, 22:23], 1, 1, past_len=22)
    check_close(o1g, o1o, dtype, f"{fam} S=1 past=22")
    if dtype == "fp32":
        check_close(o7g, f[fam + "_out7"], dtype, "S=7 vs HF")
        check_close(o1g, f[fam + "_out1"], dtype, "S=1 vs HF")


@pytest.mark.parametrize("B", [3, 20, 32])
def test_batched_decode_with_slot_offset(B):
    """Rows at a slot offset; B > 16 exercises the two-m-tile GEMV; B*S > 32 the MFMA GEMM."""
    h, nh, L, V = 256, 4, 2, 1024
    tw = B <= 4  # the emulating checker's tight bound where the rows GEMV runs (wider batches: flip noise)
    gs, os_ = pair(h, nh, L, V, 0, L, "bf16", seed=3, max_batch=B + 2, max_ctx=40, max_tokens=B * 8, twin=tw)
    ids = gen_np.prompt_ids(5, B, 8, V).astype(np.int32)
    tg, lg = gs.forward_host(ids, B, 8, slot=2, past_len=0, want_logits=True)
    to, lo = os_.forward(ids, B, 8, slot=2, past_len=0, want_logits=True)
    check_logits(lg, lo, "bf16", "prefill")
    if tw:
        check_tight(lg, os_.tight, f"B={B} prefill")
    assert_ids_match(tg, to, lo, "prefill")
    for step in range(4):
        tg, lg = gs.forward_host(to.reshape(B, 1), B, 1, slot=2, past_len=8 + step, want_logits=True)
        to, lo = os_.forward(to.reshape(B, 1), B, 1, slot=2, past_len=8 + step, want_logits=True)
        check_logits(lg, lo, "bf16", f"decode step {step}")
        if tw:
            check_tight(lg, os_.tight, f"B={B} decode step {step}")
        assert_ids_match(tg, to, lo, f"decode step {step}")


@pytest.mark.parametrize("B", [8, 32])
def test_batched_decode_real_width_split_k(B):
    """bloom-1b1 width (h = 1536, 16 heads): the batched tile GEMV with split-K on the N = h GEMVs
    (dense: 2 splits, fc2: 4 splits), the one-block-per-row LayerNorm feeding it, and the argmax head."""
    h, nh, L, V = 1536, 16, 1, 2048
    gs, os_ = pair(h, nh, L, V, 0, L, "bf16", seed=11, max_batch=B, max_ctx=24, max_tokens=B * 4)
    ids = gen_np.prompt_ids(6, B, 4, V).astype(np.int32)
    tg = gs.forward_host(ids, B, 4, slot=0, past_len=0)
    to = os_.forward(ids, B, 4, slot=0, past_len=0)
    for step in range(3):
        tg_n, lg = gs.forward_host(to.reshape(B, 1), B, 1, slot=0, past_len=4 + step, want_logits=True)
        to_n, lo = os_.forward(to.reshape(B, 1), B, 1, slot=0, past_len=4 + step, want_logits=True)
        check_logits(lg, lo, "bf16", f"B={B} decode step {step}")
        assert_ids_match(tg_n, to_n, lo, f"B={B} decode step {step}")
        tg, to = tg_n, to_n


def test_prefill_large_gemm_tiles():
    """B*S = 1024 tokens: fc1 goes through the 128x128 MFMA tile, others through 64x64."""
    h, nh, V = 1024, 16, 1024
    gs, os_ = pair(h, nh, 1, V, 0, 1, "bf16", seed=9, max_batch=2, max_ctx=512, max_tokens=1024, is_last=False)
    ids = gen_np.prompt_ids(8, 2, 512, V).astype(np.int32)
    check_close(gs.forward_host(ids, 2, 512), os_.forward(ids, 2, 512), "bf16", "prefill 2x512")


def test_nonpow2_heads_fp32_matches_hf():
    g = np.load(os.path.join(G, "tiny_nonpow2.npz"))
    h, nh, L, V, seed, B, S = (int(v) for v in g["config"])
    st = Stage(h, nh, L, V, 0, L, dtype="fp32", max_batch=B, max_ctx=S, seed=seed)
    _, lg = st.forward_host(g["ids"], B, S, want_logits=True)
    check_logits(lg, g["logits"], "fp32", "nonpow2 logits vs HF")


def canonical_weights(seed, h, L, V, lb=0, le=None, first=True, last=True):
    """The BS_WEIGHTS_HOST layout built from the numpy generator."""
    le = L if le is None else le
    sd = gen_np.hf_state_dict(seed, h, L, V)
    flat = []
    if first or last:
        flat.append(sd["transformer.word_embeddings.weight"])
    if first:
        flat += [sd["transformer.word_embeddings_layernorm.weight"], sd["transformer.word_embeddings_layernorm.bias"]]
    names = ["input_layernorm.weight", "input_layernorm.bias", "self_attention.query_key_value.weight",
             "self_attention.query_key_value.bias", "self_attention.dense.weight", "self_attention.dense.bias",
             "post_attention_layernorm.weight", "post_attention_layernorm.bias", "mlp.dense_h_to_4h.weight",
             "mlp.dense_h_to_4h.bias", "mlp.dense_4h_to_h.weight", "mlp.dense_4h_to_h.bias"]
    for l in range(lb, le):
        flat += [sd[f"transformer.h.{l}.{n}"] for n in names]
    if last:
        flat += [sd["transformer.ln_f.weight"], sd["transformer.ln_f.bias"]]
    return np.concatenate([a.reshape(-1) for a in flat])


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_device_generator_is_bit_exact(dtype):
    h, nh, L, V = 64, 4, 3, 512
    w = canonical_weights(4, h, L, V, 1, 3, first=False, last=True)
    st = Stage(h, nh, L, V, 1, 3, dtype=dtype, max_ctx=8, seed=4)
    got = st.read_weights()
    want = w if dtype == "fp32" else gen_np.bf16_round(w)
    assert got.shape == want.shape
    bad = np.flatnonzero(got.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, (bad[:10], got[bad[:5]], want[bad[:5]])


def test_host_weights_equal_synthetic():
    h, nh, L, V = 64, 4, 2, 512
    w = canonical_weights(4, h, L, V)
    ids = gen_np.prompt_ids(1, 1, 6, V).astype(np.int32)
    a = Stage(h, nh, L, V, 0, L, dtype="fp32", max_ctx=8, seed=4)
    b = Stage(h, nh, L, V, 0, L, dtype="fp32", max_ctx=8, host_weights=w)
    assert np.array_equal(b.read_weights().view(np.uint32), w.view(np.uint32))
    assert np.array_equal(a.read_weights().view(np.uint32), w.view(np.uint32))
    _, la = a.forward_host(ids, 1, 6, want_logits=True)
    _, lb = b.forward_host(ids, 1, 6, want_logits=True)
    assert np.array_equal(la, lb)


def test_jni_mirror_entry_points_two_stage_loopback():
    """createSession / runInference{Master,Worker,...LastGeneration} / deserializeInt shape."""
    m = BloomDims("tiny", 64, 4, 4, vocab=512)
    g = np.load(os.path.join(G, "tiny_e2e.npz"))
    head = create_session(m, 0, 2, dtype="fp32", max_ctx=64)
    tail = create_session(m, 2, 4, dtype="fp32", max_ctx=64)
    ids = list(g["ids"][0])
    toks = []
    seq, res = run_inference_master_residual(head, ids)
    assert res == []
    for _ in range(8):
        tok = deserialize_int(run_inference_worker_residual_last_generation(tail, seq, res, k=1))
        toks.append(tok)
        seq, res = run_inference_master_residual(head, [tok])
    assert toks == list(g["greedy"][0][:8])


def test_jni_mirror_middle_entry_three_stage_loopback():
    """Header -> middle (runInferenceWorkerResidual, native-lib.cpp:1036-1194) -> tail, every hop
    as the utils.cpp wire bytes; greedy ids equal the HF golden fixture."""
    m = BloomDims("tiny", 64, 4, 4, vocab=512)
    g = np.load(os.path.join(G, "tiny_e2e.npz"))
    head = create_session(m, 0, 1, dtype="fp32", max_ctx=64)
    mid = create_session(m, 1, 3, dtype="fp32", max_ctx=64)
    tail = create_session(m, 3, 4, dtype="fp32", max_ctx=64)
    ids = list(g["ids"][0])
    toks = []
    seq, res = run_inference_master_residual(head, ids)
    for _ in range(8):
        seq2, res2 = run_inference_worker_residual(mid, seq, res)
        assert res2 == []
        (hid,) = deserialize_tensors(seq2)
        assert hid.dtype == np.float32 and hid.shape[-1] == m.hidden
        tok = deserialize_int(run_inference_worker_residual_last_generation(tail, seq2, res2, k=1))
        toks.append(tok)
        seq, res = run_inference_master_residual(head, [tok])
    assert toks == list(g["greedy"][0][:8])


def test_errors_are_status_codes_not_crashes():
    st = Stage(64, 4, 4, 512, 0, 4, dtype="bf16", max_ctx=8)
    with pytest.raises(BloomStageError, match="max_ctx"):
        st.forward_host(np.zeros((1, 9), np.int32), 1, 9)
    with pytest.raises(BloomStageError, match="token id"):
        st.forward_host(np.full((1, 2), 512, np.int32), 1, 2)
    with pytest.raises(BloomStageError):
        Stage(66, 4, 4, 512, 0, 4)
    with pytest.raises(BloomStageError, match="slot"):
        st.forward_host(np.zeros((2, 1), np.int32), 2, 1)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_graph_replayed_decode_matches_oracle_long_context(dtype):
    """Device-buffer decode steps replay a captured hipGraph (past_len read from HBM); contexts
    of 200-330 positions span 4-6 attention chunks, exercising the last-arriver merge."""
    import torch
    h, nh, L, V, B, P = 256, 4, 2, 1024, 3, 200
    gs, os_ = pair(h, nh, L, V, 0, L, dtype, seed=21, max_batch=B, max_ctx=P + 140, max_tokens=B * P)
    ids = gen_np.prompt_ids(17, B, P, V).astype(np.int32)
    dev = torch.device("cuda", 0)
    cs = torch.cuda.Stream()
    with torch.cuda.stream(cs):
        tin = torch.from_numpy(ids).to(dev)
        tok = torch.empty(B, dtype=torch.int32, device=dev)
        lg = torch.empty((B, V), dtype=torch.float32, device=dev)
        gs.forward(tin, tok, B, P, slot=0, past_len=0, logits=lg, stream=cs.cuda_stream)
        to, lo = os_.forward(ids, B, P, want_logits=True)
        torch.cuda.synchronize()
        check_logits(lg.cpu().numpy(), lo, dtype, "prefill logits")
        for step in range(130):
            tok.copy_(torch.from_numpy(to))  # teacher-force the oracle's tokens
            gs.forward(tok, tok, B, 1, slot=0, past_len=P + step, logits=lg, stream=cs.cuda_stream)
            to, lo = os_.forward(to.reshape(B, 1), B, 1, past_len=P + step, want_logits=True)
            if step % 13 == 0 or step == 129:
                torch.cuda.synchronize()
                check_logits(lg.cpu().numpy(), lo, dtype, f"decode step {step} (ctx {P + step + 1})")


def test_graph_and_eager_paths_agree_bitwise():
    """Replays of the captured decode graph give the same bits as the eager launch sequence
    (bs_set_graphs(0) on a twin stage): 20 decode steps of 2 rows, logits compared bit for bit."""
    import torch
    from oracle import gen_np
    out = {}
    for graphs in (True, False):
        st = Stage(256, 4, 2, 1024, 0, 2, max_batch=2, max_ctx=64, seed=5)
        st.set_graphs(graphs)
        cs = torch.cuda.Stream()
        with torch.cuda.stream(cs):
            ids = torch.from_numpy(gen_np.prompt_ids(3, 2, 10, 1024).astype(np.int32)).cuda()
            tok = torch.empty(2, dtype=torch.int32, device="cuda")
            lg = torch.empty((2, 1024), device="cuda")
            st.forward(ids, tok, 2, 10, past_len=0, stream=cs.cuda_stream)
            steps = []
            for i in range(20):
                st.forward(tok, tok, 2, 1, past_len=10 + i, logits=lg, stream=cs.cuda_stream)
                steps.append(lg.cpu().numpy())
        st.close()
        out[graphs] = np.stack(steps)
    assert np.array_equal(out[True], out[False])


def test_stream_switch_rewrites_positions():
    """bs_forward's set_past shortcut is taken only on the stream the previous forward advanced past_dev on:
    decode steps alternating between two streams (each ordered behind the other by an event wait, the
    contract in include/bloomstage.h) keep every row at its own position -- logits against the checker."""
    import torch
    h, nh, L, V, B, P = 256, 4, 2, 1024, 3, 12
    gs, os_ = pair(h, nh, L, V, 0, L, "bf16", seed=41, max_batch=B, max_ctx=P + 16, max_tokens=B * P)
    ids = gen_np.prompt_ids(13, B, P, V).astype(np.int32)
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    tok = torch.empty(B, dtype=torch.int32, device=dev)
    lg = torch.empty((B, V), dtype=torch.float32, device=dev)
    with torch.cuda.stream(streams[0]):
        tin = torch.from_numpy(ids).to(dev)
        gs.forward(tin, tok, B, P, slot=0, past_len=0, stream=streams[0].cuda_stream)
    to = os_.forward(ids, B, P)
    for step in range(8):
        cur, prev = streams[(step + 1) % 2], streams[step % 2]
        cur.wait_stream(prev)
        with torch.cuda.stream(cur):
            tok.copy_(torch.from_numpy(to))
            gs.forward(tok, tok, B, 1, slot=0, past_len=P + step, logits=lg, stream=cur.cuda_stream)
        to, lo = os_.forward(to.reshape(B, 1), B, 1, past_len=P + step, want_logits=True)
        cur.synchronize()
        check_logits(lg.cpu().numpy(), lo, "bf16", f"stream-switched decode step {step}")
        assert_ids_match(tok.cpu().numpy(), to, lo, f"stream-switched decode step {step}")


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_split_kv_decode_attention(dtype):
    """B*heads small and max_ctx large: the context is split over several blocks and merged;
    short contexts leave trailing splits empty."""
    h, nh, L, V, B = 256, 4, 1, 1024, 1
    gs, os_ = pair(h, nh, L, V, 0, L, dtype, seed=33, max_batch=B, max_ctx=1100, max_tokens=700, is_last=False)
    ids = gen_np.prompt_ids(4, B, 700, V).astype(np.int32)
    # short prompt -> decode: one chunk, empty splits
    check_close(gs.forward_host(ids[:, :5], B, 5, past_len=0), os_.forward(ids[:, :5], B, 5, past_len=0), dtype, "p5")
    for p in (5, 6, 63, 64):
        check_close(gs.forward_host(ids[:, p:p + 1], B, 1, past_len=p), os_.forward(ids[:, p:p + 1], B, 1, past_len=p),
                    dtype, f"decode past={p}")
    # long prefix -> decode across many chunks
    gs.forward_host(ids[:, 65:700], B, 635, past_len=65)
    os_.forward(ids[:, 65:700], B, 635, past_len=65)
    for p in (700, 701):
        tok = ids[:, (p * 7) % 700:(p * 7) % 700 + 1]
        check_close(gs.forward_host(tok, B, 1, past_len=p), os_.forward(tok, B, 1, past_len=p), dtype, f"decode past={p}")


@pytest.mark.parametrize("B,slot,hd", [(1, 0, 96), (2, 0, 64), (1, 1, 128), (2, 1, 80)])
def test_small_batch_decode_from_empty_cache(B, slot, hd):
    """Graph-replayed decode for B <= 2 rows at the real head widths (1b1 96, 560m 64, 7b1 128,
    3b 80), from an EMPTY cache (past 0: the new position is the whole softmax) through 300
    positions (1..5 split-attention chunks), with a slot offset — against the oracle, teacher
    forced, at the listed steps."""
    import torch
    nh = 4 if hd != 80 else 8
    h, L, V = nh * hd, 2, 1024
    gs, os_ = pair(h, nh, L, V, 0, L, "bf16", seed=31, max_batch=slot + B, max_ctx=320, max_tokens=B * 300, twin=True)
    dev = torch.device("cuda", 0)
    cs = torch.cuda.Stream()
    with torch.cuda.stream(cs):
        tok = torch.empty(B, dtype=torch.int32, device=dev)
        lg = torch.empty((B, V), dtype=torch.float32, device=dev)
        # from an empty cache: S = 1 at past 0 (the new-position partial is the whole softmax)
        to = gen_np.prompt_ids(5, B, 1, V).astype(np.int32).reshape(B)
        past = 0
        steps = list(range(0, 12)) + [130, 131, 255, 256, 257, 299]
        for step in range(300):
            tok.copy_(torch.from_numpy(to))
            gs.forward(tok, tok, B, 1, slot=slot, past_len=past, logits=lg, stream=cs.cuda_stream)
            to_next, lo = os_.forward(to.reshape(B, 1), B, 1, past_len=past, slot=slot, want_logits=True)
            if step in steps:
                torch.cuda.synchronize()
                check_logits(lg.cpu().numpy(), lo, "bf16", f"fused decode step {step} (ctx {past + 1})")
                check_tight(lg.cpu().numpy(), os_.tight, f"hd={hd} fused decode step {step} (ctx {past + 1})")
            to = to_next
            past += 1


@pytest.mark.parametrize("ragged", [False, True])
def test_serve_run_on_gpu_matches_oracle_per_sample(ragged):
    """serve.py lifecycle on one GPU (fp32 stage): 5 samples, 2 (or 3) rows in flight with continuous
    admission (a row takes the next sample when its sample finishes; ragged: prompts of 2..11 tokens, so
    rows sit at different positions in every graph-replayed step), each sample's 8 greedy ids equal to
    the fp32 oracle decoding that sample alone."""
    import torch
    from distributed_inference_demo_amd.serve import RunConfig, run_rank, synthetic_prompts
    model = BloomDims("tinygpu", 256, 2, 4, vocab=1024)  # 2 layers, 4 heads
    cfg = RunConfig(model=model, num_sample=5, max_length=8, core_pool_size=3 if ragged else 2, prompt_len=9,
                    dtype="fp32", seed=11)
    prompts = synthetic_prompts(cfg, model.vocab)
    if ragged:
        prompts = [p[:n] + p[:max(0, n - len(p))] for p, n in zip(prompts, (2, 11, 5, 9, 3))]
    res = run_rank(cfg, 0, 1, torch.device("cuda", 0), prompts=prompts)
    want = []
    for p in prompts:
        o = OracleStage(256, 4, 2, 1024, 0, 2, bf16=False, max_batch=1, max_ctx=32, seed=11)
        tok = o.forward(np.array(p, np.int32).reshape(1, -1), 1, len(p))
        ids = [int(tok[0])]
        for i in range(cfg.max_length - 1):
            tok = o.forward(tok.reshape(1, 1), 1, 1, past_len=len(p) + i)
            ids.append(int(tok[0]))
        want.append(ids)
    assert res["samples"] == want
