"""Full-size parity on the real BLOOM configurations (BASELINE.json configs[1] and north_star's
128-token greedy identity), through the C-ABI against the CPU checker (oracle/bloom_oracle.c).

Reference tail these pin: run_inference_with_decoding (inference.cpp:272-327) and the tail JNI
entry (native-lib.cpp:1368-1443) -- here the greedy pick of the full V = 250880 vocabulary.

  * bloom-1b1, all 24 layers, V = 250880, B = 1: a 512-token prefill, then 128 graph-replayed decode
    steps on device buffers (north_star's fixed 128-token decode; teacher-forced with the checker's tokens,
    so every step compares logits from the same inputs).  bf16 mode against the
    bf16-mode checker (same storage roundings): the greedy id equal to the checker's unless the
    checker's own top-2 margin is < 2e-2 (north_star's id criterion); logits mean-abs <= 4e-3 and
    max-abs <= 2.5e-2.  The max bound is above north_star's example 2e-2 at this depth because the
    bf16 rounding-flip noise of the format is already that large between two CORRECT device paths:
    the fused attention + dense path and the split one differ from each other by up to 0.015 and
    from the checker by 0.0195 / 0.0201 max, 0.0030 mean, on every step alike
    (profiles/r02_attn_dense_numerics.txt, tools/diag_fused.py); reduced-depth tests keep 2e-2.
  * bloom-560m, all 24 layers, fp32: a 16-token prompt, then 128 greedy ids identical to the fp32
    checker's (north_star: "identical greedy token IDs over a fixed 128-token decode").
"""
import numpy as np
import pytest

from distributed_inference_demo_amd import config
from distributed_inference_demo_amd.stage import Stage
from oracle.oracle import OracleStage, prompt_ids

from test_gpu_parity import assert_ids_match

pytestmark = pytest.mark.gpu

BF16_FULL_TOL = 2.5e-2       # logits max-abs, full depth (see the module docstring)
BF16_FULL_MEAN_TOL = 4e-3    # logits mean-abs, full depth


def test_bloom1b1_full_prefill512_then_graph_decode_bf16():
    import torch
    m = config.get("bloom-1b1")
    P, STEPS = 512, 128
    g = Stage(m.hidden, m.n_head, m.n_layer, m.vocab, 0, m.n_layer, dtype="bf16", max_batch=1,
              max_ctx=P + STEPS + 1, max_tokens=P, seed=0)
    o = OracleStage(m.hidden, m.n_head, m.n_layer, m.vocab, 0, m.n_layer, bf16=True, max_batch=1,
                    max_ctx=P + STEPS + 1, seed=0)
    ids = prompt_ids(1234, 1, P, m.vocab)
    dev = torch.device("cuda", 0)
    cs = torch.cuda.Stream()
    errs, means, same = [], [], 0
    with torch.cuda.stream(cs):
        tin = torch.from_numpy(ids).to(dev)
        tok = torch.empty(1, dtype=torch.int32, device=dev)
        lg = torch.empty((1, m.vocab), dtype=torch.float32, device=dev)
        g.forward(tin, tok, 1, P, past_len=0, logits=lg, stream=cs.cuda_stream)
        to, lo = o.forward(ids, 1, P, want_logits=True)
        torch.cuda.synchronize()
        gl, gt = lg.cpu().numpy(), tok.cpu().numpy()
        errs.append(float(np.abs(gl - lo).max()))
        means.append(float(np.abs(gl - lo).mean()))
        assert_ids_match(gt, to, lo, "prefill")
        for step in range(STEPS):
            tok.copy_(torch.from_numpy(to))  # teacher-force the checker's token
            g.forward(tok, tok, 1, 1, past_len=P + step, logits=lg, stream=cs.cuda_stream)
            to, lo = o.forward(to.reshape(1, 1), 1, 1, past_len=P + step, want_logits=True)
            torch.cuda.synchronize()
            gl, gt = lg.cpu().numpy(), tok.cpu().numpy()
            errs.append(float(np.abs(gl - lo).max()))
            means.append(float(np.abs(gl - lo).mean()))
            assert_ids_match(gt, to, lo, f"decode step {step}")
            same += int(gt[0] == to[0])
    print(f"bloom-1b1 full: {same}/{STEPS} decode ids identical to the checker's (the rest are top-2 ties < 2e-2); "
          f" logits max-abs prefill {errs[0]:.3e}, decode max {max(errs[1:]):.3e} median {float(np.median(errs[1:])):.3e}, "
          f"max |logit| {float(np.abs(lo).max()):.2f}, mean-abs {max(means):.2e}")
    assert max(means) <= BF16_FULL_MEAN_TOL, means
    assert max(errs) <= BF16_FULL_TOL, errs
    g.close()
    o.close()


def test_bloom560m_full_fp32_128_greedy_ids_identical():
    m = config.get("bloom-560m")
    P, N = 16, 128
    g = Stage(m.hidden, m.n_head, m.n_layer, m.vocab, 0, m.n_layer, dtype="fp32", max_batch=1,
              max_ctx=P + N, max_tokens=P, seed=0)
    o = OracleStage(m.hidden, m.n_head, m.n_layer, m.vocab, 0, m.n_layer, bf16=False, max_batch=1,
                    max_ctx=P + N, seed=0)
    ids = prompt_ids(1234, 1, P, m.vocab)
    tg = [g.forward_host(ids, 1, P)]
    to = [o.forward(ids, 1, P)]
    for i in range(N - 1):  # free-running: each side feeds back its own token
        tg.append(g.forward_host(tg[-1].reshape(1, 1), 1, 1, past_len=P + i))
        to.append(o.forward(to[-1].reshape(1, 1), 1, 1, past_len=P + i))
    got, want = np.concatenate(tg), np.concatenate(to)
    assert got.shape == (N,)
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:8]
    g.close()
    o.close()


# bf16 device against the NON-emulating fp32 reference at configs[1] (bloom-1b1, 24 layers, V = 250880, 512-token
# prompt), fixed from the committed multi-seed study before this test asserted them (tools/fp32ref_study.py,
# profiles/r06_fp32ref_study.txt: 4 weight/prompt seeds, teacher-forced logits per step over the prefill and 32 decode
# steps: max-abs 0.029-0.032, mean-abs 0.0048-0.0050; 128 free-running greedy ids identical on every seed, the
# reference's smallest top-2 margin 2.0):
FP32REF_MAX_TOL = 4.5e-2     # logits max-abs, any teacher-forced step (1.4x the study's largest)
FP32REF_MEAN_TOL = 7.5e-3    # logits mean-abs, any teacher-forced step (1.5x)


def bf16_vs_fp32_reference(seed=0, prompt_seed=1234, P=512, STEPS=128, TF=32):
    """bloom-1b1 full depth: the benchmarked bf16 device path against the fp32 checker with no bf16 emulation
    (fp32 weights, fp32 everywhere -- the reference's arithmetic, inference.cpp:207-215 fp32 ORT):
      * teacher-forced (KV row 0): 1 prefill + TF decode steps fed the fp32 reference's tokens, logits max/mean-abs;
      * free-running (KV row 1): STEPS greedy tokens, each side feeding back its own; the first step where the ids
        differ and the reference's top-2 margin there.
    Returns the record (also written to $BS_PARITY_LOG)."""
    import json
    import os
    import torch
    from test_gpu_parity import record_error
    m = config.get("bloom-1b1")
    g = Stage(m.hidden, m.n_head, m.n_layer, m.vocab, 0, m.n_layer, dtype="bf16", max_batch=2,
              max_ctx=P + STEPS + 1, max_tokens=P, seed=seed)
    o = OracleStage(m.hidden, m.n_head, m.n_layer, m.vocab, 0, m.n_layer, bf16=False, max_batch=2,
                    max_ctx=P + STEPS + 1, seed=seed)
    ids = prompt_ids(prompt_seed, 1, P, m.vocab)
    dev = torch.device("cuda", 0)
    cs = torch.cuda.Stream()
    tf_max, tf_mean = [], []
    kind = "logits bf16 vs fp32 reference"
    with torch.cuda.stream(cs):
        tin = torch.from_numpy(ids).to(dev)
        tok = torch.empty(1, dtype=torch.int32, device=dev)
        lg = torch.empty((1, m.vocab), dtype=torch.float32, device=dev)
        # teacher-forced (KV row 0)
        g.forward(tin, tok, 1, P, slot=0, past_len=0, logits=lg, stream=cs.cuda_stream)
        to, lo = o.forward(ids, 1, P, slot=0, want_logits=True)
        torch.cuda.synchronize()
        first_dev, first_ref = int(tok.cpu()[0]), int(to[0])
        tf_max.append(record_error(f"1b1 full s{seed} prefill [bf16 device vs fp32 reference]", lg.cpu().numpy(), lo,
                                   FP32REF_MAX_TOL, kind))
        tf_mean.append(float(np.abs(lg.cpu().numpy() - lo).mean()))
        for step in range(TF):
            tok.copy_(torch.from_numpy(to))
            g.forward(tok, tok, 1, 1, slot=0, past_len=P + step, logits=lg, stream=cs.cuda_stream)
            to, lo = o.forward(to.reshape(1, 1), 1, 1, slot=0, past_len=P + step, want_logits=True)
            torch.cuda.synchronize()
            tf_max.append(record_error(f"1b1 full s{seed} decode step {step} [bf16 device vs fp32 reference]",
                                       lg.cpu().numpy(), lo, FP32REF_MAX_TOL, kind))
            tf_mean.append(float(np.abs(lg.cpu().numpy() - lo).mean()))
        # free-running (KV row 1): both sides greedy on their own tokens
        g.forward(tin, tok, 1, P, slot=1, past_len=0, stream=cs.cuda_stream)
        torch.cuda.synchronize()
        dtoks = [int(tok.cpu()[0])]
        rt, rl = o.forward(ids, 1, P, slot=1, want_logits=True)
        rtoks, margins = [int(rt[0])], [float(np.diff(np.sort(rl[0])[-2:])[0])]
        for step in range(STEPS - 1):
            g.forward(tok, tok, 1, 1, slot=1, past_len=P + step, stream=cs.cuda_stream)
            rt, rl = o.forward(np.asarray([[rtoks[-1]]], np.int32), 1, 1, slot=1, past_len=P + step, want_logits=True)
            torch.cuda.synchronize()
            dtoks.append(int(tok.cpu()[0]))
            rtoks.append(int(rt[0]))
            margins.append(float(np.diff(np.sort(rl[0])[-2:])[0]))
    g.close()
    o.close()
    diff = [i for i in range(STEPS) if dtoks[i] != rtoks[i]]
    first = diff[0] if diff else None
    rec = {"test": "bf16_vs_fp32_reference", "kind": "free-running bf16 vs fp32 reference", "seed": seed,
           "prompt_seed": prompt_seed, "steps": STEPS, "identical_prefix": first if first is not None else STEPS,
           "first_divergence_step": first,
           "ref_top2_margin_at_divergence": margins[first] if first is not None else None,
           "ref_top2_margin_min_before": min(margins[:first]) if first else (min(margins) if first is None else None),
           "teacher_forced_logits_max_abs": {"max": max(tf_max), "median": float(np.median(tf_max))},
           "teacher_forced_logits_mean_abs_max": max(tf_mean), "first_token_device": first_dev,
           "first_token_ref": first_ref, "tf_max": tf_max, "tf_mean": tf_mean}
    print(json.dumps({k: v for k, v in rec.items() if k not in ("tf_max", "tf_mean")}))
    path = os.environ.get("BS_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({k: v for k, v in rec.items() if k not in ("tf_max", "tf_mean")}) + "\n")
    return rec


def test_bloom1b1_full_bf16_against_fp32_reference():
    """north_star's own comparison at configs[1]: the bf16 device against the fp32 reference (not the
    bf16-emulating checker the bounds above use).  Asserted: the 128 free-running greedy ids are IDENTICAL to the
    fp32 reference's (north_star: "identical greedy token IDs over a fixed 128-token decode"), and every
    teacher-forced step's logits are within FP32REF_MAX_TOL max-abs / FP32REF_MEAN_TOL mean-abs (constants fixed
    from the multi-seed study before the assertion was added)."""
    rec = bf16_vs_fp32_reference(seed=0, prompt_seed=1234)
    assert rec["first_divergence_step"] is None, rec
    assert max(rec["tf_max"]) <= FP32REF_MAX_TOL, rec["tf_max"]
    assert max(rec["tf_mean"]) <= FP32REF_MEAN_TOL, rec["tf_mean"]


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_bloom560m_full_depth_classification_two_stages(dtype):
    """The classification task at a real configuration: bloom-560m, all 24 layers, split as the server would place it
    on two devices (header [0, 12) -> classifier tail [12, 24), n_labels = 2: run_inference_master_residual ->
    run_inference_worker_residual_last_classification, inference.cpp:220-270), 3 samples x 24 tokens.  Pooled logits
    against the checker in the same mode (fp32: relative 1e-3; bf16: the flat 2e-2) and the class ids equal unless the
    checker's own margin is inside that bound."""
    from test_gpu_parity import check_logits
    m = config.get("bloom-560m")
    B, P, half = 3, 24, m.n_layer // 2
    tw = dtype == "bf16"
    head = Stage(m.hidden, m.n_head, m.n_layer, m.vocab, 0, half, dtype=dtype, max_batch=B, max_ctx=P,
                 max_tokens=B * P, seed=7, is_last=False)
    tail = Stage(m.hidden, m.n_head, m.n_layer, m.vocab, half, m.n_layer, dtype=dtype, max_batch=B, max_ctx=P,
                 max_tokens=B * P, seed=7, n_labels=2)
    o = OracleStage(m.hidden, m.n_head, m.n_layer, m.vocab, 0, m.n_layer, bf16=tw, max_batch=B, max_ctx=P, seed=7,
                    n_labels=2)
    ids = prompt_ids(4321, B, P, m.vocab)
    hid = head.forward_host(ids, B, P)
    cg, lg = tail.forward_host(hid, B, P, want_logits=True)
    co, lo = o.forward(ids, B, P, want_logits=True)
    assert lg.shape == (B, 2)
    check_logits(lg, lo, dtype, f"bloom-560m classifier {dtype}")
    assert_ids_match(cg, co, lo, f"bloom-560m classifier {dtype}",
                     tol=2e-2 if tw else 1e-3 * float(np.abs(lo).max()))
    for s in (head, tail, o):
        s.close()
