"""GPU parity of the sequence-classification tail (BS_FLAG_CLASSIFIER), through the C-ABI.

The reference's classification task (task_type "classification", Communication.java:532, :596) runs the tail
sub-model through run_inference_with_binary_classification (inference.cpp:220-270, behind
runInferenceWorkerResidualLastClassification, native-lib.cpp:1305-1366) and reduces its logits with
binary_classify (inference.cpp:57-69: the first index of the largest).  The head here is HF
BloomForSequenceClassification's (ln_f on the row's last token, score without bias); the checker's classifier
(or_set_classifier) is pinned to HF by tests/test_oracle_golden.py::test_classifier_tail_matches_hf.
"""
import numpy as np
import pytest

from distributed_inference_demo_amd.stage import (BloomStageError, Stage, binary_classify, create_session,
                                                  deserialize_int, deserialize_tensors, run_inference_master_residual,
                                                  run_inference_worker_residual_last_classification,
                                                  serialize_tensors)
from distributed_inference_demo_amd.config import BloomDims
from oracle import gen_np
from oracle.oracle import OracleStage

from test_gpu_parity import G, assert_ids_match, canonical_weights, check_logits

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n_labels", [2, 3])
def test_classifier_fp32_matches_hf_golden(n_labels):
    """Whole model as one classifier stage (fp32) against BloomForSequenceClassification's pooled logits."""
    g = np.load(f"{G}/tiny_classify.npz")
    h, nh, L, V, seed, B, S = (int(v) for v in g["config"])
    st = Stage(h, nh, L, V, 0, L, dtype="fp32", max_batch=B, max_ctx=S, seed=seed, n_labels=n_labels)
    cls, lg = st.forward_host(g["ids"], B, S, want_logits=True)
    assert lg.shape == (B, n_labels)
    check_logits(lg, g[f"logits{n_labels}"], "fp32", f"classifier {n_labels} labels vs HF")
    assert np.array_equal(cls, g[f"class{n_labels}"])


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_classifier_tail_after_split_matches_checker(dtype):
    """Header [0, 2) + classifier tail [2, 4) at h = 256, 3 rows x 24 tokens, then 6 decode-shaped steps (the tail
    fed the header's hidden state per step)."""
    h, nh, L, V, B, S, nl = 256, 4, 4, 1024, 3, 24, 2
    tw = dtype == "bf16"
    g0 = Stage(h, nh, L, V, 0, 2, dtype=dtype, max_batch=B, max_ctx=40, seed=21)
    o0 = OracleStage(h, nh, L, V, 0, 2, bf16=tw, max_batch=B, max_ctx=40, seed=21)
    g1 = Stage(h, nh, L, V, 2, L, dtype=dtype, max_batch=B, max_ctx=40, seed=21, n_labels=nl)
    o1 = OracleStage(h, nh, L, V, 2, L, bf16=tw, max_batch=B, max_ctx=40, seed=21, n_labels=nl)
    ids = gen_np.prompt_ids(31, B, S, V).astype(np.int32)
    g0.forward_host(ids, B, S)
    hid = o0.forward(ids, B, S)
    past = S
    for step in range(7):
        n = hid.shape[1]
        cg, lg = g1.forward_host(hid, B, n, past_len=past - n, want_logits=True)
        co, lo = o1.forward(hid, B, n, past_len=past - n, want_logits=True)
        check_logits(lg, lo, dtype, f"classifier tail step {step}")
        assert_ids_match(cg, co, lo, f"classifier tail step {step}")
        nxt = gen_np.prompt_ids(40 + step, B, 1, V).astype(np.int32)
        g0.forward_host(nxt, B, 1, past_len=past)
        hid = o0.forward(nxt, B, 1, past_len=past)
        past += 1


def test_classifier_jni_entry_points():
    """runInferenceMasterResidual -> wire bytes -> runInferenceWorkerResidualLastClassification (4 bytes of the
    class); binaryClassify on the tail's serialized logits gives the same class."""
    m = BloomDims("tiny", 256, 2, 4, 1024)
    head = create_session(m, 0, 1, dtype="bf16", max_ctx=32, seed=5)
    tail = create_session(m, 1, 2, dtype="bf16", max_ctx=32, seed=5, n_labels=2)
    ref = OracleStage(256, 4, 2, 1024, 0, 2, bf16=True, max_ctx=32, seed=5, n_labels=2)
    for i, n in enumerate((7, 19, 1)):
        head.reset()
        tail.reset()
        ids = gen_np.prompt_ids(60 + i, 1, n, 1024).astype(np.int32)
        seq, res = run_inference_master_residual(head, ids)
        out = run_inference_worker_residual_last_classification(tail, seq, res)
        assert len(out) == 4
        co, lo = ref.forward(ids, 1, n, want_logits=True)
        assert_ids_match([deserialize_int(out)], co, lo, f"prompt {n}")
        tail.reset()
        _, lg = tail.forward_host(deserialize_tensors(seq)[0], 1, n, want_logits=True)
        check_logits(lg, lo, "bf16", f"prompt {n} logits")
        assert binary_classify(serialize_tensors([lg])) == deserialize_int(out)
    with pytest.raises(BloomStageError):
        run_inference_worker_residual_last_classification(head, seq, res)


def test_classifier_graph_replay_device_buffers():
    """Device I/O on a classifier tail: S = 1 steps replay a captured hipGraph; the class kernel advances the
    device copy of each row's position (no set_past launch between replays).  Checked step by step."""
    import torch
    h, nh, L, V, B, nl = 512, 8, 2, 2048, 4, 5
    g = Stage(h, nh, L, V, 1, L, dtype="bf16", max_batch=B, max_ctx=64, seed=13, n_labels=nl)
    o = OracleStage(h, nh, L, V, 1, L, bf16=True, max_batch=B, max_ctx=64, seed=13, n_labels=nl)
    rng = np.random.default_rng(3)
    dev = torch.device("cuda", 0)
    cs = torch.cuda.Stream()
    x = rng.standard_normal((B, 9, h)).astype(np.float32)
    g.forward_host(x, B, 9)
    o.forward(x, B, 9)
    with torch.cuda.stream(cs):
        hin = torch.empty((B, 1, h), dtype=torch.float32, device=dev)
        cls = torch.empty(B, dtype=torch.int32, device=dev)
        lg = torch.empty((B, nl), dtype=torch.float32, device=dev)
        for step in range(12):
            x = rng.standard_normal((B, 1, h)).astype(np.float32)
            hin.copy_(torch.from_numpy(x))
            g.forward(hin, cls, B, 1, logits=lg, stream=cs.cuda_stream)
            torch.cuda.synchronize()
            co, lo = o.forward(x, B, 1, past_len=9 + step, want_logits=True)
            check_logits(lg.cpu().numpy(), lo, "bf16", f"graph step {step}")
            assert_ids_match(cls.cpu().numpy(), co, lo, f"graph step {step}")


def test_classifier_first_maximum_on_exact_ties():
    """binary_classify keeps the first maximum (inference.cpp:62-66, strict >): a layer-free classifier whose
    score rows 1 and 2 are the same row ties them bit for bit; row 0 is their negation."""
    h, nh, V, nl = 64, 4, 512, 3
    w = canonical_weights(8, h, 2, V, 0, 0, first=True, last=True)
    v = gen_np.tensor(8, -1, gen_np.GT_SCORE, (h,))
    w = np.concatenate([w, -v, v, v]).astype(np.float32)
    B = 32
    st = Stage(h, nh, 2, V, 0, 0, dtype="fp32", max_batch=B, max_ctx=4, host_weights=w, is_first=True,
               is_last=True, n_labels=nl)
    ids = np.arange(B, dtype=np.int32).reshape(B, 1) * 13
    cls, lg = st.forward_host(ids, B, 1, want_logits=True)
    assert np.array_equal(lg[:, 1].view(np.uint32), lg[:, 2].view(np.uint32))
    want = np.where(lg[:, 1] > lg[:, 0], 1, 0)
    assert np.array_equal(cls, want) and 1 in want, (cls, lg)


def test_classifier_rejects_generation_only_calls():
    st = Stage(64, 4, 2, 512, 1, 2, dtype="bf16", max_ctx=8, seed=1, n_labels=2)
    with pytest.raises(BloomStageError, match="sampling"):
        st.set_sampling(4)
    with pytest.raises(BloomStageError):
        Stage(64, 4, 2, 512, 0, 1, dtype="bf16", max_ctx=8, seed=1, is_last=False, n_labels=2)


def test_classifier_tail_with_int8_block_weights():
    """BS_FLAG_CLASSIFIER with BS_FLAG_INT8_WEIGHTS (the reference's bloom*-int8 modules, server.py:796-799): the block
    matrices run the int8 GEMVs / GEMMs, the score head stays bf16; against the checker's int8 restatement with the same
    classifier head (prefill then decode-shaped steps)."""
    h, nh, L, V, B, S, nl = 256, 4, 2, 1024, 2, 12, 3
    g = Stage(h, nh, L, V, 1, L, dtype="bf16", max_batch=B, max_ctx=32, seed=17, n_labels=nl, int8_weights=True)
    o = OracleStage(h, nh, L, V, 1, L, bf16=True, max_batch=B, max_ctx=32, seed=17, n_labels=nl, int8=True)
    rng = np.random.default_rng(5)
    x = rng.standard_normal((B, S, h)).astype(np.float32)
    cg, lg = g.forward_host(x, B, S, want_logits=True)
    co, lo = o.forward(x, B, S, want_logits=True)
    check_logits(lg, lo, "bf16", "int8 classifier prefill")
    assert_ids_match(cg, co, lo, "int8 classifier prefill")
    for step in range(3):
        x1 = rng.standard_normal((B, 1, h)).astype(np.float32)
        cg, lg = g.forward_host(x1, B, 1, past_len=S + step, want_logits=True)
        co, lo = o.forward(x1, B, 1, past_len=S + step, want_logits=True)
        check_logits(lg, lo, "bf16", f"int8 classifier step {step}")
        assert_ids_match(cg, co, lo, f"int8 classifier step {step}")


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_serve_classification_task_on_gpu(dtype):
    """serve.run_rank with max_length = 0 (Communication.java:591-603) on cuda:0 with the product stage: ragged prompts
    batched by length, 3 rows a pass, a 2-label classifier tail; every class id against the checker run on that
    sample alone."""
    import torch
    from distributed_inference_demo_amd.serve import RunConfig, run_rank
    m = BloomDims("tiny-cls", 256, 3, 4, 1024)
    rng = np.random.default_rng(17)
    prompts = [rng.integers(0, m.vocab, size=n).tolist() for n in (9, 3, 9, 9, 17, 3, 9)]
    cfg = RunConfig(model=m, num_sample=len(prompts), max_length=0, core_pool_size=3, n_labels=2, dtype=dtype,
                    seed=23)
    res = run_rank(cfg, 0, 1, torch.device("cuda", 0), prompts=prompts)
    assert res["passes"] == 4 and len(res["samples"]) == len(prompts)
    for i, p in enumerate(prompts):
        o = OracleStage(256, 4, 3, 1024, 0, 3, bf16=dtype == "bf16", max_ctx=len(p) + 1, seed=23, n_labels=2)
        co, lo = o.forward(np.array(p, np.int32).reshape(1, -1), 1, len(p), want_logits=True)
        assert_ids_match([res["samples"][i]], co, lo, f"sample {i}")


def test_pipeline_classify_on_torch_default_stream():
    """Pipeline + StageExecutor driven from torch's default stream (handle 0, which the C-ABI reads as the stage's own
    non-blocking stream): the executor fences a side stream both ways, so the prompt upload, the stage and the class
    read-back stay ordered.  Passes of 9, 1 (a graph-replayed S = 1 step) and 5 tokens, 2 rows each."""
    import torch
    from distributed_inference_demo_amd.pipeline import build_rank, classify
    m = BloomDims("tiny-cls", 256, 3, 4, 1024)
    dev = torch.device("cuda", 0)
    with torch.cuda.stream(torch.cuda.default_stream(dev)):
        pipe, _ = build_rank(m, 0, 1, dev, dtype="bf16", mb_rows=2, max_ctx=10, max_seq=9, seed=29, n_labels=2)
        for i, n in enumerate((9, 1, 5, 9)):
            ids = gen_np.prompt_ids(70 + i, 2, n, 1024).astype(np.int32)
            got = classify(pipe, torch.from_numpy(ids).to(dev), n).cpu().numpy()
            o = OracleStage(256, 4, 3, 1024, 0, 3, bf16=True, max_batch=2, max_ctx=10, seed=29, n_labels=2)
            co, lo = o.forward(ids, 2, n, want_logits=True)
            assert_ids_match(got, co, lo, f"pass {i} ({n} tokens)")
