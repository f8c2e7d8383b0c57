"""Multi-process pipeline protocol on CPU (gloo): N ranks, N micro-batches in flight, hidden
states forwarded rank to rank, tokens returned tail -> head.  Each rank's stage math is the CPU
checker (test infrastructure standing in for the GPU stage, which needs an MI355X); the test
checks the schedule produces exactly the single-stage greedy tokens."""
import functools
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_inference_demo_amd import config
from distributed_inference_demo_amd.pipeline import build_rank, classify, generate
from oracle.oracle import OracleStage, prompt_ids

MODEL = config.BloomDims("tiny", 64, 4, 4, vocab=512)
# 30 layers: round_robin_module_arrangement(8, 30) (server.py:893-903) gives bloom-7b1's 8-stage split
# 4,4,4,4,4,4,3,3 (BASELINE.json configs[3])
MODEL30 = config.BloomDims("tiny30", 64, 30, 4, vocab=512)
SEED, P, STEPS, MB = 3, 6, 10, 2


class OracleExecutor:
    def __init__(self, lb, le, first, last, max_batch, max_ctx, hslice=None, model=MODEL, n_labels=0):
        self.model = model
        self.st = OracleStage(model.hidden, model.n_head, model.n_layer, model.vocab, lb, le, max_batch=max_batch,
                              max_ctx=max_ctx, seed=SEED, is_first=first, is_last=last, n_labels=n_labels)
        self.first, self.last, self.hslice = first, last, hslice
        if hslice is not None:  # layer-free stage owning the tied head for ln_f + the vocab slice
            self.head = OracleStage(model.hidden, model.n_head, model.n_layer, model.vocab, 0, 0, max_batch=max_batch,
                                    max_ctx=max_ctx, seed=SEED, is_first=False, is_last=True)

    def head_norm(self, hidden, batch, seq, xn):
        xn.copy_(torch.from_numpy(self.head.head_norm(hidden.numpy()[: batch * seq * self.model.hidden], batch, seq).reshape(-1)))

    def head_slice(self, xn, batch, keys_in, keys_out, tokens):
        kin = None if keys_in is None else keys_in.numpy().view(np.uint64)
        keys, toks = self.head.head_slice(xn.numpy(), batch, self.hslice[0], self.hslice[1], kin)
        if keys_out is not None:
            keys_out.copy_(torch.from_numpy(keys.view(np.int64)))
        if tokens is not None:
            tokens.copy_(torch.from_numpy(toks))

    def forward(self, inp, out, batch, seq, slot, past_len):
        x = inp.numpy()
        if isinstance(past_len, (list, tuple)):  # rows at their own positions: the checker takes one row a call
            xs = x.reshape(batch, -1)
            y = np.concatenate([np.asarray(self.st.forward(xs[r], 1, seq, slot=slot + r, past_len=past_len[r])).reshape(1, -1)
                                for r in range(batch)])
        else:
            y = self.st.forward(x, batch, seq, slot=slot, past_len=past_len)
        out.copy_(torch.from_numpy(np.ascontiguousarray(y).reshape(-1)[: out.numel()]).view(out.shape))


def _worker(rank, world, port, q, head_split=False, resume=0, model=MODEL, n_labels=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      OMP_NUM_THREADS="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if n_labels:  # classification: two passes of new samples (KV rows reused from position 0)
            pipe, rng = build_rank(model, rank, world, torch.device("cpu"), mb_rows=MB, max_ctx=P, max_seq=P,
                                   executor_factory=functools.partial(OracleExecutor, model=model), dtype="fp32",
                                   n_labels=n_labels)
            q.put(("range", rank, rng, pipe.n_mb))
            out = []
            for seed in (1234, 99):
                prompt = torch.from_numpy(prompt_ids(seed, MB * pipe.n_mb, P, model.vocab)) if rank == 0 else None
                out.append(classify(pipe, prompt, P))
            if rank == 0:
                q.put(("tokens", torch.stack(out).numpy()))
            dist.barrier()
            return
        pipe, rng = build_rank(model, rank, world, torch.device("cpu"), mb_rows=MB, max_ctx=P + STEPS + resume + 2,
                               max_seq=P, executor_factory=functools.partial(OracleExecutor, model=model),
                               head_split=head_split, dtype="fp32")
        q.put(("range", rank, rng, pipe.n_mb))
        prompt = torch.from_numpy(prompt_ids(1234, MB * pipe.n_mb, P, model.vocab)) if rank == 0 else None
        toks = generate(pipe, prompt, STEPS, P)
        if resume:  # rounds after finish() continue from the tokens finish() collected
            rec = [[] for _ in range(pipe.n_mb)] if rank == 0 else None
            for _ in range(resume):
                pipe.step(1, record=rec)
            pipe.finish(record=rec)
            if rank == 0:
                toks = torch.cat([toks, torch.cat([torch.stack(r, 1) for r in rec], 0)], 1)
        if rank == 0:
            q.put(("tokens", toks.numpy()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, head_split, resume, model=MODEL, n_labels=0):
    """Spawn `world` gloo ranks; returns (rank 0's tokens, {rank: (layer range, micro-batches)})."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, head_split, resume, model, n_labels))
             for r in range(world)]
    for p in procs:
        p.start()
    got, ranges = None, {}
    while got is None or len(ranges) < world:
        msg = q.get(timeout=420)
        if msg[0] == "tokens":
            got = msg[1]
        else:
            ranges[msg[1]] = (tuple(msg[2]), msg[3])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got, ranges


def _single_stage(model, B, steps):
    ref = OracleStage(model.hidden, model.n_head, model.n_layer, model.vocab, 0, model.n_layer, max_batch=B,
                      max_ctx=P + steps + 2, seed=SEED)
    tok = ref.forward(prompt_ids(1234, B, P, model.vocab), B, P)
    want = [tok]
    for i in range(steps):
        tok = ref.forward(tok.reshape(B, 1), B, 1, past_len=P + i)
        want.append(tok)
    return np.stack(want, 1)


def test_pipeline_eight_stages_bloom7b1_split():
    """BASELINE.json configs[3]'s shape on 8 gloo ranks: 30 layers split 4,4,4,4,4,4,3,3 by the server's
    round-robin assignment, 16 micro-batches in flight, the vocabulary-parallel head as an 8-slice ring;
    the greedy ids equal one stage's."""
    got, ranges = _run(8, True, 0, MODEL30)
    assert [ranges[r][0][1] - ranges[r][0][0] for r in range(8)] == [4, 4, 4, 4, 4, 4, 3, 3]
    assert all(ranges[r][1] == 16 for r in range(8))
    assert got.shape[0] == MB * 16
    assert np.array_equal(got, _single_stage(MODEL30, got.shape[0], STEPS))


@pytest.mark.parametrize("world,head_split,resume", [(2, False, 0), (3, False, 0), (2, True, 0), (3, True, 0),
                                                     (4, True, 0), (2, False, 3), (3, True, 3)])
def test_pipeline_matches_single_stage(world, head_split, resume):
    got, _ = _run(world, head_split, resume)
    # single stage reference, all rows at once
    B = got.shape[0]
    assert B == MB * world * (2 if head_split else 1)
    ref = OracleStage(MODEL.hidden, MODEL.n_head, MODEL.n_layer, MODEL.vocab, 0, MODEL.n_layer, max_batch=B,
                      max_ctx=P + STEPS + resume + 2, seed=SEED)
    tok = ref.forward(prompt_ids(1234, B, P, MODEL.vocab), B, P)
    want = [tok]
    for i in range(STEPS + resume):
        tok = ref.forward(tok.reshape(B, 1), B, 1, past_len=P + i)
        want.append(tok)
    assert np.array_equal(got, np.stack(want, 1))


@pytest.mark.parametrize("world", [1, 3])
def test_pipeline_classification_matches_single_stage(world):
    """Classification task (max_length == 0, Communication.java:591-603): one pass of new samples through the
    stages, the last a classifier tail; the class ids equal one whole-model classifier stage's, pass after pass."""
    n_labels = 3
    got, _ = _run(world, False, 0, n_labels=n_labels)
    B = got.shape[1]
    for i, seed in enumerate((1234, 99)):
        ref = OracleStage(MODEL.hidden, MODEL.n_head, MODEL.n_layer, MODEL.vocab, 0, MODEL.n_layer, max_batch=B,
                          max_ctx=P, seed=SEED, n_labels=n_labels)
        assert np.array_equal(got[i], ref.forward(prompt_ids(seed, B, P, MODEL.vocab), B, P))
    assert got.min() >= 0 and got.max() < n_labels


def test_build_rank_rejects_unplaceable_splits():
    """More stages than layers (an empty stage), more head slices than 16-column tiles, and an
    int8 model in fp32 are configuration errors, raised before any stage is built."""
    cpu = torch.device("cpu")
    with pytest.raises(ValueError, match="at least one layer"):
        build_rank(MODEL, 0, MODEL.n_layer + 1, cpu, executor_factory=OracleExecutor, dtype="fp32")
    narrow = config.BloomDims("narrow", 64, 8, 4, vocab=64)
    with pytest.raises(ValueError, match="16-column tile"):
        build_rank(narrow, 0, 5, cpu, executor_factory=OracleExecutor, dtype="fp32", head_split=True)
    with pytest.raises(ValueError, match="int8"):
        build_rank(config.get("bloom560m-int8"), 0, 1, cpu, executor_factory=OracleExecutor, dtype="fp32")
    with pytest.raises(ValueError, match="classifier"):
        build_rank(MODEL, 0, 2, cpu, executor_factory=OracleExecutor, dtype="fp32", head_split=True, n_labels=2)


def test_single_rank_pipeline_loops_tokens_back():
    pipe, _ = build_rank(MODEL, 0, 1, torch.device("cpu"), mb_rows=MB, n_mb=2, max_ctx=P + STEPS + 2, max_seq=P,
                         executor_factory=OracleExecutor, dtype="fp32")
    prompt = torch.from_numpy(prompt_ids(1234, 2 * MB, P, MODEL.vocab))
    got = generate(pipe, prompt, 4, P).numpy()
    ref = OracleStage(MODEL.hidden, MODEL.n_head, MODEL.n_layer, MODEL.vocab, 0, MODEL.n_layer, max_batch=2 * MB,
                      max_ctx=P + 8, seed=SEED)
    tok = ref.forward(prompt.numpy(), 2 * MB, P)
    want = [tok]
    for i in range(4):
        tok = ref.forward(tok.reshape(-1, 1), 2 * MB, 1, past_len=P + i)
        want.append(tok)
    assert np.array_equal(got, np.stack(want, 1))
