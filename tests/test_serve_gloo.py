"""The server/client run (serve.py) on CPU: num_sample samples in waves of
core_pool_size micro-batches through 1 or 2 gloo ranks, each sample's max_length greedy ids equal
to the single-stage oracle decoding that sample alone.  Stage math = the CPU checker (as in
test_pipeline_gloo.py)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_inference_demo_amd.serve import RunConfig, run_rank, synthetic_prompts
from oracle.oracle import OracleStage
from test_pipeline_gloo import MODEL, SEED, OracleExecutor, _free_port

CFG = RunConfig(model=MODEL, num_sample=5, max_length=6, core_pool_size=2, prompt_len=7, dtype="fp32")


def _reference(prompts, max_length):
    out = []
    for p in prompts:
        st = OracleStage(MODEL.hidden, MODEL.n_head, MODEL.n_layer, MODEL.vocab, 0, MODEL.n_layer, max_batch=1,
                         max_ctx=len(p) + max_length + 1, seed=SEED)
        tok = st.forward(np.array(p, np.int32).reshape(1, -1), 1, len(p))
        ids = [int(tok[0])]
        for i in range(max_length - 1):
            tok = st.forward(tok.reshape(1, 1), 1, 1, past_len=len(p) + i)
            ids.append(int(tok[0]))
        out.append(ids)
    return out


def _classes(prompts, n_labels):
    """Each sample alone through one whole-model classifier stage (the checker)."""
    out = []
    for p in prompts:
        st = OracleStage(MODEL.hidden, MODEL.n_head, MODEL.n_layer, MODEL.vocab, 0, MODEL.n_layer, max_batch=1,
                         max_ctx=len(p) + 1, seed=SEED, n_labels=n_labels)
        out.append(int(st.forward(np.array(p, np.int32).reshape(1, -1), 1, len(p))[0]))
    return out


CLS_PROMPTS = [np.random.default_rng(11).integers(0, MODEL.vocab, size=n).tolist() for n in (4, 7, 4, 4, 2, 7, 4)]


def _worker(rank, world, port, q, head_split, cls=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if cls:
            cfg = RunConfig(**{**CFG.__dict__, "num_sample": len(CLS_PROMPTS), "max_length": 0, "n_labels": 3,
                               "core_pool_size": 3})
            res = run_rank(cfg, rank, world, torch.device("cpu"), prompts=CLS_PROMPTS if rank == 0 else None,
                           executor_factory=OracleExecutor)
        else:
            cfg = RunConfig(**{**CFG.__dict__, "head_split": head_split})
            res = run_rank(cfg, rank, world, torch.device("cpu"), executor_factory=OracleExecutor)
        if rank == 0:
            q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,head_split", [(2, False), (2, True), (3, True), (3, False)])
def test_serve_two_ranks_matches_per_sample_oracle(world, head_split):
    """Admission prefill passes (Pipeline.prefill_row) interleaved with the decode rounds: the first token
    returns on its own communicator -- from the last rank, or from the head ring's closer (rank 1 at world 3,
    rank 0 itself at world 2)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, head_split)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res["num_sample"] == 5 and res["stages"] == world and len(res["samples"]) == 5
    assert res["samples"] == _reference(synthetic_prompts(CFG, MODEL.vocab), CFG.max_length)


def test_serve_single_rank_given_prompts():
    rng = np.random.default_rng(5)
    prompts = rng.integers(0, MODEL.vocab, size=(3, 4)).tolist()
    cfg = RunConfig(**{**CFG.__dict__, "num_sample": 3, "core_pool_size": 2, "max_length": 4})
    res = run_rank(cfg, 0, 1, torch.device("cpu"), prompts=prompts, executor_factory=OracleExecutor)
    assert res["prompt_lens"] == [4, 4, 4] and res["samples"] == _reference(prompts, 4)


def test_serve_ragged_prompts_continuous_admission():
    """Prompts of 1..9 tokens, 3 rows in flight: a row takes the next sample the round its sample
    finishes, rows sit at different positions; every sample's ids equal the per-sample checker."""
    rng = np.random.default_rng(8)
    prompts = [rng.integers(0, MODEL.vocab, size=n).tolist() for n in (5, 1, 9, 3, 2, 7)]
    cfg = RunConfig(**{**CFG.__dict__, "num_sample": 6, "core_pool_size": 3, "max_length": 5})
    res = run_rank(cfg, 0, 1, torch.device("cpu"), prompts=prompts, executor_factory=OracleExecutor)
    assert res["samples"] == _reference(prompts, 5)
    # the admission schedule: with the prompt as one prefill pass every sample holds its row max_length - 1
    # decode rounds, so the fourth sample takes row 0 at round 4; fed a token a round (prefill=False) it
    # takes the row the 1-token prompt frees, at round 5
    from distributed_inference_demo_amd.serve import admission_schedule
    sched, T = admission_schedule([5, 1, 9, 3, 2, 7], 5, 3)
    assert sched[:4] == [(0, 0), (1, 0), (2, 0), (0, 4)] and T == res["rounds"]
    sched, T = admission_schedule([5, 1, 9, 3, 2, 7], 5, 3, prefill=False)
    assert sched[:4] == [(0, 0), (1, 0), (2, 0), (1, 5)]
    cfg1 = RunConfig(**{**cfg.__dict__, "prefill": False})
    res1 = run_rank(cfg1, 0, 1, torch.device("cpu"), prompts=prompts, executor_factory=OracleExecutor)
    assert res1["samples"] == res["samples"] and res1["rounds"] == T


def test_serve_max_length_one_is_prefill_only():
    """max_length = 1: every sample is its prefill pass alone (no decode round); rows are reused within the
    same round."""
    rng = np.random.default_rng(9)
    prompts = [rng.integers(0, MODEL.vocab, size=n).tolist() for n in (3, 6, 2)]
    cfg = RunConfig(**{**CFG.__dict__, "num_sample": 3, "core_pool_size": 2, "max_length": 1})
    res = run_rank(cfg, 0, 1, torch.device("cpu"), prompts=prompts, executor_factory=OracleExecutor)
    assert res["rounds"] == 0 and res["samples"] == _reference(prompts, 1)


def test_serve_classification_single_rank():
    """max_length = 0 (Communication.java:591-603): one pass per sample through a classifier tail, samples of
    equal prompt length batched 3 rows a pass (lengths 4, 7, 4, 4, 2, 7, 4 -> passes of 3 + 1 + 2 + 1 rows);
    every class id equals the checker run on that sample alone."""
    cfg = RunConfig(**{**CFG.__dict__, "num_sample": len(CLS_PROMPTS), "max_length": 0, "n_labels": 3,
                       "core_pool_size": 3})
    res = run_rank(cfg, 0, 1, torch.device("cpu"), prompts=CLS_PROMPTS, executor_factory=OracleExecutor)
    assert res["task"] == "classification" and res["passes"] == 4
    assert res["samples"] == _classes(CLS_PROMPTS, 3)
    from distributed_inference_demo_amd.serve import classify_batches
    assert classify_batches([4, 7, 4, 4, 2, 7, 4], 3) == [(4, [0, 2, 3]), (4, [6]), (7, [1, 5]), (2, [4])]
    with pytest.raises(ValueError):
        run_rank(RunConfig(**{**cfg.__dict__, "max_length": -1}), 0, 1, torch.device("cpu"), prompts=CLS_PROMPTS,
                 executor_factory=OracleExecutor)


def test_serve_classification_two_ranks():
    """The same task over 2 gloo ranks: layers split, the classifier on rank 1, class ids back to rank 0."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, False, True)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res["stages"] == 2 and res["samples"] == _classes(CLS_PROMPTS, 3)


def test_serve_rejects_empty_prompts():
    with pytest.raises(ValueError):
        run_rank(RunConfig(**{**CFG.__dict__, "num_sample": 2}), 0, 1, torch.device("cpu"), prompts=[[1, 2], []],
                 executor_factory=OracleExecutor)
