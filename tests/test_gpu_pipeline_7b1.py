"""The pipeline schedules of BASELINE.json configs[3] and configs[4] with the PRODUCT stages (libbloomstage
HIP kernels), all ranks on cuda:0 as gloo processes with host-staged hops (RCCL refuses two ranks on one
device; the driver's 8-GPU node runs the same schedule over RCCL).  bloom-7b1 dims (h = 4096, 32 heads,
30 layers), vocabulary reduced to 4096 so the CPU checker stays affordable.

  configs[3] shape: 8 stages split 4,4,4,4,4,4,3,3 by round_robin_module_arrangement (server.py:893-903),
      16 one-row micro-batches in flight, the vocabulary-parallel lm_head as an 8-slice ring; fp32 greedy
      ids identical to the single-stage fp32 checker.
  configs[4] shape: B = 32 decode through a 2-stage split [0,15) [15,30), 4 micro-batches of 8 rows, a
      500-token prefill and 16 decode steps (context 516): bf16 greedy ids identical to ONE product stage
      holding all 30 layers fed the same micro-batches (the hop is the fp32 residual stream, so the split
      changes no arithmetic), and the two stages' K/V caches bitwise equal to that stage's.  The kernels
      themselves are checked against the checker at this width in tests/test_gpu_7b1_width.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_inference_demo_amd import config
from distributed_inference_demo_amd.pipeline import build_rank, generate
from distributed_inference_demo_amd.placement import stage_ranges

pytestmark = pytest.mark.gpu
M7 = config.BloomDims("bloom-7b1-v4096", 4096, 30, 32, vocab=4096)


class HipHostExecutor:
    """A product Stage on cuda:0 behind the pipeline's host (gloo) buffers."""

    def __init__(self, model, dtype, seed, lb, le, first, last, max_batch, max_ctx, max_tokens, hslice=None):
        from distributed_inference_demo_amd.stage import Stage
        self.dev = torch.device("cuda", 0)
        self.st = Stage(model.hidden, model.n_head, model.n_layer, model.vocab, lb, le, dtype=dtype, device=0,
                        max_batch=max_batch, max_ctx=max_ctx, max_tokens=max_tokens, seed=seed, is_first=first,
                        is_last=last, head_slice=hslice)

    def forward(self, inp, out, batch, seq, slot, past_len):
        y = self.st.forward_host(inp.numpy(), batch, seq, slot=slot, past_len=past_len)
        out.copy_(torch.from_numpy(np.ascontiguousarray(y).reshape(-1)[: out.numel()]).view(out.shape))

    def head_norm(self, hidden, batch, seq, xn):
        hd = hidden[: batch * seq * self.st.hidden].to(self.dev)
        xd = torch.empty(xn.shape, dtype=xn.dtype, device=self.dev)
        self.st.head_norm(hd, batch, seq, xd)
        torch.cuda.synchronize()
        xn.copy_(xd.cpu())

    def head_slice(self, xn, batch, keys_in, keys_out, tokens):
        xd = xn.to(self.dev)
        kin = None if keys_in is None else keys_in.to(self.dev)
        kout = None if keys_out is None else torch.empty_like(keys_out, device=self.dev)
        tok = None if tokens is None else torch.empty_like(tokens, device=self.dev)
        self.st.head_slice(xd, batch, kin, kout, tok)
        torch.cuda.synchronize()
        if keys_out is not None:
            keys_out.copy_(kout.cpu())
        if tokens is not None:
            tokens.copy_(tok.cpu())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, kw):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      OMP_NUM_THREADS="2")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m, dtype, seed, P, steps, mb = kw["model"], kw["dtype"], kw["seed"], kw["P"], kw["steps"], kw["mb"]

        def factory(lb, le, first, last, max_batch, max_ctx, hslice):
            return HipHostExecutor(m, dtype, seed, lb, le, first, last, max_batch, max_ctx, mb * P, hslice)
        pipe, rng = build_rank(m, rank, world, torch.device("cpu"), mb_rows=mb, n_mb=kw.get("n_mb"),
                               max_ctx=P + steps + 2, max_seq=P, executor_factory=factory,
                               head_split=kw["head_split"], dtype=dtype)
        from distributed_inference_demo_amd.stage import prompt_ids
        prompt = torch.from_numpy(prompt_ids(1234, mb * pipe.n_mb, P, m.vocab)) if rank == 0 else None
        toks = generate(pipe, prompt, steps, P)
        kv = None
        if kw.get("kv_probe"):  # (local layer 0 and last, rows 0 and B-1) K/V at positions [P-4, P+steps)
            st = pipe.ex.st
            B, L = mb * pipe.n_mb, rng[1] - rng[0]
            kv = {(rng[0] + l, r): st.read_kv(l, r, P - 4, steps + 4) for l in (0, L - 1) for r in (0, B - 1)}
        q.put((rank, rng, pipe.n_mb, None if toks is None else toks.numpy(), kv))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run(world, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, kw)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, rng, n_mb, toks, kv = q.get(timeout=300)
        res[r] = (rng, n_mb, toks, kv)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_7b1_eight_stage_split_16_micro_batches_fp32_greedy_identical():
    """configs[3]'s schedule on product stages: 8 stages (4,4,4,4,4,4,3,3), 16 one-row micro-batches, the
    8-slice vocabulary ring; fp32 greedy ids == the single-stage fp32 checker's."""
    from oracle.oracle import OracleStage, prompt_ids
    P, STEPS, SEED = 4, 3, 9
    res = _run(8, model=M7, dtype="fp32", seed=SEED, P=P, steps=STEPS, mb=1, head_split=True)
    assert [res[r][0][1] - res[r][0][0] for r in range(8)] == [4, 4, 4, 4, 4, 4, 3, 3]
    assert all(res[r][1] == 16 for r in range(8))
    got = res[0][2]
    B = got.shape[0]
    assert B == 16 and got.shape[1] == STEPS + 1
    ref = OracleStage(M7.hidden, M7.n_head, M7.n_layer, M7.vocab, 0, M7.n_layer, max_batch=B, max_ctx=P + STEPS + 2,
                      seed=SEED)
    tok = ref.forward(prompt_ids(1234, B, P, M7.vocab), B, P)
    want = [tok]
    for i in range(STEPS):
        tok = ref.forward(tok.reshape(B, 1), B, 1, past_len=P + i)
        want.append(tok)
    assert np.array_equal(got, np.stack(want, 1))


def test_7b1_batch32_two_stage_decode_to_ctx_516_bf16_equals_one_stage():
    """configs[4]'s schedule on product stages: B = 32 as 4 micro-batches of 8 through [0,15) [15,30), a
    500-token prefill and 16 decode steps; greedy ids and the K/V rows equal one 30-layer product stage
    fed the same micro-batches, bit for bit."""
    from distributed_inference_demo_amd.stage import Stage, prompt_ids
    P, STEPS, SEED, MB, NMB = 500, 16, 4, 8, 4
    assert stage_ranges(2, 30) == [(0, 15), (15, 30)]
    res = _run(2, model=M7, dtype="bf16", seed=SEED, P=P, steps=STEPS, mb=MB, n_mb=NMB, head_split=False,
               kv_probe=True)
    got = res[0][2]
    B = MB * NMB
    assert got.shape == (B, STEPS + 1)
    one = Stage(M7.hidden, M7.n_head, M7.n_layer, M7.vocab, 0, M7.n_layer, dtype="bf16", device=0, max_batch=B,
                max_ctx=P + STEPS + 2, max_tokens=MB * P, seed=SEED)
    ids = prompt_ids(1234, B, P, M7.vocab)
    want = np.empty((B, STEPS + 1), np.int32)
    tok = [one.forward_host(ids[j * MB:(j + 1) * MB], MB, P, slot=j * MB, past_len=0) for j in range(NMB)]
    want[:, 0] = np.concatenate(tok)
    for i in range(STEPS):
        tok = [one.forward_host(want[j * MB:(j + 1) * MB, i].reshape(MB, 1), MB, 1, slot=j * MB, past_len=P + i)
               for j in range(NMB)]
        want[:, i + 1] = np.concatenate(tok)
    assert np.array_equal(got, want), f"{int((got != want).sum())} of {got.size} ids differ"
    for r in range(2):
        for (layer, row), kv in res[r][3].items():
            assert np.array_equal(kv, one.read_kv(layer, row, P - 4, STEPS + 4)), (r, layer, row)
    one.close()


SERVE_M = config.BloomDims("serve-small", 256, 4, 4, vocab=1024)


def _serve_worker(rank, world, port, q, kw):
    from distributed_inference_demo_amd.serve import RunConfig, run_rank
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      OMP_NUM_THREADS="2")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        for prefill in (True, False):
            cfg = RunConfig(model=SERVE_M, num_sample=5, max_length=6, core_pool_size=2, prompt_len=7, dtype="fp32",
                            seed=kw["seed"], head_split=True, prefill=prefill)

            def factory(lb, le, first, last, max_batch, max_ctx, hslice):
                return HipHostExecutor(SERVE_M, "fp32", kw["seed"], lb, le, first, last, max_batch, max_ctx, 16, hslice)
            res = run_rank(cfg, rank, world, torch.device("cpu"), executor_factory=factory)
            out[prefill] = None if res is None else res["samples"]
            dist.barrier()
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_serve_head_split_ring_on_product_stages(world):
    """serve.run_rank with the vocabulary-parallel head ring (head_split) at world 2 and 3, the PRODUCT stages on cuda:0
    as gloo ranks: the admission prefill passes (Pipeline.prefill_row: one pass per admitted sample, its first token back
    from the ring's closer on its own communicator) give the same samples as the token-a-round feed (prefill=False), and
    both equal the fp32 checker decoding each sample alone.  (The ring's hstream / RCCL branches run only on an RCCL
    group: the driver's multi-GPU run.)"""
    from distributed_inference_demo_amd.serve import RunConfig, synthetic_prompts
    from oracle.oracle import OracleStage
    seed = 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_serve_worker, args=(r, world, port, q, {"seed": seed})) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[True] == out[False]
    cfg = RunConfig(model=SERVE_M, num_sample=5, max_length=6, core_pool_size=2, prompt_len=7, dtype="fp32", seed=seed)
    for sid, p in enumerate(synthetic_prompts(cfg, SERVE_M.vocab)):
        st = OracleStage(SERVE_M.hidden, SERVE_M.n_head, SERVE_M.n_layer, SERVE_M.vocab, 0, SERVE_M.n_layer, max_batch=1,
                         max_ctx=len(p) + 8, seed=seed)
        tok = st.forward(np.array(p, np.int32).reshape(1, -1), 1, len(p))
        ids = [int(tok[0])]
        for i in range(5):
            tok = st.forward(tok.reshape(1, 1), 1, 1, past_len=len(p) + i)
            ids.append(int(tok[0]))
        assert out[True][sid] == ids, (sid, out[True][sid], ids)
