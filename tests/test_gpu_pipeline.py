"""Multi-stage pipeline with the PRODUCT stages (libbloomstage HIP kernels) on one GPU.

BASELINE.json configs[2]: bloom-3b dims (h = 2560, 32 heads, 30 layers) split into 4 stages by the
server's round-robin assignment, [0,8), [8,16), [16,23), [23,30) (server.py:893-905), driven by
`pipeline.Pipeline` over gloo ranks that all use cuda:0 (the schedule, the hops and the
vocabulary-parallel lm_head ring of Communication.java:682-928's counterpart).  Each rank's stage is
a real `Stage`; the gloo hops carry host copies (RCCL is the multi-GPU transport; this test checks the
stage math and the schedule on the one GPU a test box has).  The vocabulary is reduced to 4096 so the
CPU checker stays fast; every layer is full width.

  fp32: greedy ids identical to the single-stage fp32 checker (north_star's identity criterion).
  bf16: every id is the bf16 checker's argmax on the pipeline's own prefix (teacher-forced),
        except where the checker's top-2 margin is under the 2e-2 tolerance.
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
from oracle.oracle import OracleStage, prompt_ids

pytestmark = pytest.mark.gpu
MODEL = config.BloomDims("bloom-3b-v4096", 2560, 30, 32, vocab=4096)
SEED, P, STEPS, MB, WORLD = 5, 8, 12, 1, 4
BF16_TOL = 2e-2


class HipHostExecutor:
    """Pipeline executor around a product Stage on cuda:0; the pipeline's buffers are host tensors
    (gloo), copied to and from the stage's device buffers around each call."""

    def __init__(self, dtype, lb, le, first, last, max_batch, max_ctx, hslice=None):
        from distributed_inference_demo_amd.stage import Stage
        self.dev = torch.device("cuda", 0)
        self.st = Stage(MODEL.hidden, MODEL.n_head, MODEL.n_layer, MODEL.vocab, lb, le, dtype=dtype, device=0,
                        max_batch=max_batch, max_ctx=max_ctx, max_tokens=max_batch * P, seed=SEED, is_first=first,
                        is_last=last, head_slice=hslice)
        self.first, self.last = first, last

    def forward(self, inp, out, batch, seq, slot, past_len):
        y = self.st.forward_host(inp.numpy(), batch, seq, slot=slot, past_len=past_len)
        out.copy_(torch.from_numpy(np.ascontiguousarray(y).reshape(-1)[: out.numel()]).view(out.shape))

    def head_norm(self, hidden, batch, seq, xn):
        hd = hidden[: batch * seq * MODEL.hidden].to(self.dev)
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


def _worker(rank, world, port, q, dtype):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def factory(lb, le, first, last, max_batch, max_ctx, hslice):
            return HipHostExecutor(dtype, lb, le, first, last, max_batch, max_ctx, hslice)
        pipe, rng = build_rank(MODEL, rank, world, torch.device("cpu"), mb_rows=MB, max_ctx=P + STEPS + 2, max_seq=P,
                               executor_factory=factory, head_split=True, dtype=dtype)
        prompt = torch.from_numpy(prompt_ids(1234, MB * pipe.n_mb, P, MODEL.vocab)) if rank == 0 else None
        toks = generate(pipe, prompt, STEPS, P)
        q.put((rank, rng, None if toks is None else toks.numpy()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_pipeline(dtype):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q, dtype)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        r, rng, toks = q.get(timeout=240)
        res[r] = (rng, toks)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [res[r][0] for r in range(WORLD)] == [(0, 8), (8, 16), (16, 23), (23, 30)]
    return res[0][1]


def test_3b_uneven_four_stage_split_fp32_greedy_identical():
    assert stage_ranges(WORLD, MODEL.n_layer) == [(0, 8), (8, 16), (16, 23), (23, 30)]
    got = _run_pipeline("fp32")
    B = got.shape[0]
    assert B == MB * 2 * WORLD and got.shape[1] == STEPS + 1
    ref = OracleStage(MODEL.hidden, MODEL.n_head, MODEL.n_layer, MODEL.vocab, 0, MODEL.n_layer, max_batch=B,
                      max_ctx=P + STEPS + 2, seed=SEED)
    tok = ref.forward(prompt_ids(1234, B, P, MODEL.vocab), B, P)
    want = [tok]
    for i in range(STEPS):
        tok = ref.forward(tok.reshape(B, 1), B, 1, past_len=P + i)
        want.append(tok)
    assert np.array_equal(got, np.stack(want, 1))


def test_3b_uneven_four_stage_split_bf16_teacher_forced():
    got = _run_pipeline("bf16")
    B = got.shape[0]
    ref = OracleStage(MODEL.hidden, MODEL.n_head, MODEL.n_layer, MODEL.vocab, 0, MODEL.n_layer, bf16=True,
                      max_batch=B, max_ctx=P + STEPS + 2, seed=SEED)
    _, lo = ref.forward(prompt_ids(1234, B, P, MODEL.vocab), B, P, want_logits=True)
    for i in range(STEPS + 1):
        want = lo.argmax(1)
        for b in np.flatnonzero(got[:, i] != want):
            top2 = np.sort(lo[b])[-2:]
            assert top2[1] - top2[0] < BF16_TOL, f"step {i} row {b}: {got[b, i]} != {want[b]}, top-2 {top2}"
        if i < STEPS:  # the checker continues on the pipeline's own tokens
            _, lo = ref.forward(got[:, i].reshape(B, 1).astype(np.int32), B, 1, past_len=P + i, want_logits=True)


_NCCL_WORLD1 = r"""
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.getcwd())
from distributed_inference_demo_amd import config
from distributed_inference_demo_amd.pipeline import build_rank, generate, init_distributed
from distributed_inference_demo_amd.stage import prompt_ids
rank, world, local = init_distributed("nccl", timeout_s=120)
assert (rank, world, dist.get_backend()) == (0, 1, "nccl")
m = config.BloomDims("tinygpu", 256, 2, 4, vocab=1024)
dev = torch.device("cuda", 0)
pipe, rng = build_rank(m, 0, 1, dev, dtype=sys.argv[2], mb_rows=2, n_mb=2, max_ctx=40, max_seq=8, seed=11)
assert rng == (0, 2) and type(pipe.ex).__name__ == "StageExecutor"
cs = torch.cuda.Stream()
torch.cuda.set_stream(cs)
prompt = torch.from_numpy(prompt_ids(1234, 4, 8, m.vocab)).to(dev)
toks = generate(pipe, prompt, 12, 8)
np.save(sys.argv[1], toks.cpu().numpy())
dist.destroy_process_group()
"""


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_pipeline_nccl_world1_stage_executor_graph_decode(dtype, tmp_path):
    """The product pipeline path end to end on one GPU: init_distributed("nccl") (an RCCL world-1 group
    with a timeout), build_rank -> a libbloomstage Stage behind StageExecutor, 2 micro-batches of 2 rows
    whose decode steps replay captured hipGraphs on device buffers.  fp32: greedy ids identical to the
    single-stage checker; bf16: every id the bf16 checker's argmax on the pipeline's own prefix unless the
    checker's top-2 margin is < 2e-2."""
    import subprocess
    import sys
    out = str(tmp_path / "toks.npy")
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run([sys.executable, "-c", _NCCL_WORLD1, out, dtype], check=True, env=env, cwd=root, timeout=180)
    got = np.load(out)
    B, steps = 4, 12
    assert got.shape == (B, steps + 1)
    ref = OracleStage(256, 4, 2, 1024, 0, 2, bf16=(dtype == "bf16"), max_batch=B, max_ctx=40, seed=11)
    tok, lo = ref.forward(prompt_ids(1234, B, 8, 1024), B, 8, want_logits=True)
    for i in range(steps + 1):
        if dtype == "fp32":
            assert np.array_equal(got[:, i], tok), (i, got[:, i], tok)
        else:
            for b in np.flatnonzero(got[:, i] != lo.argmax(1)):
                top2 = np.sort(lo[b])[-2:]
                assert top2[1] - top2[0] < BF16_TOL, f"step {i} row {b}: top-2 {top2}"
        if i < steps:  # the checker continues on the pipeline's own tokens
            tok, lo = ref.forward(got[:, i].reshape(B, 1).astype(np.int32), B, 1, past_len=8 + i, want_logits=True)
