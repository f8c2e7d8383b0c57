"""Pipeline-parallel BLOOM decode across GPUs: one process (rank) per stage, activations over
RCCL point-to-point (torch.distributed "nccl" == RCCL on ROCm) over xGMI.

Counterpart of the reference's per-device runtime:
  - placement   : `round_robin_module_arrangement` (server.py:893-905) -> placement.stage_ranges
  - hop         : ZeroMQ "Request Data" pull + serialized fp32 tensors (Communication.java:706-821,
                  utils.cpp:124-264) -> raw fp32 hidden [mb, S, h] device buffers, RCCL send/recv
  - token return: tail -> header 4-byte id (Communication.java:823-852) -> int32 [mb] RCCL send
                  on a dedicated communicator (separate stream, so it never queues behind
                  hidden-state sends between the same two ranks)
  - in-flight   : `core_pool_size` samples in flight (Communication.java:418-464) -> `n_mb`
                  micro-batches, each owning its own KV slots, so stage s computes micro-batch
                  j while stage s+1 computes j-1 and the hops overlap compute.
The schedule per rank is a static loop; every send/recv is posted in the same order on both
peers, so the pattern is deadlock free.  All P2P waits are stream-level (no host blocking on
RCCL), so the host enqueues ahead and the GPU stays busy.
"""
import os
import time

import torch
import torch.distributed as dist

from . import config
from .placement import stage_ranges


class StageExecutor:
    """Product executor: a libbloomstage Stage fed device tensors on the current stream."""

    def __init__(self, stage):
        self.stage = stage

    def forward(self, inp, out, batch, seq, slot, past_len):
        self.stage.forward(inp, out, batch, seq, slot=slot, past_len=past_len,
                           stream=torch.cuda.current_stream().cuda_stream)


class Pipeline:
    """Static pipeline schedule for one rank.

    rank 0 feeds prompt / token ids, rank N-1 returns token ids to rank 0.  With world == 1
    the single stage loops its own tokens back (no communication)."""

    def __init__(self, executor, *, rank, world, hidden, mb_rows, n_mb, device, is_first, is_last,
                 tok_group=None, max_seq=1):
        self.ex, self.rank, self.world = executor, rank, world
        self.h, self.mb, self.n_mb, self.dev = hidden, mb_rows, n_mb, device
        self.is_first, self.is_last = is_first, is_last
        self.tok_group = tok_group
        f32, i32 = torch.float32, torch.int32
        self.hin = [torch.empty(mb_rows * max_seq * hidden, dtype=f32, device=device) for _ in range(n_mb)]
        self.hout = [torch.empty(mb_rows * max_seq * hidden, dtype=f32, device=device) for _ in range(n_mb)]
        self.tok = [torch.zeros(mb_rows, dtype=i32, device=device) for _ in range(n_mb)]
        self.pending = [[] for _ in range(n_mb)]
        self.past = [0] * n_mb

    def _drain(self, j):
        for w in self.pending[j]:
            w.wait()
        self.pending[j] = []

    def step(self, seq, prompt=None, record=None):
        """One pipeline round: every micro-batch advances by `seq` tokens (seq = prompt length
        on the prefill round, 1 on decode rounds).  `prompt` [n_mb*mb, seq] int32 on rank 0
        for the prefill round; rank 0 appends the tokens it receives to `record`."""
        n_el = self.mb * seq * self.h
        last_rank = self.world - 1
        for j in range(self.n_mb):
            slot = j * self.mb
            self._drain(j)
            if self.is_first:
                if prompt is not None:
                    inp = prompt[j * self.mb:(j + 1) * self.mb].contiguous()
                else:
                    if self.world > 1:
                        dist.recv(self.tok[j], src=last_rank, group=self.tok_group) if _is_gloo() else \
                            dist.irecv(self.tok[j], src=last_rank, group=self.tok_group).wait()
                        if record is not None:
                            record[j].append(self.tok[j].clone())
                    inp = self.tok[j]
            else:
                buf = self.hin[j][:n_el]
                if _is_gloo():
                    dist.recv(buf, src=self.rank - 1)
                else:
                    dist.irecv(buf, src=self.rank - 1).wait()
                inp = buf
            if self.is_last:
                self.ex.forward(inp, self.tok[j], self.mb, seq, slot, self.past[j])
                if self.world > 1:
                    self.pending[j].append(dist.isend(self.tok[j], dst=0, group=self.tok_group))
                elif record is not None:
                    record[j].append(self.tok[j].clone())
            else:
                out = self.hout[j][:n_el]
                self.ex.forward(inp, out, self.mb, seq, slot, self.past[j])
                self.pending[j].append(dist.isend(out, dst=self.rank + 1))
            self.past[j] += seq

    def finish(self, record=None):
        """Rank 0 collects the tokens of the last round; everyone drains its sends."""
        if self.is_first and self.world > 1:
            for j in range(self.n_mb):
                if _is_gloo():
                    dist.recv(self.tok[j], src=self.world - 1, group=self.tok_group)
                else:
                    dist.irecv(self.tok[j], src=self.world - 1, group=self.tok_group).wait()
                if record is not None:
                    record[j].append(self.tok[j].clone())
        for j in range(self.n_mb):
            self._drain(j)


def _is_gloo():
    return dist.is_initialized() and dist.get_backend() == "gloo"


def generate(pipe: Pipeline, prompt, steps, prompt_len):
    """Greedy-decode `steps` tokens for every row after a `prompt_len`-token prompt (`prompt`
    [n_mb*mb, prompt_len] on rank 0, None elsewhere).  Rank 0 returns the ids
    [n_mb*mb, steps+1] (first generated token .. last); other ranks return None."""
    rec = [[] for _ in range(pipe.n_mb)] if pipe.is_first else None
    pipe.step(prompt_len, prompt=prompt, record=rec)
    for _ in range(steps):
        pipe.step(1, record=rec)
    pipe.finish(record=rec)
    if not pipe.is_first:
        return None
    return torch.cat([torch.stack(r, 1) for r in rec], 0)


def init_distributed(backend=None):
    """Read RANK/WORLD_SIZE/LOCAL_RANK/MASTER_* (torchrun) and initialise the process group."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        kw = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, world, local


def build_rank(model: config.BloomDims, rank, world, device, *, dtype="bf16", mb_rows=1, n_mb=None, max_ctx=1024,
               max_seq=512, seed=0, executor_factory=None):
    """Create this rank's stage (server.py:893-905 layer range) and its Pipeline."""
    n_mb = world if n_mb is None else n_mb
    lb, le = stage_ranges(world, model.n_layer)[rank]
    if executor_factory is None:
        from .stage import Stage
        st = Stage(model.hidden, model.n_head, model.n_layer, model.vocab, lb, le, dtype=dtype,
                   device=device.index if device.type == "cuda" else 0, max_batch=mb_rows * n_mb,
                   max_ctx=max_ctx, max_tokens=mb_rows * max_seq, seed=seed, is_first=(rank == 0),
                   is_last=(rank == world - 1))
        ex = StageExecutor(st)
    else:
        ex = executor_factory(lb, le, rank == 0, rank == world - 1, mb_rows * n_mb, max_ctx)
    tok_group = dist.new_group(ranks=sorted({0, world - 1})) if world > 1 else None
    pipe = Pipeline(ex, rank=rank, world=world, hidden=model.hidden, mb_rows=mb_rows, n_mb=n_mb, device=device,
                    is_first=(rank == 0), is_last=(rank == world - 1), tok_group=tok_group, max_seq=max_seq)
    return pipe, (lb, le)


def bench_pipeline(args):
    """bench.py --gpus N under torchrun: N stages, N micro-batches of `batch` rows in flight."""
    rank, world, local = init_distributed("nccl")
    dev = torch.device("cuda", local)
    model = config.get(args.model)
    B, P, K, W = args.batch, args.prompt, args.steps, args.warmup
    pipe, (lb, le) = build_rank(model, rank, world, dev, dtype=args.dtype, mb_rows=B, n_mb=world,
                                max_ctx=P + W + K + 2, max_seq=P, seed=args.seed)
    cs = torch.cuda.Stream()  # a real stream: decode steps are captured as hipGraphs
    torch.cuda.set_stream(cs)
    prompt = None
    if rank == 0:
        from .stage import prompt_ids
        prompt = torch.from_numpy(prompt_ids(1234, B * world, P, model.vocab)).to(dev)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pipe.step(P, prompt=prompt)
    for _ in range(W):
        pipe.step(1)
    torch.cuda.synchronize()
    dist.barrier()
    t_prefill_warm = time.perf_counter() - t0
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        pipe.step(1)
    pipe.finish()
    torch.cuda.synchronize()
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt.item())
    per_stage = [b - a for a, b in stage_ranges(world, model.n_layer)]
    res = None
    if rank == 0:
        toks = B * world * K
        res = {
            "metric": "decode tokens/s, BLOOM pipeline", "value": toks / dt, "unit": "tokens/s", "n_gpus": world,
            "steps": K, "warmup": W, "ms_per_step": dt * 1e3 / K, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic: repo-generator random-init weights (seed %d), prompt ids U[0,V) seed 1234" % args.seed,
            "config": {"workload": f"{model.name} split into {world} stages by the server's round-robin layer "
                                   f"assignment, {world} micro-batches x {B} rows in flight, RCCL send/recv",
                       "model": model.name, "stages": world, "layers_per_stage": per_stage, "batch": B * world,
                       "micro_batch": B, "prompt": P, "parallelism": f"pp{world}"},
            "prefill_plus_warmup_s": t_prefill_warm,
        }
    dist.barrier()
    dist.destroy_process_group()
    return res
