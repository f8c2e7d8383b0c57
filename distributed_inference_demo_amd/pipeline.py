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

    def head_norm(self, hidden, batch, seq, xn):
        self.stage.head_norm(hidden, batch, seq, xn, stream=torch.cuda.current_stream().cuda_stream)

    def head_slice(self, xn, batch, keys_in, keys_out, tokens):
        self.stage.head_slice(xn, batch, keys_in, keys_out, tokens, stream=torch.cuda.current_stream().cuda_stream)


def vocab_slices(vocab, world):
    """Contiguous 16-aligned vocabulary slices, one per rank (the vocabulary-parallel head)."""
    per = ((vocab + world - 1) // world + 15) // 16 * 16
    return [(min(vocab, r * per), min(vocab, (r + 1) * per)) for r in range(world)]


def _is_gloo():
    return dist.is_initialized() and dist.get_backend() == "gloo"


def _recv(buf, src, group=None):
    if _is_gloo():
        dist.recv(buf, src=src, group=group)
    else:
        dist.irecv(buf, src=src, group=group).wait()  # stream-level wait on the current stream


class Pipeline:
    """Static pipeline schedule for one rank.

    Layer chain: rank 0 feeds prompt / token ids, hidden states go rank -> rank+1.
    Token pick, two modes:
      head_split=False: the last rank holds the whole lm_head and returns int32 tokens to rank 0
                        (on `tok_group`).
      head_split=True : every rank holds a V/N slice of the tied lm_head.  The last rank computes
                        ln_f -> xn and its slice's argmax keys, and the (xn, keys) pair travels the
                        head ring N-1 -> 0 -> 1 -> ... -> N-2 on `head_group` (its own stream); the
                        rank closing the ring decodes the token and returns it to rank 0 (on
                        `tok_group`, or locally when that rank is 0).  The layer assignment is
                        unchanged; the per-rank head work is 1/N of the lm_head.
    With world == 1 the single stage loops its own tokens back (no communication)."""

    def __init__(self, executor, *, rank, world, hidden, mb_rows, n_mb, device, is_first, is_last,
                 tok_group=None, head_group=None, head_split=False, act_dtype=torch.float32, max_seq=1):
        self.ex, self.rank, self.world = executor, rank, world
        self.h, self.mb, self.n_mb, self.dev = hidden, mb_rows, n_mb, device
        self.is_first, self.is_last = is_first, is_last
        self.tok_group, self.head_group = tok_group, head_group
        self.head_split = head_split and world > 1
        f32, i32 = torch.float32, torch.int32
        self.hin = [torch.empty(mb_rows * max_seq * hidden, dtype=f32, device=device) for _ in range(n_mb)]
        self.hout = [torch.empty(mb_rows * max_seq * hidden, dtype=f32, device=device) for _ in range(n_mb)]
        self.tok = [torch.zeros(mb_rows, dtype=i32, device=device) for _ in range(n_mb)]
        self.pending = [[] for _ in range(n_mb)]
        self.hpending = [[] for _ in range(n_mb)]
        self.past = [0] * n_mb
        self.tokens_held = False  # after finish(): rank 0 already holds every micro-batch's next input
        if self.head_split:
            self.xn = [torch.empty(mb_rows * hidden, dtype=act_dtype, device=device) for _ in range(n_mb)]
            self.kin = [torch.zeros(mb_rows, dtype=torch.int64, device=device) for _ in range(n_mb)]
            self.kout = [torch.zeros(mb_rows, dtype=torch.int64, device=device) for _ in range(n_mb)]
            cuda = device.type == "cuda"
            self.hstream = torch.cuda.Stream(device) if cuda else None
            self.tok_ready = [torch.cuda.Event() for _ in range(n_mb)] if cuda else None
            self.closer = world - 2  # rank whose slice closes the head ring

    @staticmethod
    def _drain(lst):
        for w in lst:
            w.wait()
        lst.clear()

    # -- head ring (head_split) -------------------------------------------------------
    def _hctx(self):
        return torch.cuda.stream(self.hstream) if self.hstream is not None else _nullctx()

    def _head_role(self, j, record):
        """Ranks 0..N-2: receive (xn, keys) from the previous ring rank, fold in this slice, pass on."""
        prev = self.world - 1 if self.rank == 0 else self.rank - 1
        with self._hctx():
            self._drain(self.hpending[j])
            _recv(self.xn[j], prev, self.head_group)
            _recv(self.kin[j], prev, self.head_group)
            if self.rank == self.closer:
                self.ex.head_slice(self.xn[j], self.mb, self.kin[j], None, self.tok[j])
                if self.rank == 0:
                    if self.tok_ready is not None:
                        self.tok_ready[j].record()
                else:
                    self.hpending[j].append(dist.isend(self.tok[j], dst=0, group=self.tok_group))
            else:
                self.ex.head_slice(self.xn[j], self.mb, self.kin[j], self.kout[j], None)
                self.hpending[j].append(dist.isend(self.xn[j], dst=self.rank + 1, group=self.head_group))
                self.hpending[j].append(dist.isend(self.kout[j], dst=self.rank + 1, group=self.head_group))

    def _token_in(self, j, record):
        """Rank 0: the token of micro-batch j from the previous round."""
        if self.world == 1:
            return
        if self.head_split and self.closer == 0:
            if self.tok_ready is not None:
                torch.cuda.current_stream().wait_event(self.tok_ready[j])
        else:
            src = self.closer if self.head_split else self.world - 1
            _recv(self.tok[j], src, self.tok_group)
        if record is not None:
            record[j].append(self.tok[j].clone())

    def step(self, seq, prompt=None, record=None, feed=None, pasts=None):
        """One pipeline round: every micro-batch advances by `seq` tokens (seq = prompt length
        on the prefill round, 1 on decode rounds).  `prompt` [n_mb*mb, seq] int32 on rank 0
        for the prefill round; rank 0 appends the tokens it receives to `record`.
        Continuous batching (serve.py): `pasts[j]` = every row's own position this round (all
        ranks, the same schedule); `feed[j]` = (tokens, mask) int32/bool [mb] on rank 0's device:
        rows with mask set take `tokens` (a prompt token, or a new sample's first token) instead of
        the token the pipeline returned for them."""
        n_el = self.mb * seq * self.h
        for j in range(self.n_mb):
            slot = j * self.mb
            if pasts is not None:
                self.past[j] = list(pasts[j])
            self._drain(self.pending[j])
            if self.is_first:
                if prompt is not None:
                    inp = prompt[j * self.mb:(j + 1) * self.mb].contiguous()
                else:
                    if not self.tokens_held:
                        self._token_in(j, record)
                    inp = self.tok[j]
                    if feed is not None:
                        inp = torch.where(feed[j][1], feed[j][0], inp)
            else:
                inp = self.hin[j][:n_el]
                _recv(inp, self.rank - 1)
            if self.is_last and not self.head_split:
                self.ex.forward(inp, self.tok[j], self.mb, seq, slot, self.past[j])
                if self.world > 1:
                    self.pending[j].append(dist.isend(self.tok[j], dst=0, group=self.tok_group))
                elif record is not None:
                    record[j].append(self.tok[j].clone())
            else:
                out = self.hout[j][:n_el]
                self.ex.forward(inp, out, self.mb, seq, slot, self.past[j])
                if not self.is_last:
                    self.pending[j].append(dist.isend(out, dst=self.rank + 1))
                else:  # head_split: open the head ring with ln_f and this rank's slice
                    self.ex.head_norm(out, self.mb, seq, self.xn[j])
                    self.ex.head_slice(self.xn[j], self.mb, None, self.kout[j], None)
                    self.pending[j].append(dist.isend(self.xn[j], dst=0, group=self.head_group))
                    self.pending[j].append(dist.isend(self.kout[j], dst=0, group=self.head_group))
            if self.head_split and self.rank <= self.closer:
                self._head_role(j, record)
            self.past[j] = [p + seq for p in self.past[j]] if isinstance(self.past[j], list) else self.past[j] + seq
        self.tokens_held = False

    def finish(self, record=None):
        """Rank 0 collects the tokens of the last round; everyone drains its sends.  Later steps
        continue from those tokens."""
        if self.is_first and self.world > 1 and not self.tokens_held:
            for j in range(self.n_mb):
                self._token_in(j, record)
            self.tokens_held = True
        for j in range(self.n_mb):
            self._drain(self.pending[j])
            self._drain(self.hpending[j])
        if self.head_split and self.hstream is not None:
            torch.cuda.current_stream().wait_stream(self.hstream)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


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
               max_seq=512, seed=0, head_split=None, executor_factory=None):
    """Create this rank's stage (server.py:893-905 layer range, plus a vocabulary slice of the
    tied lm_head when head_split) and its Pipeline.  Collective: every rank must call it."""
    head_split = (world > 1) if head_split is None else (head_split and world > 1)
    n_mb = (2 * world if head_split else world) if n_mb is None else n_mb
    if world > model.n_layer:
        raise ValueError(f"{world} stages for {model.n_layer} layers: every stage needs at least one layer")
    if head_split and world > model.vocab // 16:
        raise ValueError(f"vocabulary-parallel head: {world} slices of a {model.vocab}-token vocabulary "
                         "leave a slice without a 16-column tile")
    if model.int8_weights and dtype != "bf16":
        raise ValueError(f"{model.name}: weight-only int8 stages need dtype bf16 (got {dtype})")
    lb, le = stage_ranges(world, model.n_layer)[rank]
    is_first, is_last = rank == 0, rank == world - 1
    hslice = vocab_slices(model.vocab, world)[rank] if head_split else None
    if executor_factory is None:
        from .stage import Stage
        st = Stage(model.hidden, model.n_head, model.n_layer, model.vocab, lb, le, dtype=dtype,
                   device=device.index if device.type == "cuda" else 0, max_batch=mb_rows * n_mb,
                   max_ctx=max_ctx, max_tokens=mb_rows * max_seq, seed=seed, is_first=is_first,
                   is_last=is_last and not head_split, head_slice=hslice, int8_weights=model.int8_weights)
        ex = StageExecutor(st)
    else:
        ex = executor_factory(lb, le, is_first, is_last and not head_split, mb_rows * n_mb, max_ctx, hslice)
    # communicators are created collectively, in the same order on every rank
    tok_group = head_group = None
    if world > 1:
        tok_group = dist.new_group(ranks=list(range(world)))
        head_group = dist.new_group(ranks=list(range(world)))
    act = torch.bfloat16 if dtype == "bf16" else torch.float32
    pipe = Pipeline(ex, rank=rank, world=world, hidden=model.hidden, mb_rows=mb_rows, n_mb=n_mb, device=device,
                    is_first=is_first, is_last=is_last, tok_group=tok_group, head_group=head_group,
                    head_split=head_split, act_dtype=act, max_seq=max_seq)
    return pipe, (lb, le)


def _stage_step_bytes(model, lb, le, rows, ctx, first, last, hslice, w_bytes, kv_bytes):
    """Algorithmic HBM bytes of one decode forward of a stage (BASELINE.md formula) plus, with the
    vocabulary-parallel head, the stage's lm_head slice and ln_f."""
    b = config.decode_step_bytes(model, le - lb, rows, ctx, first, last, w_bytes=w_bytes, kv_bytes=kv_bytes)
    if hslice is not None:
        b += (hslice[1] - hslice[0]) * model.hidden * w_bytes + 2 * model.hidden * w_bytes
    return b


def bench_pipeline(args):
    """bench.py --gpus N under torchrun: N stages, n_mb micro-batches of `batch` rows in flight.
    Rank 0 returns the JSON dict (with per-stage roofline / HBM figures gathered from every rank) and
    the stage ranges (for the host-CPU baseline of the same split)."""
    rank, world, local = init_distributed("nccl")
    dev = torch.device("cuda", local)
    model = config.get(args.model)
    if getattr(args, "weights", "bf16") == "int8":
        model = config.get(model.name if model.int8_weights else model.name + "-int8")
    B, P, K, W = args.batch, args.prompt, args.steps, args.warmup
    prof_rounds = 0 if getattr(args, "no_profile", False) else 8
    head_split = not getattr(args, "no_head_split", False)
    pipe, (lb, le) = build_rank(model, rank, world, dev, dtype=args.dtype, mb_rows=B,
                                max_ctx=P + W + K + prof_rounds + 2, max_seq=P, seed=args.seed, head_split=head_split)
    n_mb = pipe.n_mb
    cs = torch.cuda.Stream()  # a real stream: decode steps are captured as hipGraphs
    torch.cuda.set_stream(cs)
    prompt = None
    if rank == 0:
        from .stage import prompt_ids
        prompt = torch.from_numpy(prompt_ids(1234, B * n_mb, P, model.vocab)).to(dev)
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
    t_round = dt / K
    # per-stage roofline: eager rounds with HIP events around every decode weight GEMV of this stage
    st = pipe.ex.stage if hasattr(pipe.ex, "stage") else None
    g = None
    if st is not None and prof_rounds:
        st.profile_enable(1)
        for _ in range(prof_rounds):
            pipe.step(1)
        pipe.finish()
        torch.cuda.synchronize()
        g = st.profile_read()
        st.profile_enable(0)
    dist.barrier()
    hslice = vocab_slices(model.vocab, world)[rank] if pipe.head_split else None
    w_b = 2 if args.dtype == "bf16" else 4
    ctx_mid = P + W + K / 2
    step_bytes = _stage_step_bytes(model, lb, le, B, ctx_mid, rank == 0, rank == world - 1 and not pipe.head_split,
                                   hslice, w_b, w_b)
    if model.int8_weights:
        step_bytes -= (le - lb) * (12.0 * model.hidden * model.hidden * 1 - 9.0 * model.hidden * 4)
    mine = {"rank": rank, "layers": [lb, le], "head_slice": list(hslice) if hslice else None,
            "algo_bytes_per_forward": step_bytes,
            "achieved_GBps": n_mb * step_bytes / t_round / 1e9}
    mine["frac_of_peak"] = mine["achieved_GBps"] / 8000.0
    if g is not None and g[1]:
        ms, n, byts = g
        mine["gemv"] = {"launches": n, "avg_us": ms / n * 1e3, "achieved_GBps": (byts / n) / (ms / n * 1e-3) / 1e9}
    allst = [None] * world
    dist.all_gather_object(allst, mine)
    per_stage = [b - a for a, b in stage_ranges(world, model.n_layer)]
    res = None
    if rank == 0:
        toks = B * n_mb * K
        gemv = [x["gemv"] for x in allst if "gemv" in x]
        res = {
            "metric": "decode tokens/s, BLOOM pipeline", "value": toks / dt, "unit": "tokens/s", "n_gpus": world,
            "steps": K, "warmup": W, "ms_per_step": dt * 1e3 / K, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic: repo-generator random-init weights (seed %d), prompt ids U[0,V) seed 1234" % args.seed,
            "config": {"workload": f"{model.name} split into {world} stages by the server's round-robin layer "
                                   f"assignment, {n_mb} micro-batches x {B} rows in flight, RCCL send/recv"
                                   + (", vocabulary-parallel lm_head ring" if pipe.head_split else ""),
                       "model": model.name, "stages": world, "layers_per_stage": per_stage, "batch": B * n_mb,
                       "micro_batch": B, "prompt": P, "parallelism": f"pp{world}",
                       "head": "vocab-split ring" if pipe.head_split else "last stage",
                       "hop": "fp32 hidden [mb, S, h] (the reference wire dtype; keeps the split bit-identical to one stage)"},
            "prefill_plus_warmup_s": t_prefill_warm,
            "per_stage": allst,
            "stage_hbm": {"achieved_GBps_min": min(x["achieved_GBps"] for x in allst),
                          "achieved_GBps_mean": sum(x["achieved_GBps"] for x in allst) / world,
                          "frac_of_peak_min": min(x["frac_of_peak"] for x in allst),
                          "frac_of_peak_mean": sum(x["frac_of_peak"] for x in allst) / world,
                          "note": "per stage: n_mb x algorithmic bytes of one forward / time of one pipeline round"},
        }
        if gemv:
            tot_t = sum(x["launches"] * x["avg_us"] for x in gemv)
            tot_b = sum(x["launches"] * x["avg_us"] * 1e-6 * x["achieved_GBps"] * 1e9 for x in gemv)
            ach = tot_b / (tot_t * 1e-6) / 1e9
            res["roofline"] = {"bound": "hbm", "kernel": "gemv_rows_kernel (decode weight GEMVs of every stage)",
                               "achieved": ach, "peak": 8000.0, "unit": "GB/s", "frac": ach / 8000.0, "traffic": None,
                               "launches": sum(x["launches"] for x in gemv), "avg_us": tot_t / sum(x["launches"] for x in gemv),
                               "measured": f"HIP events per launch on each stage's stream, {prof_rounds} eager pipeline "
                                           "rounds after the timed region; bytes and time summed over all stages"}
    dist.barrier()
    dist.destroy_process_group()
    return res, stage_ranges(world, model.n_layer), model
