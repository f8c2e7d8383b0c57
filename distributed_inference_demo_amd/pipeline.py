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
peers (DESIGN.md section 6 "Why the schedule cannot deadlock"), and every point-to-point pair is
connected in one global order before the first round (`connect_p2p`).  All P2P waits are
stream-level (no host blocking on RCCL), so the host enqueues ahead and the GPU stays busy.
"""
import datetime
import os
import time

import torch
import torch.distributed as dist

from . import config
from .placement import stage_ranges


class StageExecutor:
    """Product executor: a libbloomstage Stage fed device tensors on the current stream.  Pipeline.step hands it the
    round's stream handle once (set_stream) so the per-micro-batch forward does not look it up through torch again
    (tools/host_enqueue.py: the host enqueue per micro-batch is what an N = 8 rank must keep ahead of the GPU)."""

    def __init__(self, stage):
        self.stage = stage
        self._sh = None
        self._side = None

    def set_stream(self, handle):
        self._sh = handle

    def _run(self, call, tensors):
        """Enqueue `call(stream handle)` ordered with torch's current stream.  Torch's default stream has handle 0,
        which the C-ABI reads as NULL = the stage's own (non-blocking) stream, unordered with it: on the default
        stream the call runs on a side stream fenced both ways instead."""
        sh = torch.cuda.current_stream().cuda_stream
        if sh:
            call(sh)
            return
        cur = torch.cuda.current_stream()
        if self._side is None:
            self._side = torch.cuda.Stream(cur.device)
        self._side.wait_stream(cur)
        call(self._side.cuda_stream)
        for t in tensors:
            if t is not None:
                t.record_stream(self._side)
        cur.wait_stream(self._side)

    def forward(self, inp, out, batch, seq, slot, past_len):
        sh = self._sh if self._sh is not None else torch.cuda.current_stream().cuda_stream
        if sh:  # the pipeline's rounds: a stream of their own (the host enqueue stays one call)
            self.stage.forward(inp, out, batch, seq, slot=slot, past_len=past_len, stream=sh)
            return
        self._run(lambda h: self.stage.forward(inp, out, batch, seq, slot=slot, past_len=past_len, stream=h),
                  (inp, out))

    def head_norm(self, hidden, batch, seq, xn):
        sh = torch.cuda.current_stream().cuda_stream
        if sh:
            self.stage.head_norm(hidden, batch, seq, xn, stream=sh)
            return
        self._run(lambda h: self.stage.head_norm(hidden, batch, seq, xn, stream=h), (hidden, xn))

    def head_slice(self, xn, batch, keys_in, keys_out, tokens):
        sh = torch.cuda.current_stream().cuda_stream
        if sh:
            self.stage.head_slice(xn, batch, keys_in, keys_out, tokens, stream=sh)
            return
        self._run(lambda h: self.stage.head_slice(xn, batch, keys_in, keys_out, tokens, stream=h),
                  (xn, keys_in, keys_out, tokens))


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
                 tok_group=None, head_group=None, head_split=False, act_dtype=torch.float32, max_seq=1,
                 pf_group=None):
        self.ex, self.rank, self.world = executor, rank, world
        self.h, self.mb, self.n_mb, self.dev = hidden, mb_rows, n_mb, device
        self.is_first, self.is_last = is_first, is_last
        self.tok_group, self.head_group, self.pf_group = tok_group, head_group, pf_group
        self.head_split = head_split and world > 1
        f32, i32 = torch.float32, torch.int32
        self.hin = [torch.empty(mb_rows * max_seq * hidden, dtype=f32, device=device) for _ in range(n_mb)]
        self.hout = [torch.empty(mb_rows * max_seq * hidden, dtype=f32, device=device) for _ in range(n_mb)]
        self.tok = [torch.zeros(mb_rows, dtype=i32, device=device) for _ in range(n_mb)]
        self.pf_tok = [torch.zeros(mb_rows, dtype=i32, device=device) for _ in range(n_mb)]  # prefill_row's tokens
        self.pending = [[] for _ in range(n_mb)]
        self.hpending = [[] for _ in range(n_mb)]
        # token returns of the decode rounds (tok_group), kept apart: rank 0 receives a round's tokens only at
        # the start of the next round, so a prefill_row pass in between must not wait for them
        self.tsend = [[] for _ in range(n_mb)]
        self.past = [0] * n_mb
        self.tokens_held = False  # after finish(): rank 0 already holds every micro-batch's next input
        self._views = {}  # (buffer list id, micro-batch, elements) -> the sliced view (a torch slice costs ~3 us)
        if self.head_split:
            # one packed ring message per micro-batch: [xn (mb x h, activation dtype) | argmax keys (mb x int64)],
            # so a ring hop is ONE send and ONE receive (each RCCL call costs the host ~8-11 us: tools/host_enqueue.py);
            # ring ranks fold their slice into the keys in place (bs_head_slice allows keys_in == keys_out).
            # prefill_row's one-row passes use a one-row message of the same layout.
            self.hmsg, self.xn, self.hkeys = self._ring_buffers(mb_rows, hidden, act_dtype, device, n_mb)
            self.pmsg, self.pxn, self.pkeys = self._ring_buffers(1, hidden, act_dtype, device, n_mb)
            cuda = device.type == "cuda"
            self.hstream = torch.cuda.Stream(device) if cuda else None
            self.tok_ready = [torch.cuda.Event() for _ in range(n_mb)] if cuda else None
            self.closer = world - 2  # rank whose slice closes the head ring

    def _view(self, bufs, j, n):
        key = (id(bufs), j, n)
        v = self._views.get(key)
        if v is None:
            v = self._views[key] = bufs[j][:n]
        return v

    @staticmethod
    def _ring_buffers(rows, hidden, act_dtype, device, n):
        esz = torch.tensor([], dtype=act_dtype).element_size()
        nx = rows * hidden * esz
        nx8 = (nx + 7) // 8 * 8
        msgs = [torch.zeros(nx8 + 8 * rows, dtype=torch.uint8, device=device) for _ in range(n)]
        return msgs, [m[:nx].view(act_dtype) for m in msgs], [m[nx8:].view(torch.int64) for m in msgs]

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
            self._drain(self.tsend[j])
            _recv(self.hmsg[j], prev, self.head_group)
            if self.rank == self.closer:
                self.ex.head_slice(self.xn[j], self.mb, self.hkeys[j], None, self.tok[j])
                if self.rank == 0:
                    if self.tok_ready is not None:
                        self.tok_ready[j].record()
                else:
                    self.tsend[j].append(dist.isend(self.tok[j], dst=0, group=self.tok_group))
            else:
                self.ex.head_slice(self.xn[j], self.mb, self.hkeys[j], self.hkeys[j], None)
                self.hpending[j].append(dist.isend(self.hmsg[j], dst=self.rank + 1, group=self.head_group))

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

    def _forward(self, inp, out, seq, slot, j, timing):
        if timing is None:
            self.ex.forward(inp, out, self.mb, seq, slot, self.past[j])
            return
        if self.dev.type != "cuda":  # host executors run synchronously: host-clock pairs in ms
            t0 = time.perf_counter() * 1e3
            self.ex.forward(inp, out, self.mb, seq, slot, self.past[j])
            timing.append((t0, time.perf_counter() * 1e3))
            return
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        self.ex.forward(inp, out, self.mb, seq, slot, self.past[j])
        e1.record()
        timing.append((e0, e1))

    def step(self, seq, prompt=None, record=None, feed=None, pasts=None, timing=None):
        """One pipeline round: every micro-batch advances by `seq` tokens (seq = prompt length
        on the prefill round, 1 on decode rounds).  `prompt` [n_mb*mb, seq] int32 on rank 0
        for the prefill round; rank 0 appends the tokens it receives to `record`.
        Continuous batching (serve.py): `pasts[j]` = every row's own position this round (all
        ranks, the same schedule); `feed[j]` = (tokens, mask) int32/bool [mb] on rank 0's device:
        rows with mask set take `tokens` (a prompt token, or a new sample's first token) instead of
        the token the pipeline returned for them.  `timing` (a list): one (start, end) pair per stage
        forward of this round is appended -- HIP events on CUDA ranks, host-clock ms otherwise (stage
        busy time, pipeline_bench's prefill overlap)."""
        n_el = self.mb * seq * self.h
        if self.dev.type == "cuda" and hasattr(self.ex, "set_stream"):
            self.ex.set_stream(torch.cuda.current_stream().cuda_stream)
        for j in range(self.n_mb):
            slot = j * self.mb
            if pasts is not None:
                self.past[j] = list(pasts[j])
            self._drain(self.pending[j])
            if not self.head_split:
                self._drain(self.tsend[j])
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
                inp = self._view(self.hin, j, n_el)
                _recv(inp, self.rank - 1)
            if self.is_last and not self.head_split:
                self._forward(inp, self.tok[j], seq, slot, j, timing)
                if self.world > 1:
                    self.tsend[j].append(dist.isend(self.tok[j], dst=0, group=self.tok_group))
                elif record is not None:
                    record[j].append(self.tok[j].clone())
            else:
                out = self._view(self.hout, j, n_el)
                self._forward(inp, out, seq, slot, j, timing)
                if not self.is_last:
                    self.pending[j].append(dist.isend(out, dst=self.rank + 1))
                else:  # head_split: open the head ring with ln_f and this rank's slice
                    self.ex.head_norm(out, self.mb, seq, self.xn[j])
                    self.ex.head_slice(self.xn[j], self.mb, None, self.hkeys[j], None)
                    self.pending[j].append(dist.isend(self.hmsg[j], dst=0, group=self.head_group))
            if self.head_split and self.rank <= self.closer:
                self._head_role(j, record)
            self.past[j] = [p + seq for p in self.past[j]] if isinstance(self.past[j], list) else self.past[j] + seq
        self.tokens_held = False
        if hasattr(self.ex, "set_stream"):
            # the handle is this round's: a later prefill_row (or a caller that switched streams) looks the current
            # stream up again, so its forward stays ordered with its own receive and send
            self.ex.set_stream(None)

    def prefill_row(self, j, r, ids, n):
        """One pipeline pass of row r of micro-batch j alone: its n prompt tokens at positions 0..n-1 of KV slot
        j * mb + r (a new sample taking the row: serve.py's admission prefill, Communication.java:418-464).
        `ids` int32 [1, n] on rank 0 (None elsewhere).  The first generated token lands in self.pf_tok[j][r] on
        rank 0 (stream-ordered); it travels on `pf_group`, so it never interleaves with the decode rounds'
        token returns on `tok_group`.  Every rank calls this in the same order as every other rank."""
        n_el = n * self.h
        slot = j * self.mb + r
        tok = self.pf_tok[j][r:r + 1]
        self._drain(self.pending[j])
        if self.is_first:
            inp = ids
        else:
            inp = self.hin[j][:n_el]
            _recv(inp, self.rank - 1)
        if self.is_last and not self.head_split:
            self.ex.forward(inp, tok, 1, n, slot, 0)
            if self.world > 1:
                self.pending[j].append(dist.isend(tok, dst=0, group=self.pf_group))
        else:
            out = self.hout[j][:n_el]
            self.ex.forward(inp, out, 1, n, slot, 0)
            if not self.is_last:
                self.pending[j].append(dist.isend(out, dst=self.rank + 1))
            else:  # head_split: open the head ring
                self.ex.head_norm(out, 1, n, self.pxn[j])
                self.ex.head_slice(self.pxn[j], 1, None, self.pkeys[j], None)
                self.pending[j].append(dist.isend(self.pmsg[j], dst=0, group=self.head_group))
        if self.head_split and self.rank <= self.closer:
            prev = self.world - 1 if self.rank == 0 else self.rank - 1
            with self._hctx():
                self._drain(self.hpending[j])
                _recv(self.pmsg[j], prev, self.head_group)
                if self.rank == self.closer:
                    self.ex.head_slice(self.pxn[j], 1, self.pkeys[j], None, tok)
                    if self.rank != 0:
                        self.hpending[j].append(dist.isend(tok, dst=0, group=self.pf_group))
                else:
                    self.ex.head_slice(self.pxn[j], 1, self.pkeys[j], self.pkeys[j], None)
                    self.hpending[j].append(dist.isend(self.pmsg[j], dst=self.rank + 1, group=self.head_group))
            if self.rank == 0 and self.closer == 0 and self.hstream is not None:
                torch.cuda.current_stream().wait_stream(self.hstream)
        if self.is_first and self.world > 1 and not (self.head_split and self.closer == 0):
            _recv(tok, self.closer if self.head_split else self.world - 1, self.pf_group)
        return tok

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
            self._drain(self.tsend[j])
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


def classify(pipe: Pipeline, prompt, prompt_len):
    """The reference's classification task (max_length == 0: one OneStep pass per sample, Communication.java:591-603,
    the tail running runInferenceWorkerResidualLastClassification, native-lib.cpp:1305-1366): one pipeline pass of
    `prompt` [n_mb*mb, prompt_len] (rank 0; None elsewhere) from empty KV rows through a pipeline whose last stage
    is a classifier (build_rank(..., n_labels=...)).  Rank 0 returns the class ids [n_mb*mb]; other ranks None.
    Collective: every rank calls it."""
    pipe.past = [0] * pipe.n_mb  # every pass classifies new samples
    rec = [[] for _ in range(pipe.n_mb)] if pipe.is_first else None
    pipe.step(prompt_len, prompt=prompt, record=rec)
    pipe.finish(record=rec)
    if not pipe.is_first:
        return None
    return torch.cat([r[-1] for r in rec], 0)


def init_distributed(backend=None, timeout_s=None):
    """Read RANK/WORLD_SIZE/LOCAL_RANK/MASTER_* (torchrun) and initialise the process group.  Every
    collective and point-to-point wait is bounded by `timeout_s` (env BS_PIPELINE_TIMEOUT_S, default
    600 s): a schedule that stalls fails with an error instead of hanging the node."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if timeout_s is None:
        timeout_s = float(os.environ.get("BS_PIPELINE_TIMEOUT_S", "600"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        kw = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, world, local


def p2p_edges(world, head_split):
    """Every directed point-to-point edge the schedule uses, as (group name, src, dst), in one global order:
    hidden states r -> r+1 ("hidden"), the head ring N-1 -> 0 -> 1 -> ... -> N-2 ("head", a chain that ends
    at the closer N-2: no edge closes the cycle), tokens back to rank 0 ("tok", from the closer or from the
    last rank) and the admission prefills' first tokens ("pf", the same two ranks on a communicator of
    their own)."""
    if world <= 1:
        return []
    e = [("hidden", r, r + 1) for r in range(world - 1)]
    if head_split:
        closer = world - 2
        ring = [world - 1] + list(range(0, closer + 1))
        e += [("head", a, b) for a, b in zip(ring, ring[1:])]
        if closer != 0:
            e.append(("tok", closer, 0))
            e.append(("pf", closer, 0))
    else:
        e.append(("tok", world - 1, 0))
        e.append(("pf", world - 1, 0))
    return e


def connect_p2p(rank, world, head_split, groups, device):
    """Open every point-to-point connection of the schedule before the first round, one edge at a time in
    p2p_edges' global order, each a blocking 1-element exchange between its two ranks.  RCCL/NCCL connect a
    pair lazily on its first send/recv and the host blocks there until the peer arrives; done here in one
    order that every rank follows, the earliest unfinished edge always has both its ranks waiting on it, so
    the exchanges complete (deadlock-free), and the timed rounds never block the host on a connection."""
    buf = torch.zeros(1, dtype=torch.int32, device=device)
    for name, a, b in p2p_edges(world, head_split):
        g = groups[name]
        if rank == a:
            dist.send(buf, dst=b, group=g)
        elif rank == b:
            dist.recv(buf, src=a, group=g)
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def build_rank(model: config.BloomDims, rank, world, device, *, dtype="bf16", mb_rows=1, n_mb=None, max_ctx=1024,
               max_seq=512, seed=0, head_split=None, executor_factory=None, n_labels=0):
    """Create this rank's stage (server.py:893-905 layer range, plus a vocabulary slice of the
    tied lm_head when head_split) and its Pipeline.  n_labels > 0: the last stage is a sequence-classification
    tail (BS_FLAG_CLASSIFIER; `classify` runs the task) and there is no head ring.  Collective: every rank must
    call it."""
    if n_labels and head_split:
        raise ValueError("a classifier tail holds its own score head: no vocabulary-parallel head ring")
    head_split = (world > 1 and not n_labels) if head_split is None else (head_split and world > 1)
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
                   is_last=is_last and not head_split, head_slice=hslice, int8_weights=model.int8_weights,
                   n_labels=n_labels if is_last else 0)
        ex = StageExecutor(st)
    else:
        kw = {"n_labels": n_labels} if (n_labels and is_last) else {}
        ex = executor_factory(lb, le, is_first, is_last and not head_split, mb_rows * n_mb, max_ctx, hslice, **kw)
    # communicators are created collectively, in the same order on every rank
    tok_group = head_group = pf_group = None
    if world > 1:
        tok_group = dist.new_group(ranks=list(range(world)))
        head_group = dist.new_group(ranks=list(range(world)))
        pf_group = dist.new_group(ranks=list(range(world)))
        connect_p2p(rank, world, head_split, {"hidden": None, "head": head_group, "tok": tok_group, "pf": pf_group},
                    device)
    act = torch.bfloat16 if dtype == "bf16" else torch.float32
    pipe = Pipeline(ex, rank=rank, world=world, hidden=model.hidden, mb_rows=mb_rows, n_mb=n_mb, device=device,
                    is_first=is_first, is_last=is_last, tok_group=tok_group, head_group=head_group,
                    head_split=head_split, act_dtype=act, max_seq=max_seq, pf_group=pf_group)
    return pipe, (lb, le)
