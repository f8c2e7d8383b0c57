"""serve.py — the reference's server/client run on one node.

Reference: `server.py:893-1042` builds the run config {num_sample, max_length, core_pool_size,
num_device, graph, ...}, places contiguous layer ranges with `round_robin_module_arrangement`
(`server.py:893-905`) and drives every device through Ready -> Running -> Finish -> Close
(`Client.java:50-173`); on each device `Communication.running` (`Communication.java:389-470`) keeps
`core_pool_size` samples in flight until `num_sample` samples are done, and every sample produces
`max_length` tokens, one pipeline round each (`Communication.java:621-651`).

Here: one process per GPU (torchrun), rank r = device r of the graph, layers from the same
placement (`placement.stage_ranges`).  Lifecycle:
  init   — RunConfig -> this rank's stage + Pipeline (`pipeline.build_rank`); the `core_pool_size`
           samples in flight = min(pool, stages) micro-batches x the rest as rows, every row a KV slot
           holding one sample at its own position (bs_step.past_lens), so every stage computes while
           the hops overlap;
  run    — continuous admission (Communication.java:418-464: a new sample starts as soon as one in
           flight finishes): a row takes the next sample the round its previous sample produced its
           `max_length`-th token.  The admitted sample's whole prompt goes through the stages as one
           prefill pass of that row (S = len(prompt) at its KV slot, Pipeline.prefill_row) just before
           the decode round, which it joins with its first generated token; decode rounds are S = 1 for
           every row, each at its own position.  (prefill=False feeds the prompt one token a round, as
           the reference header does, Communication.java:322-326.)  Prompts may have different lengths.
           The admission schedule depends only on the prompt lengths, so every rank derives the same
           per-row positions and prefill passes;
  finish — rank 0 returns every sample's `max_length` greedy token ids and the run's tokens/s.
max_length == 0 is the classification task (Communication.java:591-603: one OneStep pass per sample, the
last device's classifier tail, binaryClassify at Communication.java:532-534): the last stage holds a
score head of `n_labels` labels (BS_FLAG_CLASSIFIER), samples of equal prompt length go through
together, `core_pool_size` rows a pass, and rank 0 returns each sample's class id (first maximal label).
Differences from the reference, by design: full-context decode (the reference
header feeds only the last token), argmax instead of unseeded top-k, token ids in (no tokenizer).

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \\
      -m distributed_inference_demo_amd.serve --model bloom-560m --num-sample 8 --max-length 40 \\
      --core-pool-size 2
"""
import argparse
import dataclasses
import json
import os
import sys
import time

import torch
import torch.distributed as dist

from . import config
from .pipeline import build_rank, init_distributed

STATES = ("Ready", "Running", "Finish", "Close")  # Client.java status strings, in order


@dataclasses.dataclass
class RunConfig:
    """The run config of server.py:998-1013 that shapes the computation."""
    model: str = "bloom-560m"
    num_sample: int = 8
    max_length: int = 40          # tokens generated per sample; 0 = the classification task
    core_pool_size: int = 1       # samples in flight
    n_labels: int = 2             # classification: score-head labels (the reference's binary classifier)
    prompt_len: int = 16          # synthetic prompts (token ids U[0, V), seed 1234 + sample id)
    dtype: str = "bf16"
    seed: int = 0                 # weight generator seed
    head_split: bool = True       # vocabulary-parallel lm_head ring when world > 1
    prefill: bool = True          # an admitted sample's prompt as one prefill pass of its row (else a token a round)


def synthetic_prompts(cfg: RunConfig, vocab):
    from .stage import prompt_ids
    return [prompt_ids(1234 + i, 1, cfg.prompt_len, vocab).reshape(-1).tolist() for i in range(cfg.num_sample)]


def admission_schedule(lens, max_length, rows, prefill=True):
    """Row-level continuous admission: sample i (in order) takes the row that frees first (lowest row
    on ties) at the round it frees.
      prefill=True : the sample's whole prompt is one prefill pass of that row just before decode round t0
                     (Pipeline.prefill_row; it yields generated token 1), then it decodes max_length - 1 rounds
                     (tokens 2..max_length); the row frees at t0 + max_length - 1.
      prefill=False: the prompt is fed one token a round (the reference header's single-token feed), so the
                     row is held len(prompt) - 1 + max_length rounds.
    Returns ([(row, t0)] per sample, total decode rounds)."""
    import heapq
    free = [(0, r) for r in range(rows)]
    heapq.heapify(free)
    out = []
    hold = (lambda n: max_length - 1) if prefill else (lambda n: n - 1 + max_length)
    for n in lens:
        t, r = heapq.heappop(free)
        out.append((r, t))
        heapq.heappush(free, (t + hold(n), r))
    return out, max(t + hold(n) for (r, t), n in zip(out, lens))


def run_rank(cfg: RunConfig, rank, world, device, prompts=None, executor_factory=None, log=None):
    """Run the whole job on this rank.  `prompts` (rank 0): num_sample lists of token ids of any
    lengths (None: synthetic).  Returns {"samples": [[max_length ids] per sample], ...} on rank 0,
    None elsewhere.  Collective: every rank calls it with the same cfg."""
    say = log if (log is not None and rank == 0) else (lambda *_: None)
    if cfg.num_sample < 1 or cfg.max_length < 0 or cfg.core_pool_size < 1:
        raise ValueError("num_sample and core_pool_size must be >= 1, max_length >= 0 (0: classification)")
    model = config.get(cfg.model) if isinstance(cfg.model, str) else cfg.model
    if rank == 0:
        prompts = synthetic_prompts(cfg, model.vocab) if prompts is None else [list(p) for p in prompts]
        if len(prompts) != cfg.num_sample:
            raise ValueError(f"{len(prompts)} prompts for num_sample = {cfg.num_sample}")
        if any(len(p) < 1 for p in prompts):
            raise ValueError("every prompt needs at least one token")
        lens = [len(p) for p in prompts]
    else:
        lens = [0] * cfg.num_sample
    if world > 1:  # the prompt lengths travel with the config (server -> devices)
        t = torch.tensor(lens, dtype=torch.int64)
        if dist.get_backend() == "nccl":
            t = t.to(device)
        dist.broadcast(t, src=0)
        lens = [int(v) for v in t.tolist()]
    if cfg.max_length == 0:
        return _classify_run(cfg, model, rank, world, device, prompts, lens, executor_factory, say)
    # samples in flight = n_mb micro-batches x mb rows: one micro-batch per stage keeps every stage
    # busy; the rest of the pool rides as rows of a micro-batch (one GPU: one batched decode)
    n_mb = min(cfg.core_pool_size, world)
    mb = -(-cfg.core_pool_size // n_mb)
    rows = n_mb * mb
    pf = cfg.prefill
    sched, T = admission_schedule(lens, cfg.max_length, rows, prefill=pf)
    # per decode round and row: position, and (rank 0) the fed token / whether it overrides the returned one;
    # with prefill, `take_pf` marks a sample's first decode round, whose input is its prefill's token
    pos = [[0] * rows for _ in range(T)]
    feed_tok = [[0] * rows for _ in range(T)]
    feed_mask = [[True] * rows for _ in range(T)]
    take_pf = [[False] * rows for _ in range(T)]
    admit = [[] for _ in range(T + 1)]  # prefill passes before decode round t: (sample, row)
    for i, ((r, t0), n) in enumerate(zip(sched, lens)):
        if pf:
            admit[t0].append((i, r))
            for t in range(t0, t0 + cfg.max_length - 1):
                pos[t][r] = n + (t - t0)
                feed_mask[t][r] = t == t0
                take_pf[t][r] = t == t0
        else:
            for t in range(t0, t0 + n - 1 + cfg.max_length):
                pos[t][r] = t - t0
                if t - t0 < n:
                    feed_tok[t][r] = prompts[i][t - t0] if rank == 0 else 0
                else:
                    feed_mask[t][r] = False
    # ---- init (Ready)
    max_seq = -(-max(lens) // mb) if pf else 1  # a prefill pass of one row fits a micro-batch's hop buffers
    pipe, (lb, le) = build_rank(model, rank, world, device, dtype=cfg.dtype, mb_rows=mb, n_mb=n_mb,
                                max_ctx=max(lens) + cfg.max_length + 1, max_seq=max_seq, seed=cfg.seed,
                                head_split=cfg.head_split, executor_factory=executor_factory)
    say(STATES[0], {"rank_layers": [lb, le], "stages": world, "core_pool_size": cfg.core_pool_size,
                    "micro_batches": n_mb, "rows_per_micro_batch": mb, "rounds": T, "prefill": pf})
    cuda = device.type == "cuda"
    if cuda:
        torch.cuda.set_stream(torch.cuda.Stream(device))  # decode steps are captured as hipGraphs
    shape = (max(T, 1), n_mb, mb)
    ft = torch.tensor(feed_tok or [[0] * rows], dtype=torch.int32, device=device).view(shape)
    fm = torch.tensor(feed_mask or [[True] * rows], dtype=torch.bool, device=device).view(shape)
    tp = torch.tensor(take_pf or [[False] * rows], dtype=torch.bool, device=device).view(shape)
    pids = ([torch.tensor(p, dtype=torch.int32, device=device).view(1, -1) for p in prompts]
            if (pf and rank == 0) else None)
    if world > 1:
        dist.barrier()
    # ---- run (Running)
    say(STATES[1], {"num_sample": cfg.num_sample, "max_length": cfg.max_length})
    rec = [[] for _ in range(n_mb)] if pipe.is_first else None
    first = [None] * cfg.num_sample  # prefill: each sample's first generated token (rank 0)
    pipe.tokens_held = True  # round 0 feeds every row
    t_start = time.perf_counter()
    for t in range(T + 1):
        for i, r in admit[t] if pf else ():
            tok = pipe.prefill_row(r // mb, r % mb, pids[i] if pids is not None else None, lens[i])
            if rank == 0:
                first[i] = tok.clone()
        if t == T:
            break
        pasts = [pos[t][j * mb:(j + 1) * mb] for j in range(n_mb)]
        feed = None
        if pipe.is_first:
            feed = [((torch.where(tp[t, j], pipe.pf_tok[j], ft[t, j]) if pf else ft[t, j]), fm[t, j])
                    for j in range(n_mb)]
        pipe.step(1, record=rec, feed=feed, pasts=pasts)
    if T:
        pipe.finish(record=rec)
    if cuda:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t_start
    # ---- finish (Finish, Close)
    if world > 1:
        dist.barrier()
    if rank != 0:
        return None
    y = torch.stack([torch.stack(r, 0) for r in rec], 1).view(T, rows).cpu() if T else None  # round t's tokens
    if pf:
        out = [[int(first[i].item())] + (y[t0:t0 + cfg.max_length - 1, r].tolist() if T else [])
               for i, (r, t0) in enumerate(sched)]
    else:
        out = [y[t0 + n - 1:t0 + n - 1 + cfg.max_length, r].tolist() for (r, t0), n in zip(sched, lens)]
    res = {"samples": out, "num_sample": cfg.num_sample, "max_length": cfg.max_length,
           "core_pool_size": cfg.core_pool_size, "stages": world, "prompt_lens": lens, "rounds": T,
           "prefill": pf, "seconds": dt, "tokens_per_s": cfg.num_sample * cfg.max_length / dt}
    say(STATES[2], {k: v for k, v in res.items() if k != "samples"})
    say(STATES[3], {})
    return res


def classify_batches(lens, rows):
    """The classification passes: samples grouped by prompt length (a pass is one prompt length for every
    row, Pipeline.step), in sample order within a group, `rows` samples a pass.  Returns [(length, [sample
    ids])]; a short last pass of a group is padded by the caller."""
    groups = {}
    for i, n in enumerate(lens):
        groups.setdefault(n, []).append(i)
    return [(n, ids[k:k + rows]) for n, ids in groups.items() for k in range(0, len(ids), rows)]


def _classify_run(cfg, model, rank, world, device, prompts, lens, executor_factory, say):
    """max_length == 0 (Communication.java:591-603): every sample is one pass through the stages from empty KV
    rows; the last stage's classifier tail returns its class id."""
    from .pipeline import classify
    if cfg.n_labels < 1:
        raise ValueError("classification needs n_labels >= 1")
    n_mb = min(cfg.core_pool_size, world)
    mb = -(-cfg.core_pool_size // n_mb)
    rows = n_mb * mb
    passes = classify_batches(lens, rows)
    pipe, (lb, le) = build_rank(model, rank, world, device, dtype=cfg.dtype, mb_rows=mb, n_mb=n_mb,
                                max_ctx=max(lens) + 1, max_seq=max(lens), seed=cfg.seed, head_split=False,
                                executor_factory=executor_factory, n_labels=cfg.n_labels)
    say(STATES[0], {"rank_layers": [lb, le], "stages": world, "core_pool_size": cfg.core_pool_size,
                    "micro_batches": n_mb, "rows_per_micro_batch": mb, "passes": len(passes),
                    "task": "classification", "n_labels": cfg.n_labels})
    cuda = device.type == "cuda"
    if cuda:
        torch.cuda.set_stream(torch.cuda.Stream(device))  # as the generation task (1-token prompts replay graphs)
    if world > 1:
        dist.barrier()
    say(STATES[1], {"num_sample": cfg.num_sample, "max_length": 0})
    out = [None] * cfg.num_sample
    t_start = time.perf_counter()
    for n, ids in passes:
        prompt = None
        if rank == 0:  # a short pass repeats its first sample in the spare rows (their classes are dropped)
            prompt = torch.tensor([prompts[i] for i in ids] + [prompts[ids[0]]] * (rows - len(ids)),
                                  dtype=torch.int32, device=device)
        cls = classify(pipe, prompt, n)
        if rank == 0:
            for i, c in zip(ids, cls.tolist()):
                out[i] = int(c)
    if cuda:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t_start
    if world > 1:
        dist.barrier()
    if rank != 0:
        return None
    res = {"samples": out, "task": "classification", "n_labels": cfg.n_labels, "num_sample": cfg.num_sample,
           "max_length": 0, "core_pool_size": cfg.core_pool_size, "stages": world, "prompt_lens": lens,
           "passes": len(passes), "seconds": dt, "samples_per_s": cfg.num_sample / dt}
    say(STATES[2], {k: v for k, v in res.items() if k != "samples"})
    say(STATES[3], {})
    return res


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    for f in dataclasses.fields(RunConfig):
        flag = "--" + f.name.replace("_", "-")
        if f.type is bool or f.type == "bool":
            p.add_argument(flag, type=int, default=int(f.default))
        else:
            p.add_argument(flag, type=type(f.default), default=f.default)
    p.add_argument("--prompts-file", default=None, help="JSON list of token-id lists (one per sample)")
    p.add_argument("--out", default=None, help="write the samples' token ids here (JSON)")
    a = p.parse_args(argv)
    cfg = RunConfig(**{f.name: (bool(getattr(a, f.name)) if f.type is bool or f.type == "bool"
                                else getattr(a, f.name)) for f in dataclasses.fields(RunConfig)})
    rank, world, local = init_distributed() if int(os.environ.get("WORLD_SIZE", "1")) > 1 else (0, 1, 0)
    device = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    prompts = json.load(open(a.prompts_file)) if (a.prompts_file and rank == 0) else None
    log = lambda state, info: print(json.dumps({"state": state, **info}), flush=True)  # noqa: E731
    res = run_rank(cfg, rank, world, device, prompts=prompts, log=log)
    if res is not None:
        if a.out:
            json.dump(res["samples"], open(a.out, "w"))
        print(json.dumps({k: v for k, v in res.items() if k != "samples"}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
