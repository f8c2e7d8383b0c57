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
           samples in flight = min(pool, stages) micro-batches x the rest as rows (each sample
           owns a KV slot), so every stage computes while the hops overlap;
  run    — samples in waves of the pool: one prompt prefill round, then max_length - 1
           decode rounds, all micro-batches in flight through the stages (a short last wave is
           padded with copies of its last sample, whose outputs are dropped);
  finish — rank 0 returns every sample's `max_length` greedy token ids and the run's tokens/s.
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
    max_length: int = 40          # tokens generated per sample
    core_pool_size: int = 1       # samples in flight
    prompt_len: int = 16          # synthetic prompts (token ids U[0, V), seed 1234 + sample id)
    dtype: str = "bf16"
    seed: int = 0                 # weight generator seed
    head_split: bool = True       # vocabulary-parallel lm_head ring when world > 1


def synthetic_prompts(cfg: RunConfig, vocab):
    from .stage import prompt_ids
    return [prompt_ids(1234 + i, 1, cfg.prompt_len, vocab).reshape(-1).tolist() for i in range(cfg.num_sample)]


def run_rank(cfg: RunConfig, rank, world, device, prompts=None, executor_factory=None, log=None):
    """Run the whole job on this rank.  `prompts` (rank 0): num_sample lists of token ids, all of
    one length (None: synthetic).  Returns {"samples": [[max_length ids] per sample], ...} on
    rank 0, None elsewhere.  Collective: every rank calls it with the same cfg."""
    say = log if (log is not None and rank == 0) else (lambda *_: None)
    if cfg.num_sample < 1 or cfg.max_length < 1 or cfg.core_pool_size < 1:
        raise ValueError("num_sample, max_length and core_pool_size must be >= 1")
    model = config.get(cfg.model) if isinstance(cfg.model, str) else cfg.model
    if rank == 0:
        prompts = synthetic_prompts(cfg, model.vocab) if prompts is None else [list(p) for p in prompts]
        if len(prompts) != cfg.num_sample:
            raise ValueError(f"{len(prompts)} prompts for num_sample = {cfg.num_sample}")
        lens = {len(p) for p in prompts}
        if len(lens) != 1:
            raise ValueError("all prompts of a run must have one length (no padding masks on this path)")
        plen = lens.pop()
    else:
        plen = cfg.prompt_len
    if world > 1:  # the prompt length travels with the config (server -> devices)
        t = torch.tensor([plen], dtype=torch.int64)
        if dist.get_backend() == "nccl":
            t = t.to(device)
        dist.broadcast(t, src=0)
        plen = int(t.item())
    # samples in flight = n_mb micro-batches x mb rows: one micro-batch per stage keeps every stage
    # busy; the rest of the pool rides as rows of a micro-batch (one GPU: one batched decode)
    n_mb = min(cfg.core_pool_size, world)
    mb = -(-cfg.core_pool_size // n_mb)
    pool = n_mb * mb
    # ---- init (Ready)
    pipe, (lb, le) = build_rank(model, rank, world, device, dtype=cfg.dtype, mb_rows=mb, n_mb=n_mb,
                                max_ctx=plen + cfg.max_length + 1, max_seq=plen, seed=cfg.seed,
                                head_split=cfg.head_split, executor_factory=executor_factory)
    say(STATES[0], {"rank_layers": [lb, le], "stages": world, "core_pool_size": cfg.core_pool_size,
                    "micro_batches": n_mb, "rows_per_micro_batch": mb})
    cuda = device.type == "cuda"
    if cuda:
        torch.cuda.set_stream(torch.cuda.Stream(device))  # decode steps are captured as hipGraphs
    if world > 1:
        dist.barrier()
    # ---- run (Running)
    say(STATES[1], {"num_sample": cfg.num_sample, "max_length": cfg.max_length})
    out = []
    t0 = time.perf_counter()
    for w0 in range(0, cfg.num_sample, pool):
        prompt = None
        if rank == 0:
            wave = prompts[w0:w0 + pool]
            wave = wave + [wave[-1]] * (pool - len(wave))  # pad a short last wave
            prompt = torch.tensor(wave, dtype=torch.int32, device=device)
        pipe.past = [0] * n_mb  # each micro-batch's slot starts a new sample
        rec = [[] for _ in range(n_mb)] if pipe.is_first else None
        pipe.step(plen, prompt=prompt, record=rec)
        for _ in range(cfg.max_length - 1):
            pipe.step(1, record=rec)
        pipe.finish(record=rec)
        if rank == 0:
            ids = torch.cat([torch.stack(r, 1) for r in rec], 0).cpu()
            out.extend(ids[: min(pool, cfg.num_sample - w0)].tolist())
    if cuda:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # ---- finish (Finish, Close)
    if world > 1:
        dist.barrier()
    if rank != 0:
        return None
    res = {"samples": out, "num_sample": cfg.num_sample, "max_length": cfg.max_length,
           "core_pool_size": cfg.core_pool_size, "stages": world, "prompt_len": plen, "seconds": dt,
           "tokens_per_s": cfg.num_sample * cfg.max_length / dt}
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
