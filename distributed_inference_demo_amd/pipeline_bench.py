"""Pipeline measurements: bench.py's N-GPU line and its BASELINE.json configs[3] / configs[4] records.

One process per GPU (torchrun or bench.py's own launcher), rank r = stage r of the server's round-robin
layer assignment (server.py:893-905), hidden states over RCCL send/recv (pipeline.Pipeline).  Every
measurement here is collective: every rank calls it with the same arguments, rank 0 gets the record.

Records (all built by `run_pipeline`, the same code at every N):
  weak     : the line's `value` -- 2N micro-batches of `batch` rows of args.model (per-GPU layer-forwards
             per round fixed at 2 x n_layer, so the ideal curve is N x the N = 1 point)
  strong   : 16 x batch rows in flight at every N (2N micro-batches); the rows actually run are reported
  configs3 : BASELINE.json configs[3] -- bloom-7b1, B = 8 as 8 micro-batches of one row, 512-token prefill
             streamed through the stages (per-stage busy fraction vs the ideal fill-and-drain overlap),
             then decode
  configs2 : BASELINE.json configs[2] -- bloom-3b on the server's uneven split at this N ([0,8) [8,16)
             [16,23) [23,30) at N = 4), B = 1 and B = 8, 64-token prompt, 128 decode rounds
  configs4 : BASELINE.json configs[4] -- bloom-7b1, B = 32 as 2N micro-batches, decode tokens/s and
             per-stage HBM at contexts 256 / 512 / 1024 / 2048 (a prefill to each context, then decode
             rounds ending at it)
  replicas : the alternative SURVEY §8(e) names (every config fits one MI355X): each rank runs the WHOLE
             model alone on its GPU with the same total rows / N (weak: 2 x batch rows per GPU; strong:
             16 x batch / N), no communication; the line reports the summed tokens/s, so the pipeline
             curve can be read against simply running more rows per GPU
The counterpart in the reference is the per-device loop of Communication.java:389-470 with
`core_pool_size` samples in flight and the hop of Communication.java:706-852.

The gloo backend (CPU tensors, a caller-supplied executor factory) runs the same schedule and bookkeeping
on the host: tests use it with the CPU checker as the stage (tests/bench_checker.py).
"""
import os
import sys
import time

import torch
import torch.distributed as dist

from . import config
from .pipeline import build_rank, init_distributed, vocab_slices
from .placement import stage_ranges

HBM_PEAK_GBPS = 8000.0      # MI355X HBM3E vendor peak
BF16_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA vendor peak


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _max_over_ranks(x, dev):
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _busy_ms(timing):
    """Sum of a stage's forward times this round: HIP event pairs (cuda) or host-clock pairs in ms (cpu)."""
    return sum((b - a) if isinstance(a, float) else a.elapsed_time(b) for a, b in timing)


def stage_step_bytes(model, lb, le, rows, ctx, first, last, hslice, w_bytes, kv_bytes):
    """Algorithmic HBM bytes of one decode forward of a stage (BASELINE.md formula) plus, with the
    vocabulary-parallel head, the stage's lm_head slice and ln_f."""
    b = config.decode_step_bytes(model, le - lb, rows, ctx, first, last, w_bytes=w_bytes, kv_bytes=kv_bytes)
    if hslice is not None:
        b += (hslice[1] - hslice[0]) * model.hidden * w_bytes + 2 * model.hidden * w_bytes
    if model.int8_weights:  # block matrices: 1 byte per weight + one fp32 scale per output row
        b -= (le - lb) * (12.0 * model.hidden * model.hidden * 1 - 9.0 * model.hidden * 4)
    return b


def _prompt(rows, P, vocab, dev):
    from .stage import prompt_ids
    return torch.from_numpy(prompt_ids(1234, rows, P, vocab)).to(dev)


def _progress(msg):
    """BS_PROGRESS=1: one stderr line per phase (long profiled runs show where they are)."""
    if os.environ.get("BS_PROGRESS") == "1":
        print(f"[pipeline_bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def run_pipeline(model, rank, world, dev, *, mb_rows, n_mb, head_split, prompts, steps, warmup, dtype="bf16",
                 seed=0, prof_rounds=0, executor_factory=None, replica=False):
    """Build this rank's stage + Pipeline once, then for each prompt length P in `prompts`: a timed P-token
    prefill round (every micro-batch streams through the stages; per-stage forward times), `warmup` and
    `steps` timed decode rounds (barrier + sync on both sides, max over ranks).  After the first point,
    `prof_rounds` eager decode rounds time every decode weight GEMV with HIP events (the per-stage
    roofline).  Rank 0 returns [one record per P], other ranks None.
    replica=True: every rank builds the WHOLE model as one stage on its own GPU (a world-1 pipeline, no
    communication on the data path) and runs n_mb x mb_rows rows of its own; the timing brackets (barrier +
    sync, max over ranks) are the same, and the record's value counts the rows of all ranks."""
    W, K = warmup, steps
    pmax = max(prompts)
    b_rank, b_world = (0, 1) if replica else (rank, world)
    _progress(f"{model.name}: build (mb_rows {mb_rows}, n_mb {n_mb}, prompts {list(prompts)})")
    pipe, (lb, le) = build_rank(model, b_rank, b_world, dev, dtype=dtype, mb_rows=mb_rows, n_mb=n_mb,
                                max_ctx=pmax + W + K + prof_rounds + 2, max_seq=pmax, seed=seed,
                                head_split=head_split and not replica, executor_factory=executor_factory)
    cuda = dev.type == "cuda"
    prev = torch.cuda.current_stream() if cuda else None
    if cuda:
        torch.cuda.set_stream(torch.cuda.Stream())  # a real stream: decode steps are captured as hipGraphs
    hslice = vocab_slices(model.vocab, world)[rank] if pipe.head_split else None
    last_head = pipe.is_last and not pipe.head_split
    w_b = 2 if dtype == "bf16" else 4
    st = pipe.ex.stage if hasattr(pipe.ex, "stage") else None
    out = []
    for i, P in enumerate(prompts):
        pipe.past = [0] * n_mb  # a new request per row: the prefill rewrites positions [0, P)
        prompt = _prompt(mb_rows * n_mb, P, model.vocab, dev) if pipe.is_first else None
        dist.barrier()
        _sync(dev)
        timing = []
        _progress(f"{model.name}: prefill {P}")
        t0 = time.perf_counter()
        pipe.step(P, prompt=prompt, timing=timing)
        _sync(dev)
        t_pre = _max_over_ranks(time.perf_counter() - t0, dev)  # the round's time: the slowest rank's
        busy_ms = _busy_ms(timing)
        for _ in range(W):
            pipe.step(1)
        _sync(dev)
        dist.barrier()
        _sync(dev)
        t0 = time.perf_counter()
        for _ in range(K):
            pipe.step(1)
        pipe.finish()
        _sync(dev)
        dist.barrier()
        dt = _max_over_ranks(time.perf_counter() - t0, dev)
        g = None
        if i == 0 and st is not None and prof_rounds:
            st.profile_enable(1)
            for _ in range(prof_rounds):
                pipe.step(1)
            pipe.finish()
            _sync(dev)
            g = st.profile_read()
            st.profile_enable(0)
            dist.barrier()
        ctx_mid = P + W + K / 2
        step_bytes = stage_step_bytes(model, lb, le, mb_rows, ctx_mid, pipe.is_first, last_head, hslice, w_b, w_b)
        pre_flops = config.prefill_flops(model, le - lb, mb_rows * n_mb, P, False)
        mine = {"rank": rank, "layers": [lb, le], "head_slice": list(hslice) if hslice else None,
                "algo_bytes_per_forward": step_bytes, "achieved_GBps": n_mb * step_bytes / (dt / K) / 1e9,
                "prefill": {"busy_ms": busy_ms, "busy_frac": busy_ms / (t_pre * 1e3),
                            "stage_TFLOPs": pre_flops / (busy_ms * 1e-3) / 1e12 if busy_ms > 0 else None}}
        mine["frac_of_peak"] = mine["achieved_GBps"] / HBM_PEAK_GBPS
        if g is not None and g[1]:
            ms, n, byts = g
            mine["gemv"] = {"launches": n, "avg_us": ms / n * 1e3, "achieved_GBps": (byts / n) / (ms / n * 1e-3) / 1e9}
        allst = [None] * world
        _progress(f"{model.name}: decode done, gathering the record")
        dist.all_gather_object(allst, mine)
        if rank == 0:
            out.append(_record(model, world, allst, mb_rows, n_mb, P, W, K, dt, t_pre,
                               head_split and world > 1 and not replica, replica))
    if cuda:
        torch.cuda.set_stream(prev)
    st_close = getattr(st, "close", None)
    del pipe
    if st_close:
        st_close()
    _progress(f"{model.name}: closed")
    return out if rank == 0 else None


def _record(model, world, allst, mb_rows, n_mb, P, W, K, dt, t_pre, vocab_ring, replica=False):
    rows = mb_rows * n_mb * (world if replica else 1)
    res = {"value": rows * K / dt, "unit": "tokens/s", "ms_per_step": dt * 1e3 / K, "rows": rows,
           "micro_batch": mb_rows, "n_mb": n_mb, "prompt": P, "decode_positions": [P + W, P + W + K],
           "head": "whole model per GPU" if replica else ("vocab-split ring" if vocab_ring else "last stage"),
           "per_stage": allst,
           "stage_hbm": {"achieved_GBps_min": min(x["achieved_GBps"] for x in allst),
                         "achieved_GBps_mean": sum(x["achieved_GBps"] for x in allst) / world,
                         "frac_of_peak_min": min(x["frac_of_peak"] for x in allst),
                         "frac_of_peak_mean": sum(x["frac_of_peak"] for x in allst) / world,
                         "note": "per stage: n_mb x algorithmic bytes of one forward / time of one pipeline round"}}
    tot_flops = config.prefill_flops(model, model.n_layer, rows, P, True)
    if replica:
        res["per_gpu_rows"] = mb_rows * n_mb
        res["prefill"] = {"tokens": rows * P, "ms": t_pre * 1e3, "tokens_per_s": rows * P / t_pre,
                          "achieved_TFLOPs": tot_flops / t_pre / 1e12,
                          "frac_of_peak": tot_flops / t_pre / 1e12 / BF16_PEAK_TFLOPS / world}
        return res
    res["prefill"] = {"tokens": rows * P, "ms": t_pre * 1e3, "tokens_per_s": rows * P / t_pre,
                      "achieved_TFLOPs": tot_flops / t_pre / 1e12,
                      "frac_of_peak": tot_flops / t_pre / 1e12 / BF16_PEAK_TFLOPS,
                      "stage_busy_frac": [x["prefill"]["busy_frac"] for x in allst],
                      "ideal_busy_frac": n_mb / (n_mb + world - 1),
                      "note": "busy = sum of a stage's forward times / the prefill round's wall time (max over "
                              "ranks); ideal = n_mb / (n_mb + stages - 1) for a perfectly overlapped fill-and-drain"}
    gemv = [x["gemv"] for x in allst if "gemv" in x]
    if gemv:
        tot_t = sum(x["launches"] * x["avg_us"] for x in gemv)
        tot_b = sum(x["launches"] * x["avg_us"] * 1e-6 * x["achieved_GBps"] * 1e9 for x in gemv)
        ach = tot_b / (tot_t * 1e-6) / 1e9
        res["roofline"] = {"bound": "hbm", "kernel": "decode weight GEMVs of every stage (gemv_rows_kernel, "
                                                     "gemv_ldsw4_kernel)",
                           "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBPS,
                           "traffic": None,
                           "traffic_note": "PMC passes need one rocprofv3 process per rank; collected at N = 1 only",
                           "launches": sum(x["launches"] for x in gemv),
                           "avg_us": tot_t / sum(x["launches"] for x in gemv),
                           "measured": "HIP events per launch on each stage's stream, eager pipeline rounds after "
                                       "the timed region; bytes and time summed over all stages"}
    return res


def _parse_ctx(s):
    return [int(v) for v in str(s).split(",") if v.strip()]


def configs4_prompts(ctxs, warmup, steps):
    """configs[4]: each context c is reached by a (c - warmup - steps)-token prefill and warmup + steps decode
    rounds.  Contexts that leave no prompt token are skipped (and named in the record), not run."""
    keep = [c for c in ctxs if c - warmup - steps >= 1]
    return keep, [c for c in ctxs if c not in keep], [c - warmup - steps for c in keep]


def configs2_split(rows, world):
    """configs[2]: `rows` rows as n_mb micro-batches of rows / n_mb, n_mb = the largest divisor of `rows` that is
    at most 2N (the micro-batches the other records keep in flight), so every N runs exactly `rows` rows."""
    n_mb = max(d for d in range(1, min(2 * world, rows) + 1) if rows % d == 0)
    return rows // n_mb, n_mb


def bench_pipeline(args, backend="nccl", executor_factory=None):
    """bench.py at N ranks (and its N = 1 reference point): the model split into N stages.  `value` is the
    weak line; `strong`, `configs2`, `configs3`, `configs4` and `replicas` ride along (skipped by --no-strong /
    --no-configs / --no-replicas).
    `executor_factory(model, dtype, seed)` (gloo tests) returns build_rank's per-stage executor factory.
    Rank 0 returns (line dict, stage ranges, model); other ranks (None, ranges, model)."""
    rank, world, local = init_distributed(backend)
    if world != args.gpus:
        raise RuntimeError(f"bench.py --gpus {args.gpus} but the process group has {world} ranks")
    dev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")
    model = config.get(args.model)
    if getattr(args, "weights", "bf16") == "int8":
        model = config.get(model.name if model.int8_weights else model.name + "-int8")
    prof_rounds = 0 if getattr(args, "no_profile", False) else 8
    head_split = not getattr(args, "no_head_split", False)
    dtype, seed = args.dtype, args.seed

    def factory(m):
        return None if executor_factory is None else executor_factory(m, dtype, seed)

    n_mb = 2 * world
    common = dict(head_split=head_split, steps=args.steps, warmup=args.warmup, dtype=dtype, seed=seed)
    (weak,) = run_pipeline(model, rank, world, dev, mb_rows=args.batch, n_mb=n_mb, prompts=[args.prompt],
                           prof_rounds=prof_rounds, executor_factory=factory(model), **common) or [None]
    strong = None
    if not getattr(args, "no_strong", False):
        want = 16 * args.batch
        mb = -(-want // n_mb)  # rows actually run: mb x n_mb (== want whenever 2N divides 16 x batch)
        r = run_pipeline(model, rank, world, dev, mb_rows=mb, n_mb=n_mb, prompts=[args.prompt],
                         executor_factory=factory(model), **common)
        if r:
            strong = dict(r[0], definition=f"{mb * n_mb} rows in flight ({n_mb} micro-batches of {mb}); the target "
                                           f"is 16 x batch = {want} rows at every N"
                                           + ("" if mb * n_mb == want else f" -- {want} rows do not split "
                                              f"evenly over {n_mb} micro-batches, so this N runs {mb * n_mb}"))
    c2 = c3 = c4 = None
    if not getattr(args, "no_configs", False):
        m2 = config.get(getattr(args, "configs2_model", "bloom-3b"))
        c2 = {}
        for b2 in _parse_ctx(getattr(args, "configs2_batch", "1,8")):
            mb2, nmb2 = configs2_split(b2, world)
            r = run_pipeline(m2, rank, world, dev, mb_rows=mb2, n_mb=nmb2, prompts=[getattr(args, "configs2_prompt", 64)],
                             executor_factory=factory(m2), head_split=head_split,
                             steps=getattr(args, "configs2_steps", 128), warmup=args.warmup, dtype=dtype, seed=seed)
            if rank == 0:
                c2[f"B{b2}"] = {k: r[0][k] for k in ("value", "ms_per_step", "rows", "micro_batch", "n_mb", "prompt",
                                                     "decode_positions", "head", "stage_hbm", "per_stage", "prefill")}
        cm = config.get(getattr(args, "configs_model", "bloom-7b1"))
        c3r = run_pipeline(cm, rank, world, dev, mb_rows=1, n_mb=getattr(args, "configs3_mb", 8),
                           prompts=[getattr(args, "configs3_prompt", 512)], executor_factory=factory(cm), **common)
        rows4 = getattr(args, "configs4_rows", 32)
        mb4 = -(-rows4 // n_mb)
        ctxs, skipped4, p4 = configs4_prompts(_parse_ctx(getattr(args, "configs4_ctx", "256,512,1024,2048")),
                                              args.warmup, args.steps)
        c4r = run_pipeline(cm, rank, world, dev, mb_rows=mb4, n_mb=n_mb, prompts=p4, executor_factory=factory(cm),
                           **common) if p4 else []
        if rank == 0:
            c2 = {"workload": f"BASELINE.json configs[2]: {m2.name} split into {world} stages by the server's "
                              f"round-robin assignment {stage_ranges(world, m2.n_layer)}, B = 1 and B = 8 "
                              f"(n_mb = the largest divisor of B <= 2N), {getattr(args, 'configs2_prompt', 64)}-token prompt, "
                              f"{getattr(args, 'configs2_steps', 128)} timed decode rounds", **c2}
            c3 = dict(c3r[0], workload=f"BASELINE.json configs[3]: {cm.name}, {world} stages, B = {c3r[0]['rows']} as "
                                       f"{c3r[0]['n_mb']} micro-batches of 1 row, {c3r[0]['prompt']}-token prefill "
                                       "streamed through the stages, then decode")
            c4 = {"workload": f"BASELINE.json configs[4]: {cm.name} B = {mb4 * n_mb} decode ({n_mb} micro-batches "
                              f"of {mb4}), {world} stages, tokens/s at each context (a prefill, then decode "
                              "rounds ending at the context)",
                  "by_ctx": {str(c): {k: r[k] for k in ("value", "ms_per_step", "rows", "decode_positions",
                                                        "stage_hbm", "per_stage", "prefill")}
                             for c, r in zip(ctxs, c4r or [])}}
            if skipped4:
                c4["skipped_ctx"] = {"ctx": skipped4, "why": f"context <= warmup + steps = {args.warmup + args.steps}: "
                                                              "no prompt token left for the prefill"}
    rep = None
    if not getattr(args, "no_replicas", False):
        rep = {}
        want = 16 * args.batch
        for name, rows in (("weak", 2 * args.batch), ("strong", max(1, -(-want // world)))):
            mbr, nmbr = -(-rows // 2) if rows > 1 else 1, 2 if rows > 1 else 1
            r = run_pipeline(model, rank, world, dev, mb_rows=mbr, n_mb=nmbr, prompts=[args.prompt],
                             executor_factory=factory(model), replica=True, **common)
            if rank == 0:
                rep[name] = {k: r[0][k] for k in ("value", "ms_per_step", "rows", "per_gpu_rows", "micro_batch", "n_mb",
                                                  "stage_hbm", "prefill")}
    dist.barrier()
    dist.destroy_process_group()
    ranges = stage_ranges(world, model.n_layer)
    if rank != 0:
        return None, ranges, model
    per_stage = [b - a for a, b in ranges]
    res = {
        "metric": "decode tokens/s, BLOOM pipeline", "value": weak["value"], "unit": "tokens/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": weak["ms_per_step"], "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": dtype,
        "data": "synthetic: repo-generator random-init weights (seed %d), prompt ids U[0,V) seed 1234" % seed,
        "config": {"workload": f"{model.name} split into {world} stages by the server's round-robin layer "
                               f"assignment, {n_mb} micro-batches x {args.batch} rows in flight, "
                               + ("RCCL send/recv" if backend == "nccl" else f"{backend} send/recv")
                               + (", vocabulary-parallel lm_head ring" if weak["head"] == "vocab-split ring" else ""),
                   "model": model.name, "stages": world, "layers_per_stage": per_stage, "batch": weak["rows"],
                   "micro_batch": args.batch, "prompt": args.prompt, "parallelism": f"pp{world}",
                   "head": weak["head"],
                   "hop": "fp32 hidden [mb, S, h] (the reference wire dtype; keeps the split bit-identical to one stage)"},
        "weak_definition": "2N micro-batches x batch rows: per-GPU layer-forwards per round fixed at 2 x n_layer, "
                           "so the ideal value at N is N x the N = 1 point",
        "scaling_ref": {"n1_point": "pipeline_n1 of the N = 1 line (this same code on an RCCL world-1 group: 2 "
                                    "micro-batches of `batch` rows); the N = 1 line's own `value` is the single-stage "
                                    "configs[1] bench, one row, within 1-2 % of it",
                        "weak_value": weak["value"], "weak_rows": weak["rows"],
                        "strong_value": strong["value"] if strong else None,
                        "strong_rows": strong["rows"] if strong else None,
                        "replicas_weak_value": rep["weak"]["value"] if rep else None,
                        "replicas_strong_value": rep["strong"]["value"] if rep else None,
                        "note": "equal work: `strong` (fixed 16 x batch rows) and `replicas_*` (the whole model on "
                                "every GPU, same total rows) are the lines to compare across N; `value` (weak) "
                                "grows its rows with N"},
        "per_stage": weak["per_stage"], "stage_hbm": weak["stage_hbm"], "prefill": weak["prefill"],
    }
    if "roofline" in weak:
        res["roofline"] = weak["roofline"]
    if strong is not None:
        res["strong"] = {k: strong[k] for k in ("value", "ms_per_step", "rows", "micro_batch", "n_mb", "stage_hbm",
                                                "prefill", "definition")}
    if c3 is not None:
        res["configs2"] = c2
        res["configs3"] = c3
        res["configs4"] = c4
    if rep is not None:
        res["replicas"] = dict(rep, definition="every GPU runs the whole model as one stage, no communication, "
                                               "n_mb = 2 micro-batches of the per-GPU rows; value = all rows of all "
                                               "GPUs x steps / the slowest GPU's time (SURVEY §8(e) alternative)")
    return res, ranges, model
