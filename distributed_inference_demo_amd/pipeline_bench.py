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
  configs4 : BASELINE.json configs[4] -- bloom-7b1, B = 32 as 2N micro-batches, decode tokens/s and
             per-stage HBM at contexts 256 / 512 / 1024 / 2048 (a prefill to each context, then decode
             rounds ending at it)
The counterpart in the reference is the per-device loop of Communication.java:389-470 with
`core_pool_size` samples in flight and the hop of Communication.java:706-852.

The gloo backend (CPU tensors, a caller-supplied executor factory) runs the same schedule and bookkeeping
on the host: tests use it with the CPU checker as the stage (tests/bench_checker.py).
"""
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


def run_pipeline(model, rank, world, dev, *, mb_rows, n_mb, head_split, prompts, steps, warmup, dtype="bf16",
                 seed=0, prof_rounds=0, executor_factory=None):
    """Build this rank's stage + Pipeline once, then for each prompt length P in `prompts`: a timed P-token
    prefill round (every micro-batch streams through the stages; per-stage forward times), `warmup` and
    `steps` timed decode rounds (barrier + sync on both sides, max over ranks).  After the first point,
    `prof_rounds` eager decode rounds time every decode weight GEMV with HIP events (the per-stage
    roofline).  Rank 0 returns [one record per P], other ranks None."""
    W, K = warmup, steps
    pmax = max(prompts)
    pipe, (lb, le) = build_rank(model, rank, world, dev, dtype=dtype, mb_rows=mb_rows, n_mb=n_mb,
                                max_ctx=pmax + W + K + prof_rounds + 2, max_seq=pmax, seed=seed,
                                head_split=head_split, executor_factory=executor_factory)
    cuda = dev.type == "cuda"
    prev = torch.cuda.current_stream() if cuda else None
    if cuda:
        torch.cuda.set_stream(torch.cuda.Stream())  # a real stream: decode steps are captured as hipGraphs
    hslice = vocab_slices(model.vocab, world)[rank] if pipe.head_split else None
    last_head = rank == world - 1 and not pipe.head_split
    w_b = 2 if dtype == "bf16" else 4
    st = pipe.ex.stage if hasattr(pipe.ex, "stage") else None
    out = []
    for i, P in enumerate(prompts):
        pipe.past = [0] * n_mb  # a new request per row: the prefill rewrites positions [0, P)
        prompt = _prompt(mb_rows * n_mb, P, model.vocab, dev) if rank == 0 else None
        dist.barrier()
        _sync(dev)
        timing = []
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
        step_bytes = stage_step_bytes(model, lb, le, mb_rows, ctx_mid, rank == 0, last_head, hslice, w_b, w_b)
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
        dist.all_gather_object(allst, mine)
        if rank == 0:
            out.append(_record(model, world, allst, mb_rows, n_mb, P, W, K, dt, t_pre, head_split and world > 1))
    if cuda:
        torch.cuda.set_stream(prev)
    st_close = getattr(st, "close", None)
    del pipe
    if st_close:
        st_close()
    return out if rank == 0 else None


def _record(model, world, allst, mb_rows, n_mb, P, W, K, dt, t_pre, vocab_ring):
    rows = mb_rows * n_mb
    res = {"value": rows * K / dt, "unit": "tokens/s", "ms_per_step": dt * 1e3 / K, "rows": rows,
           "micro_batch": mb_rows, "n_mb": n_mb, "prompt": P, "decode_positions": [P + W, P + W + K],
           "head": "vocab-split ring" if vocab_ring else "last stage", "per_stage": allst,
           "stage_hbm": {"achieved_GBps_min": min(x["achieved_GBps"] for x in allst),
                         "achieved_GBps_mean": sum(x["achieved_GBps"] for x in allst) / world,
                         "frac_of_peak_min": min(x["frac_of_peak"] for x in allst),
                         "frac_of_peak_mean": sum(x["frac_of_peak"] for x in allst) / world,
                         "note": "per stage: n_mb x algorithmic bytes of one forward / time of one pipeline round"}}
    tot_flops = config.prefill_flops(model, model.n_layer, rows, P, True)
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


def bench_pipeline(args, backend="nccl", executor_factory=None):
    """bench.py at N ranks (and its N = 1 reference point): the model split into N stages.  `value` is the
    weak line; `strong`, `configs3` and `configs4` ride along (skipped by --no-strong / --no-configs).
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
    c3 = c4 = None
    if not getattr(args, "no_configs", False):
        cm = config.get(getattr(args, "configs_model", "bloom-7b1"))
        c3r = run_pipeline(cm, rank, world, dev, mb_rows=1, n_mb=getattr(args, "configs3_mb", 8),
                           prompts=[getattr(args, "configs3_prompt", 512)], executor_factory=factory(cm), **common)
        rows4 = getattr(args, "configs4_rows", 32)
        mb4 = -(-rows4 // n_mb)
        ctxs = _parse_ctx(getattr(args, "configs4_ctx", "256,512,1024,2048"))
        c4r = run_pipeline(cm, rank, world, dev, mb_rows=mb4, n_mb=n_mb,
                           prompts=[c - args.warmup - args.steps for c in ctxs], executor_factory=factory(cm),
                           **common)
        if rank == 0:
            c3 = dict(c3r[0], workload=f"BASELINE.json configs[3]: {cm.name}, {world} stages, B = {c3r[0]['rows']} as "
                                       f"{c3r[0]['n_mb']} micro-batches of 1 row, {c3r[0]['prompt']}-token prefill "
                                       "streamed through the stages, then decode")
            c4 = {"workload": f"BASELINE.json configs[4]: {cm.name} B = {mb4 * n_mb} decode ({n_mb} micro-batches "
                              f"of {mb4}), {world} stages, tokens/s at each context (a prefill, then decode "
                              "rounds ending at the context)",
                  "by_ctx": {str(c): {k: r[k] for k in ("value", "ms_per_step", "rows", "decode_positions",
                                                        "stage_hbm", "per_stage", "prefill")}
                             for c, r in zip(ctxs, c4r)}}
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
                                    "configs[1] bench, one row, within 1-2 % of it"},
        "per_stage": weak["per_stage"], "stage_hbm": weak["stage_hbm"], "prefill": weak["prefill"],
    }
    if "roofline" in weak:
        res["roofline"] = weak["roofline"]
    if strong is not None:
        res["strong"] = {k: strong[k] for k in ("value", "ms_per_step", "rows", "micro_batch", "n_mb", "stage_hbm",
                                                "prefill", "definition")}
    if c3 is not None:
        res["configs3"] = c3
        res["configs4"] = c4
    return res, ranges, model
