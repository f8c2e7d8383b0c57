"""bench.py — decode tokens/s of the BLOOM stage pipeline on MI355X (BASELINE.json metric).

N=1 (default): BASELINE.json configs[1] — bloom-1b1 as one stage on one GPU, batch 1,
512-token prefill (timed separately, reported under "prefill"), then W untimed and K timed
decode steps.  One "step" = one decode token for every row of the batch through the whole
model.  N>1 (one rank per GPU: under torchrun, or `bench.py --gpus N` starts the N ranks
itself): the same model split into N stages by the server's round-robin layer assignment
(server.py:893-905), activations over RCCL send/recv, 2N micro-batches in flight, plus the
configs[3] / configs[4] records — see distributed_inference_demo_amd/pipeline_bench.py.

Prints ONE JSON line (rank 0).  Inputs are resident in HBM before the timed region.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0      # MI355X HBM3E vendor peak (MI355X_MICROARCH.md)
BF16_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA vendor peak


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=128)
    p.add_argument("--warmup", type=int, default=8)
    p.add_argument("--model", default="bloom-1b1")
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--prompt", type=int, default=512)
    p.add_argument("--dtype", default="bf16")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--weights", default="bf16", choices=["bf16", "int8"],
                   help="int8: weight-only int8 block matrices (BS_FLAG_INT8_WEIGHTS, the bloom*-int8 variants)")
    p.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU checker on a bounded sample")
    p.add_argument("--cpu-steps", type=int, default=24)
    p.add_argument("--no-profile", action="store_true")
    p.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC passes for roofline.traffic")
    p.add_argument("--no-head-split", action="store_true", help="pipeline: keep the whole lm_head on the last stage")
    p.add_argument("--pipeline", action="store_true",
                   help="N = 1: report the pipeline code's line (weak + strong) instead of the single-stage one")
    p.add_argument("--no-pipeline-n1", action="store_true",
                   help="N = 1: skip the pipeline code's N = 1 point (the reference point of the N > 1 curve)")
    p.add_argument("--no-strong", action="store_true", help="pipeline: skip the fixed-rows (strong) measurement")
    p.add_argument("--no-configs", action="store_true",
                   help="pipeline: skip the BASELINE.json configs[3] / configs[4] records")
    p.add_argument("--no-replicas", action="store_true",
                   help="pipeline: skip the replicas record (the whole model on every GPU, same total rows)")
    p.add_argument("--configs2-model", default="bloom-3b", help="configs[2]: model (uneven split at N = 4)")
    p.add_argument("--configs2-batch", default="1,8", help="configs[2]: batch sizes B")
    p.add_argument("--configs2-prompt", type=int, default=64, help="configs[2]: prompt tokens per row")
    p.add_argument("--configs2-steps", type=int, default=128, help="configs[2]: timed decode rounds")
    p.add_argument("--configs-model", default="bloom-7b1", help="pipeline: model of the configs[3] / [4] records")
    p.add_argument("--configs3-mb", type=int, default=8, help="configs[3]: micro-batches of one row (B)")
    p.add_argument("--configs3-prompt", type=int, default=512, help="configs[3]: prefill tokens per row")
    p.add_argument("--configs4-rows", type=int, default=32, help="configs[4]: decode batch B")
    p.add_argument("--configs4-ctx", default="256,512,1024,2048", help="configs[4]: contexts reported")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="pipeline process-group backend (gloo: host tensors, needs --executor)")
    p.add_argument("--executor", default=None,
                   help="pipeline: module:function returning the per-stage executor factory for (model, dtype, "
                        "seed) -- a test hook for the gloo backend (tests/bench_checker.py)")
    return p.parse_args(argv)


def pmc_traffic(args, kernel_tag, timeout=240):
    """roofline.traffic: HBM bytes per decode-GEMV launch from two separate rocprofv3 --pmc passes
    (FETCH_SIZE, then WRITE_SIZE) over a short child run of this same workload.  gfx950 correction
    (MI355X_MICROARCH.md section HBM): FETCH_SIZE counts half the bytes of wide coalesced reads ->
    x2; WRITE_SIZE is exact; both in KB.  Returns (bytes_per_launch, launches) or (None, reason)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    out = tempfile.mkdtemp(prefix="bench_pmc_")
    tot = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        cmd = [prof, "--pmc", counter, "-d", out, "-o", counter.lower(), "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--steps", "8", "--warmup", "2", "--cpu-baseline", "0",
               "--no-profile", "--no-pmc", "--no-pipeline-n1", "--model", args.model, "--batch", str(args.batch), "--prompt",
               str(args.prompt), "--dtype", args.dtype, "--seed", str(args.seed),
               "--weights", args.weights]
        # decode steps launched eagerly under counter collection: rocprofiler-sdk's dispatch interception faulted on
        # graph-launched kernels (profiles/r06_rocprof_pmc_segv.txt); same kernels, bit-identical results
        env = dict(os.environ, BS_GRAPHS="0")
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
        except subprocess.TimeoutExpired:
            return None, f"rocprofv3 {counter} pass timed out"
        files = [os.path.join(dp, f) for dp, _, fs in os.walk(out) for f in fs
                 if f.startswith(counter.lower()) and f.endswith("counter_collection.csv")]
        if r.returncode != 0 or not files:
            return None, f"rocprofv3 {counter} pass failed (rc {r.returncode})"
        vals = []
        for row in csv.DictReader(open(files[0])):
            if row["Counter_Name"] == counter and kernel_tag in row["Kernel_Name"]:
                vals.append(float(row["Counter_Value"]))
        if not vals:
            return None, f"no {kernel_tag} dispatches in the {counter} pass"
        vals = vals[len(vals) // 4:]  # drop the prefill/warm-up quarter
        scale = 2 * 1024 if counter == "FETCH_SIZE" else 1024
        tot[counter] = (sum(vals) / len(vals) * scale, len(vals))
    shutil.rmtree(out, ignore_errors=True)
    return tot["FETCH_SIZE"][0] + tot["WRITE_SIZE"][0], tot["FETCH_SIZE"][1]


def _host_info():
    import platform
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count()
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cpu_model": _cpu_model(), "machine": platform.machine()}


def _cpu_stages(model, ranges, n_ctx, seed):
    from oracle.oracle import OracleStage
    return [OracleStage(model.hidden, model.n_head, model.n_layer, model.vocab, a, b, bf16=False, max_batch=1,
                        max_ctx=n_ctx, seed=seed, is_first=(a == 0), is_last=(b == model.n_layer))
            for a, b in ranges]


def _run_cpu_stages(model, stages, prompt, steps, mode, warmup=3):
    """The reference's CPU execution model on the C restatement (oracle/bloom_oracle.c, fp32, OpenMP):
    one stage object per layer range, every hop serialized in the utils.cpp wire format
    (SerializeTensorVectorToBytes / DeserializeTensorVectorFromBytes, utils.cpp:124-368, here bs_codec_*),
    greedy tokens.  mode "cpu-kv": KV-cached decode; "cpu-ref": every token recomputes the whole
    sequence without a cache (what the reference's input_ids-only ONNX modules compute,
    Communication.java:322-326).  Returns tokens/s over `steps` timed tokens."""
    import numpy as np
    from distributed_inference_demo_amd.stage import deserialize_tensors, serialize_tensors
    from oracle.oracle import prompt_ids
    seq = [int(t) for t in prompt_ids(1234, 1, prompt, model.vocab).reshape(-1)]

    def token(ids, past):
        x = np.asarray(ids, np.int32).reshape(1, -1)
        S = x.shape[1]
        for st in stages:
            y = st.forward(x, 1, S, past_len=past)
            if not st.is_last:
                (x,) = deserialize_tensors(serialize_tensors([y]))  # the inter-stage hop
        return int(y[0])

    if mode == "cpu-kv":
        tok = token(seq, 0)
        seq.append(tok)
        for _ in range(warmup):
            tok = token([tok], len(seq) - 1)
            seq.append(tok)
        t0 = time.perf_counter()
        for _ in range(steps):
            tok = token([tok], len(seq) - 1)
            seq.append(tok)
    else:
        for _ in range(1 + warmup):
            seq.append(token(seq, 0))
        t0 = time.perf_counter()
        for _ in range(steps):
            seq.append(token(seq, 0))
    return steps / (time.perf_counter() - t0)


def cpu_baseline(model, steps, seed, ranges=None):
    """Host-CPU baseline of the same run (BASELINE.md "CPU baseline plan"): the fp32 C restatement on a
    bounded sample of the benchmarked model and stage split (cpu-kv: `steps` tokens, cpu-ref: a few),
    plus BASELINE.json configs[0] (bloom-560m, 2 stages [0,12) [12,24), wire-format loopback).  Prompts
    are 16 tokens (a 512-token CPU prefill alone would take minutes; the per-token cost of a cached
    decode changes by < 3 % of its FLOPs between 16 and 512 positions), 3 warm-up tokens excluded."""
    from distributed_inference_demo_amd import config
    from distributed_inference_demo_amd.placement import stage_ranges
    from oracle.oracle import num_threads
    ranges = ranges or [(0, model.n_layer)]
    n_ref, n_ctx = max(8, steps // 3), 16 + 3 + 1 + max(steps, max(8, steps // 3)) + 4
    t0 = time.perf_counter()
    st = _cpu_stages(model, ranges, n_ctx, seed)
    t_init = time.perf_counter() - t0
    kv = _run_cpu_stages(model, st, 16, steps, "cpu-kv")
    ref = _run_cpu_stages(model, st, 16, n_ref, "cpu-ref")
    del st
    m560 = config.get("bloom-560m")
    r560 = stage_ranges(2, m560.n_layer)
    st = _cpu_stages(m560, r560, n_ctx, seed)
    kv560 = _run_cpu_stages(m560, st, 16, steps, "cpu-kv")
    ref560 = _run_cpu_stages(m560, st, 16, n_ref, "cpu-ref")
    del st
    host = _host_info()
    thr = num_threads()
    return {"value": kv, "unit": "tokens/s", "cores": thr, "kind": "port",
            "sample": f"{model.name} fp32 C restatement (oracle/bloom_oracle.c), stages {ranges} joined by the "
                      f"utils.cpp wire format, batch 1, cpu-kv: {steps} decode tokens after a 16-token prompt, "
                      f"cpu-ref: {n_ref} tokens each recomputing the whole sequence (3 warm-up tokens excluded), "
                      f"{thr} OpenMP threads; weight generation {t_init:.1f}s excluded",
            "threads_note": (f"{thr} OpenMP threads = OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}: "
                             "the GPU box's CPU share per GPU (the harness sets it and asks that worker pools be "
                             "sized to it); nproc / affinity_cpus count the whole host"),
            "modes": {"cpu-kv": kv, "cpu-ref": ref},
            "configs0_bloom560m_2stage_loopback": {"stages": r560, "cpu-kv": kv560, "cpu-ref": ref560,
                                                   "unit": "tokens/s", "prompt": 16},
            **host}


def hbm_measured(dev):
    """STREAM-like HBM figures on this GPU (report measured beside vendor peaks): the
    library's bs_hbm_probe (2 GiB, non-temporal 16-B loads, best of 10: read-only and copy rates) and a
    torch copy_ of the same size for comparison."""
    import torch
    from distributed_inference_demo_amd.stage import hbm_probe
    rd, cp = hbm_probe(dev.index or 0, 2 << 30)
    n = 1 << 30
    a = torch.empty(n, dtype=torch.bfloat16, device=dev).fill_(1)
    b = torch.empty_like(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(12):
        e0.record()
        b.copy_(a)
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1))
    del a, b
    torch.cuda.empty_cache()
    return {"read_GBps": rd, "copy_GBps": cp, "torch_copy_GBps": 2 * 2 * n / (best * 1e-3) / 1e9,
            "method": "bs_hbm_probe: 2 GiB, 16-B non-temporal loads (8 in flight per thread), 2048 x 256 threads, best of 10, HIP events"}


def mfma_measured(dev):
    """Measured dense bf16 MFMA rate (re-measure the vendor peaks on the box): bs_mfma_probe,
    register-operand MFMA chains on every CU, best of 5."""
    from distributed_inference_demo_amd.stage import mfma_probe
    a, b = mfma_probe(dev.index or 0)
    return {"bf16_TFLOPs": max(a, b), "v_mfma_f32_32x32x16_bf16": a, "v_mfma_f32_16x16x32_bf16": b,
            "method": "bs_mfma_probe: 8 independent accumulator chains per wave, 8 waves per CU, no memory "
                      "traffic, best of 5, HIP events"}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def bench_single(args):
    import torch
    from distributed_inference_demo_amd import config
    from distributed_inference_demo_amd.stage import Stage

    m = config.get(args.model)
    if m.int8_weights:  # "-int8" model name
        args.weights = "int8"
    B, P, K, W = args.batch, args.prompt, args.steps, args.warmup
    prof_steps = 0 if args.no_profile else min(16, K)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    max_ctx = P + W + K + prof_steps + 1
    st = Stage(m.hidden, m.n_head, m.n_layer, m.vocab, 0, m.n_layer, dtype=args.dtype, device=0, max_batch=B,
               max_ctx=max_ctx, max_tokens=max(B * P, B), seed=args.seed,
               int8_weights=args.weights == "int8" or m.int8_weights)
    wbytes = st.info()["weight_bytes"]
    cs = torch.cuda.Stream()  # a real stream (the legacy default stream cannot be graph-captured)
    with torch.cuda.stream(cs):
        stream = cs.cuda_stream
        ids = torch.from_numpy(_prompt(B, P, m.vocab)).to(dev)
        tok = torch.empty(B, dtype=torch.int32, device=dev)
        # prefill: one untimed pass (first launch of every kernel), the timed pass (bracketed by syncs,
        # no events), then a pass with HIP events around every GEMM for the GEMM/other split.  Every pass
        # rewrites the same KV rows of slot 0 with the same values.
        st.forward(ids, tok, B, P, slot=0, past_len=0, stream=stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.forward(ids, tok, B, P, slot=0, past_len=0, stream=stream)
        torch.cuda.synchronize()
        t_prefill = time.perf_counter() - t0
        pf_ms = pf_n = pf_flops = 0
        if not args.no_profile:
            st.profile_enable(2)
            st.forward(ids, tok, B, P, slot=0, past_len=0, stream=stream)
            torch.cuda.synchronize()
            pf_ms, pf_n, pf_flops = st.profile_read()
            st.profile_enable(0)
        past = P
        for _ in range(W):  # warm-up (captures the decode graph)
            st.forward(tok, tok, B, 1, slot=0, past_len=past, stream=stream)
            past += 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):  # timed region: graph replays, inputs resident in HBM
            st.forward(tok, tok, B, 1, slot=0, past_len=past, stream=stream)
            past += 1
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        # roofline pass: the same decode steps, HIP events around every weight GEMV (class 1, eager)
        g_ms = g_n = g_bytes = 0
        if prof_steps:
            st.profile_enable(1)
            for _ in range(prof_steps):
                # the eager step's ~100 launches are enqueued behind a spin, so the event pairs time
                # the GPU's execution, not the host's launch cadence
                Stage.stream_delay(stream, 3000)
                st.forward(tok, tok, B, 1, slot=0, past_len=past, stream=stream)
                past += 1
            g_ms, g_n, g_bytes = st.profile_read()
            st.profile_enable(0)
    ms_step = dt * 1e3 / K
    ctx_mid = P + W + K / 2
    step_bytes = config.decode_step_bytes(m, m.n_layer, B, ctx_mid, True, True,
                                          w_bytes=2 if args.dtype == "bf16" else 4,
                                          kv_bytes=2 if args.dtype == "bf16" else 4)
    if args.weights == "int8":  # block matrices: 1 byte per weight + one fp32 scale per output row
        step_bytes -= m.n_layer * (12.0 * m.hidden * m.hidden * 1 - 9.0 * m.hidden * 4)
    res = {
        "metric": "decode tokens/s, BLOOM pipeline",
        "value": B * K / dt, "unit": "tokens/s", "n_gpus": 1, "steps": K, "warmup": W,
        "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic: repo-generator random-init weights (seed %d), prompt ids U[0,V) seed 1234" % args.seed,
        "config": {"workload": f"{m.name} single stage on 1 MI355X, batch {B} decode after a {P}-token prefill "
                               "(BASELINE.json configs[1])",
                   "model": m.name, "stages": 1, "layers_per_stage": [m.n_layer], "batch": B, "prompt": P,
                   "ctx_range": [P + W, P + W + K], "parallelism": "pp1", "weight_bytes": wbytes,
                   "weights": args.weights},
    }
    if g_n:
        avg_ms = g_ms / g_n
        ach = (g_bytes / g_n) / (avg_ms * 1e-3) / 1e9
        tag, kname = "gemv", "gemv_rows_kernel (every decode weight GEMV: LN+QKV, dense, LN+fc1, fc2, ln_f+lm_head)"
        if args.weights == "int8":
            kname = "gemv_q8_kernel (qkv, dense, fc1, fc2 on int8 weights) + gemv_rows_kernel (ln_f+lm_head, bf16)"
        unit_note = "algorithmic bytes per launch = weights + bias + activations of the GEMV"
        traffic, note = (None, "--no-pmc") if args.no_pmc else pmc_traffic(args, tag)
        res["roofline"] = {"bound": "hbm", "kernel": kname,
                           "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBPS,
                           "traffic": traffic, "launches": g_n, "avg_us": avg_ms * 1e3,
                           "algo_bytes_per_launch": g_bytes / g_n, "algo_note": unit_note,
                           "traffic_note": ("HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024), "
                                            "separate rocprofv3 --pmc passes, gfx950 x2 fetch correction; "
                                            f"{note} launches" if traffic else f"traffic unavailable: {note}"),
                           "measured": f"HIP events on the stage stream around each launch, {prof_steps} "
                                       "eager decode steps right after the timed region, each enqueued "
                                       "behind a 3 ms stream spin (no host-submission gaps)"}
    res["stage_hbm"] = {"algo_bytes_per_step": step_bytes, "achieved_GBps": step_bytes / (ms_step * 1e-3) / 1e9,
                        "frac_of_peak": step_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBPS}
    res["prefill"] = {"tokens": B * P, "ms": t_prefill * 1e3, "tokens_per_s": B * P / t_prefill,
                      "algo_flops": config.prefill_flops(m, m.n_layer, B, P, True),
                      "timing": "second of three identical prefills (the first warms every kernel), host clock "
                                "between device syncs, no events; gemm_TFLOPs from HIP events around every "
                                "GEMM in the third"}
    res["prefill"]["achieved_TFLOPs"] = res["prefill"]["algo_flops"] / t_prefill / 1e12
    if pf_n:
        res["prefill"]["gemm_TFLOPs"] = pf_flops / (pf_ms * 1e-3) / 1e12
        res["prefill"]["gemm_frac_of_peak"] = res["prefill"]["gemm_TFLOPs"] / BF16_PEAK_TFLOPS
    st.close()
    hbm = hbm_measured(dev)
    res["hbm_measured"] = dict(hbm, vendor_peak_GBps=HBM_PEAK_GBPS)
    if "roofline" in res:  # the decode GEMVs only read: compare them with the measured read rate
        res["roofline"]["peak_measured_read"] = hbm["read_GBps"]
        res["roofline"]["frac_of_measured_read"] = res["roofline"]["achieved"] / hbm["read_GBps"]
    res["stage_hbm"]["frac_of_measured_read"] = res["stage_hbm"]["achieved_GBps"] / hbm["read_GBps"]
    mf = mfma_measured(dev)
    res["mfma_measured"] = dict(mf, vendor_peak_TFLOPs=BF16_PEAK_TFLOPS)
    if "gemm_TFLOPs" in res["prefill"]:
        res["prefill"]["gemm_frac_of_measured_peak"] = res["prefill"]["gemm_TFLOPs"] / mf["bf16_TFLOPs"]
    return res


def _prompt(B, P, V):
    from distributed_inference_demo_amd.stage import prompt_ids
    return prompt_ids(1234, B, P, V)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _pipeline(args):
    """pipeline_bench.bench_pipeline on this process's rank (torchrun env, or a world-1 group at N = 1: the
    point the N > 1 lines -- the same code -- scale from)."""
    from distributed_inference_demo_amd.pipeline_bench import bench_pipeline
    if "WORLD_SIZE" not in os.environ:
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    factory = None
    if args.executor:
        import importlib
        mod, fn = args.executor.split(":")
        factory = getattr(importlib.import_module(mod), fn)
    return bench_pipeline(args, backend=args.backend, executor_factory=factory)


def launch_ranks(n, argv):
    """`bench.py --gpus N` run plainly (no torchrun env): start N rank processes of this same script under
    torch.distributed.run (one per GPU, rendezvous on 127.0.0.1) and return their exit status.  The parent
    touches no GPU -- it only waits -- and rank 0's JSON line reaches stdout through the shared descriptor;
    torchrun stops every rank and exits non-zero if any rank fails."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} started with WORLD_SIZE={world}")
    # the driver reads ONE JSON line from stdout: libraries that print banners there (RCCL prints its version
    # block when a communicator is created) are sent to stderr at the file-descriptor level
    out_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    ranges = model = None
    rc = 0
    if world > 1 or args.pipeline:
        res, ranges, model = _pipeline(args)
    else:
        res = bench_single(args)
        if os.environ.get("BS_DUMP_MAPS"):  # diagnostics: the process's mappings, to symbolise a native fault's frames
            import shutil
            shutil.copyfile("/proc/self/maps", os.environ["BS_DUMP_MAPS"])
        if not args.no_pipeline_n1:
            # the N = 1 point of the pipeline curve and its configs records ride on the headline: a failure there
            # (out of memory on a shared GPU, a 7b1-shape error) is reported in the line, never loses it
            try:
                p1, _, _ = _pipeline(args)
                res["pipeline_n1"] = {k: p1[k] for k in ("value", "ms_per_step", "config", "weak_definition",
                                                         "scaling_ref", "stage_hbm", "prefill", "strong", "configs2",
                                                         "configs3", "configs4", "replicas") if k in p1}
                res["pipeline_n1"]["note"] = ("pipeline_bench.bench_pipeline at N = 1 (nccl world-1 group, "
                                              "StageExecutor, graph-replayed decode): the same code and definitions "
                                              "as the N > 1 lines")
            except Exception as e:  # noqa: BLE001 -- recorded in the line, the headline stands
                import traceback
                import torch
                traceback.print_exc()
                res["pipeline_n1"] = {"error": f"{type(e).__name__}: {e}"}
                # out of memory (a shared GPU) is the one failure the run survives; any other error (a HIP fault, an
                # RCCL error, a regression in a configs record) still prints the line but fails the run
                if not isinstance(e, torch.cuda.OutOfMemoryError):
                    rc = 1
                try:
                    import torch.distributed as dist
                    if dist.is_initialized():
                        dist.destroy_process_group()
                except Exception:  # noqa: BLE001
                    pass
        from distributed_inference_demo_amd import config
        model = config.get(args.model)
    if res is not None and args.cpu_baseline:  # rank 0, after the process group is gone
        res["cpu_baseline"] = cpu_baseline(model, args.cpu_steps, args.seed, ranges=ranges)
    sys.stdout.flush()
    if res is not None:
        os.write(out_fd, (json.dumps(res) + "\n").encode())
    return rc


if __name__ == "__main__":
    sys.exit(main())
