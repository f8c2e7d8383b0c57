"""Does the host keep ahead of the GPU at 16 micro-batches per round?  (VERDICT r4 "next" #6)

The N = 8 stage shape of bloom-1b1: 3 layers (24 / 8) per stage, 16 one-row micro-batches in flight
(2N, the reference's core_pool_size, Communication.java:418-437), and a 1/8 slice of the tied lm_head
(vocabulary-parallel head).  On one GPU that stage runs as a world-1 Pipeline (no RCCL on the data path):

  host_us_per_mb : host wall time of one Pipeline.step(1) round / 16 (ctypes bs_forward + the pipeline's
                   Python bookkeeping per micro-batch), with the stream kept busy by a spin so the host never
                   waits on the GPU
  gpu_us_per_mb  : GPU time of one round / 16 (HIP events around 20 rounds, replays back to back)
  rccl_us        : host cost of one RCCL call on this box (a 1-element all_reduce on the world-1 nccl group,
                   enqueue only); an N = 8 middle rank issues 4 per micro-batch (irecv + wait, isend, and one
                   packed receive + one packed send on the head ring), so host_us_per_mb + 4 * rccl_us models
                   the N = 8 host cost.
Prints one JSON line.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (before the library: torch's libamdhip64 must serve the process)
import torch.distributed as dist  # noqa: E402

from distributed_inference_demo_amd import config  # noqa: E402
from distributed_inference_demo_amd.pipeline import build_rank, init_distributed  # noqa: E402
from distributed_inference_demo_amd.stage import Stage  # noqa: E402


def p2p_rounds(st, cs, dev, m, n_mb, past, rounds):
    """the N = 8 middle rank's per-micro-batch enqueue with its RCCL traffic actually issued on this
    box.  Per micro-batch: the stage forward (graph replay), then the two hops a middle rank makes -- the hidden row
    (receive from the previous stage, send to the next) and the packed head-ring message (receive, send) -- each
    issued here as a matched send + receive addressed to this rank itself on the world-1 nccl group (RCCL pairs a
    self send with its receive only inside one group call, so each hop is one batch_isend_irecv; the product
    pipeline's single isend / irecv calls cost less host time each: 'rccl_call_host_us').  Host time per micro-batch
    with the stream kept busy by a spin, against the GPU time of the same rounds (HIP events).
    Variant 'graph': forward + both hops of one micro-batch captured into one torch CUDA graph (RCCL in stream
    capture; the stage launches eagerly into the capture) and replayed, one replay per micro-batch."""
    h = m.hidden
    act = [torch.zeros(h, device=dev) for _ in range(n_mb)]
    act_in = [torch.empty(h, device=dev) for _ in range(n_mb)]
    ring = [torch.zeros(h // 2 + 8, device=dev) for _ in range(n_mb)]  # [xn bf16 | keys] packed message, as floats
    ring_in = [torch.empty_like(r) for r in ring]
    tok = torch.zeros(n_mb, dtype=torch.int32, device=dev)

    def mb(j, pos):
        st.forward(tok[j:j + 1], tok[j:j + 1], 1, 1, slot=j, past_len=pos, stream=cs.cuda_stream)
        for w_ in dist.batch_isend_irecv([dist.P2POp(dist.isend, act[j], 0), dist.P2POp(dist.irecv, act_in[j], 0)]):
            w_.wait()  # stream-level (nccl): the host does not block
        for w_ in dist.batch_isend_irecv([dist.P2POp(dist.isend, ring[j], 0), dist.P2POp(dist.irecv, ring_in[j], 0)]):
            w_.wait()

    out = {"p2p_shape": f"per micro-batch: stage forward + 2 self-addressed send/recv pairs ({h * 4} B hidden row, "
                        f"{(h // 2 + 8) * 4} B ring message), {n_mb} micro-batches per round"}
    pos = [st.past[j] for j in range(n_mb)]
    for j in range(n_mb):  # warm-up (connects the self pair)
        mb(j, pos[j])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    Stage.stream_delay(cs.cuda_stream, 20000)
    e0.record(cs)
    for _ in range(rounds):
        for j in range(n_mb):
            mb(j, pos[j])
    e1.record(cs)
    torch.cuda.synchronize()
    gpu_mb = e0.elapsed_time(e1) * 1e3 / (rounds * n_mb)
    Stage.stream_delay(cs.cuda_stream, 100000)
    t0 = time.perf_counter()
    for _ in range(rounds):
        for j in range(n_mb):
            mb(j, pos[j])
    host_mb = (time.perf_counter() - t0) * 1e6 / (rounds * n_mb)
    torch.cuda.synchronize()
    out.update(p2p_eager_host_us_per_mb=host_mb, p2p_eager_gpu_us_per_mb=gpu_mb, p2p_eager_host_over_gpu=host_mb / gpu_mb)
    # graph variant (opt-in, P2P_GRAPH=1): on this stack (torch 2.10 + RCCL 2.26.6, HIP 7.0) the capture of the RCCL
    # pairs segfaults in torch.cuda.graph's capture_end (hipStreamEndCapture) -- a native fault, not an exception
    # (round 6, gpurun_out/r6d_host_enqueue.err with python -X faulthandler)
    if os.environ.get("P2P_GRAPH") != "1":
        out["p2p_graph_note"] = ("not run: capturing the RCCL send/recv pairs into a torch CUDA graph segfaulted in "
                                 "capture_end on this stack (torch 2.10, RCCL 2.26.6)")
        return out
    try:
        st.set_graphs(False)
        graphs = []
        for j in range(n_mb):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cs):
                mb(j, pos[j])
            graphs.append(g)
        torch.cuda.synchronize()
        for g in graphs:
            g.replay()
        torch.cuda.synchronize()
        Stage.stream_delay(cs.cuda_stream, 20000)
        e0.record(cs)
        for _ in range(rounds):
            for g in graphs:
                g.replay()
        e1.record(cs)
        torch.cuda.synchronize()
        ggpu = e0.elapsed_time(e1) * 1e3 / (rounds * n_mb)
        Stage.stream_delay(cs.cuda_stream, 100000)
        t0 = time.perf_counter()
        for _ in range(rounds):
            for g in graphs:
                g.replay()
        ghost = (time.perf_counter() - t0) * 1e6 / (rounds * n_mb)
        torch.cuda.synchronize()
        out.update(p2p_graph_host_us_per_mb=ghost, p2p_graph_gpu_us_per_mb=ggpu, p2p_graph_host_over_gpu=ghost / ggpu)
    except Exception as e:  # noqa: BLE001 -- recorded: capture of RCCL p2p refused on this stack
        out["p2p_graph_error"] = f"{type(e).__name__}: {e}"[:300]
    finally:
        st.set_graphs(True)
    return out


def main():
    os.environ.setdefault("MASTER_PORT", "29533")
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    init_distributed("nccl")
    dev = torch.device("cuda", 0)
    n_mb, P, rounds = int(os.environ.get("N_MB", "16")), 64, 20
    m = config.BloomDims("bloom-1b1/8-stage", 1536, 3, 16, vocab=31360)  # 3 layers + a 1/8 head slice
    pipe, _ = build_rank(m, 0, 1, dev, mb_rows=1, n_mb=n_mb, max_ctx=P + 4 * rounds + 8, max_seq=P, head_split=False)
    cs = torch.cuda.Stream()
    torch.cuda.set_stream(cs)
    prompt = torch.randint(0, m.vocab, (n_mb, P), dtype=torch.int32, device=dev)
    pipe.step(P, prompt=prompt)
    for _ in range(3):
        pipe.step(1)
    torch.cuda.synchronize()
    # GPU time per round: replays back to back, HIP events on the stage stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    Stage.stream_delay(cs.cuda_stream, 20000)
    e0.record(cs)
    for _ in range(rounds):
        pipe.step(1)
    e1.record(cs)
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / rounds
    # host time per round, the stream busy with a spin the whole time (enqueue never blocks on the GPU)
    Stage.stream_delay(cs.cuda_stream, 100000)
    t0 = time.perf_counter()
    for _ in range(rounds):
        pipe.step(1)
    host_ms = (time.perf_counter() - t0) * 1e3 / rounds
    torch.cuda.synchronize()
    # one RCCL call's host cost (enqueue only, stream busy)
    x = torch.zeros(1, device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    Stage.stream_delay(cs.cuda_stream, 100000)
    t0 = time.perf_counter()
    for _ in range(200):
        dist.all_reduce(x)
    rccl_us = (time.perf_counter() - t0) * 1e6 / 200
    torch.cuda.synchronize()
    # a matched send + receive of one micro-batch's hidden row, to this rank itself in one group call (RCCL allows
    # self p2p inside a group): the host cost of the p2p pair an N = 8 rank issues per hop
    a = torch.zeros(m.hidden, device=dev)
    b2 = torch.empty_like(a)
    ops = [dist.P2POp(dist.isend, a, 0), dist.P2POp(dist.irecv, b2, 0)]
    for w_ in dist.batch_isend_irecv(ops):
        w_.wait()
    torch.cuda.synchronize()
    Stage.stream_delay(cs.cuda_stream, 100000)
    t0 = time.perf_counter()
    for _ in range(100):
        for w_ in dist.batch_isend_irecv(ops):
            w_.wait()
    p2p_pair_us = (time.perf_counter() - t0) * 1e6 / 100
    torch.cuda.synchronize()
    # the pieces of one micro-batch's enqueue (stream busy): torch's current-stream handle, one Stage.forward
    # (Step struct + ctypes + bs_forward's graph launch), and a bare bs_forward with a prebuilt Step
    import ctypes
    from distributed_inference_demo_amd.stage import Step, lib
    Stage.stream_delay(cs.cuda_stream, 100000)
    t0 = time.perf_counter()
    for _ in range(1000):
        torch.cuda.current_stream().cuda_stream
    cur_us = (time.perf_counter() - t0) * 1e3
    st = pipe.ex.stage
    tok = pipe.tok[0]
    past = st.past[0]
    t0 = time.perf_counter()
    for _ in range(200):
        st.forward(tok, tok, 1, 1, slot=0, past_len=past, stream=cs.cuda_stream)
    fwd_us = (time.perf_counter() - t0) * 1e6 / 200
    torch.cuda.synchronize()
    Stage.stream_delay(cs.cuda_stream, 100000)
    stp = Step(1, 1, 0, past, 0, None)
    L, h, ip, sh = lib(), st._h, tok.data_ptr(), cs.cuda_stream
    t0 = time.perf_counter()
    for _ in range(200):
        L.bs_forward(h, ctypes.byref(stp), ip, ip, None, sh)
    raw_us = (time.perf_counter() - t0) * 1e6 / 200
    torch.cuda.synchronize()
    host_mb, gpu_mb = host_ms * 1e3 / n_mb, gpu_ms * 1e3 / n_mb
    p2p = p2p_rounds(st, cs, dev, m, n_mb, past, rounds) if os.environ.get("P2P", "1") == "1" else {}
    res = {"shape": f"bloom-1b1 N = 8 stage: 3 layers, {n_mb} one-row micro-batches, vocab slice {m.vocab}",
           "host_us_per_mb": host_mb, "gpu_us_per_mb": gpu_mb, "host_over_gpu": host_mb / gpu_mb,
           "rccl_call_host_us": rccl_us, "current_stream_handle_us": cur_us, "stage_forward_us": fwd_us,
           "bare_bs_forward_us": raw_us, "p2p_send_recv_pair_host_us": p2p_pair_us,
           "torch_nccl_avoid_record_streams": os.environ.get("TORCH_NCCL_AVOID_RECORD_STREAMS"),
           "n8_middle_rank_rccl_calls_per_mb": 4,
           "modeled_n8_host_us_per_mb": host_mb + 4 * rccl_us,
           "modeled_n8_host_over_gpu": (host_mb + 4 * rccl_us) / gpu_mb, **p2p}
    print(json.dumps(res))
    pipe.ex.stage.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
