"""Single-GPU decode measurements across BASELINE.json model/batch/context configurations.

Each row: one full model as one stage (the per-stage kernels are the same ones a pipeline stage
runs), prefill `prompt` tokens, then time `steps` graph-replayed decode steps.  Reports tokens/s,
ms/step and the stage's algorithmic HBM bytes/step (BASELINE.md formula) / step time.
    python tools/bench_matrix.py [--quick]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from distributed_inference_demo_amd import config  # noqa: E402
from distributed_inference_demo_amd.stage import Stage, prompt_ids  # noqa: E402

HBM_PEAK = 8000.0
CONFIGS = [  # (model, batch, prompt, steps)
    ("bloom-560m", 1, 16, 128), ("bloom-1b1", 1, 512, 128), ("bloom-3b", 1, 64, 128), ("bloom-3b", 8, 64, 128),
    ("bloom-7b1", 1, 128, 128), ("bloom-7b1", 8, 512, 64), ("bloom-7b1", 32, 128, 64), ("bloom-7b1", 32, 1024, 32),
    ("bloom-7b1", 32, 1984, 32), ("bloom-7b1", 16, 128, 64), ("bloom-3b", 32, 64, 64), ("bloom-1b1", 8, 128, 64),
    ("bloom-1b1", 32, 128, 64), ("bloom-560m", 16, 16, 128), ("bloom-560m", 32, 16, 128),
]


def run(name, B, P, K, W=4):
    m = config.get(name)
    st = Stage(m.hidden, m.n_head, m.n_layer, m.vocab, 0, m.n_layer, dtype="bf16", max_batch=B,
               max_ctx=P + W + K + 1, max_tokens=max(B * P, B), seed=0)
    cs = torch.cuda.Stream()
    with torch.cuda.stream(cs):
        ids = torch.from_numpy(prompt_ids(1234, B, P, m.vocab)).cuda()
        tok = torch.empty(B, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.forward(ids, tok, B, P, past_len=0, stream=cs.cuda_stream)
        torch.cuda.synchronize()
        tp = time.perf_counter() - t0
        past = P
        for _ in range(W):
            st.forward(tok, tok, B, 1, past_len=past, stream=cs.cuda_stream)
            past += 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            st.forward(tok, tok, B, 1, past_len=past, stream=cs.cuda_stream)
            past += 1
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    st.close()
    ctx = P + W + K / 2
    byts = config.decode_step_bytes(m, m.n_layer, B, ctx, True, True)
    ms = dt * 1e3 / K
    return {"model": name, "batch": B, "prompt": P, "ctx_mid": ctx, "tokens_per_s": B * K / dt, "ms_per_step": ms,
            "algo_GB_per_step": byts / 1e9, "hbm_GBps": byts / (ms * 1e-3) / 1e9,
            "hbm_frac": byts / (ms * 1e-3) / 1e9 / HBM_PEAK, "prefill_ms": tp * 1e3,
            "prefill_TFLOPs": config.prefill_flops(m, m.n_layer, B, P, True) / tp / 1e12}


BATCHED = [("bloom-1b1", 8, 128, 64), ("bloom-560m", 8, 16, 128), ("bloom-1b1", 32, 128, 64), ("bloom-560m", 16, 16, 128), ("bloom-560m", 32, 16, 128),
           ("bloom-3b", 8, 64, 128), ("bloom-3b", 32, 64, 64), ("bloom-7b1", 16, 128, 64), ("bloom-7b1", 32, 128, 64),
           ("bloom-7b1", 32, 1024, 32)]

if __name__ == "__main__":
    cfgs = CONFIGS[:3] if "--quick" in sys.argv else (BATCHED if "batched" in sys.argv else CONFIGS)
    only = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--only=")]  # --only=bloom-1b1:8,bloom-560m:32
    if only:
        keep = {tuple(x.split(":")) for x in only[0].split(",")}
        cfgs = [c for c in cfgs if (c[0], str(c[1])) in keep]
    for c in cfgs:
        print(json.dumps(run(*c)), flush=True)
