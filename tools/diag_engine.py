"""Engine diagnostics on one GPU: graph-replayed B=1 decode of a bloom-1b1-width stage from 16 to ~1000
positions, checking the engine's timeout word after every step; on the first nonzero word, dumps the
sync region (edge counters, merged-head counts, tickets, status)."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from distributed_inference_demo_amd.stage import Stage, lib  # noqa: E402
from oracle import gen_np  # noqa: E402

h, nh, L, V, P = 1536, 16, 2, 2048, 16
g = Stage(h, nh, L, V, 0, L, dtype="bf16", max_batch=1, max_ctx=1024, max_tokens=P, seed=91)
g.set_decode_engine(True)
L_ = lib()
L_.bs_debug_engine_sync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
ids = gen_np.prompt_ids(93, 1, P, V).astype(np.int32)
dev = torch.device("cuda", 0)
cs = torch.cuda.Stream()
eager = len(sys.argv) > 1 and sys.argv[1] == "eager"


def dump(tag):
    w = np.zeros(4096, np.uint32)
    n = L_.bs_debug_engine_sync(g._h, w.ctypes.data, 4096)
    w = w[:n]
    nz = np.flatnonzero(w)
    print(tag, "sync words", n, "nonzero:", [(int(i), hex(int(w[i]))) for i in nz][:80], flush=True)


with torch.cuda.stream(cs):
    tin = torch.from_numpy(ids).to(dev)
    tok = torch.empty(1, dtype=torch.int32, device=dev)
    g.forward(tin, tok, 1, P, past_len=0, stream=cs.cuda_stream)
    past = P
    while past < 1000:
        if eager:
            t = tok.cpu().numpy().reshape(1, 1)
            t = g.forward_host(t, 1, 1, past_len=past)
            tok.copy_(torch.from_numpy(t))
        else:
            g.forward(tok, tok, 1, 1, past_len=past, stream=cs.cuda_stream)
        cs.synchronize()
        used, st = g.engine_status()
        if st != 0 or past in (P, 200, 600, 999):
            dump(f"past {past} used {used} status {st}")
            if st != 0:
                break
        past += 1
print("done at past", past)
