"""Where a persistent decode step spends its time: per-phase durations from the in-kernel
s_memrealtime stamps (BS_ENGINE_TRACE=1, 100 MHz), median and max over workgroups, averaged over
the stage's layers.  Diagnostic only (the stamps are plain stores of lane 0 per phase).

    BS_ENGINE_TRACE=1 python tools/engine_trace.py [model] [batch] [prompt]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("BS_ENGINE_TRACE", "1")

import torch  # noqa: E402

from distributed_inference_demo_amd import config  # noqa: E402
from distributed_inference_demo_amd.stage import Stage, prompt_ids  # noqa: E402

PHASES = ["qkv.wait", "qkv.ln+gemv", "qkv.epi+pub", "att.wait", "att.units", "dense.pf+wait", "dense.gemv",
          "dense.epi+pub", "fc1.pf+wait", "fc1.ln+gemv+pub", "fc2.pf+wait", "fc2.gemv+pub"]


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "bloom-1b1"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    P = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    m = config.get(name)
    torch.cuda.init()
    st = Stage(m.hidden, m.n_head, m.n_layer, m.vocab, 0, m.n_layer, dtype="bf16", max_batch=B, max_ctx=P + 16,
               max_tokens=B * P, seed=0)
    cs = torch.cuda.Stream()
    with torch.cuda.stream(cs):
        ids = torch.from_numpy(prompt_ids(1234, B, P, m.vocab)).cuda()
        tok = torch.empty(B, dtype=torch.int32, device="cuda")
        st.forward(ids, tok, B, P, past_len=0, stream=cs.cuda_stream)
        for i in range(8):
            st.forward(tok, tok, B, 1, past_len=P + i, stream=cs.cuda_stream)
        torch.cuda.synchronize()
    tr = st.engine_trace().astype(np.int64)
    code = st.engine_status()
    L = m.n_layer
    t0 = tr[:, 0].min()
    t = (tr - t0) * 10e-3  # us
    total = t[:, 1 + 12 * L + 3].max() if t[:, 1 + 12 * L + 3].max() > 0 else t.max()
    print(f"{name} B={B} ctx={P + 8}: {tr.shape[0]} workgroups, kernel span {total:.1f} us, give-up code {code}")
    prev = t[:, 0]
    acc = np.zeros((L, len(PHASES), 2))
    for l in range(L):
        b = 1 + 12 * l
        for k in range(12):
            d = t[:, b + k] - (prev if k == 0 else t[:, b + k - 1])
            acc[l, k] = (np.median(d), d.max())
        prev = t[:, b + 11]
    layer_end = np.array([t[:, 1 + 12 * l + 11].max() for l in range(L)])
    print(f"per-layer span (last workgroup): mean {np.diff(layer_end).mean():.2f} us")
    print(f"{'phase':18s} {'median':>8s} {'max':>8s}  (us, mean over layers)")
    for k, nm in enumerate(PHASES):
        print(f"{nm:18s} {acc[1:, k, 0].mean():8.2f} {acc[1:, k, 1].mean():8.2f}")
    hb = 1 + 12 * L
    for k, nm in enumerate(["head.pf+wait", "head.ln+gemv", "head.argmax"]):
        d = t[:, hb + k] - (t[:, hb - 1] if k == 0 else t[:, hb + k - 1])
        print(f"{nm:18s} {np.median(d):8.2f} {d.max():8.2f}")
    st.close()


if __name__ == "__main__":
    main()
