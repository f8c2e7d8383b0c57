"""A/B numerics of a decode-path env switch on the full bloom-1b1 stage (GPU), against the bf16 checker.

    SWITCH=1 python tools/diag_fused.py gpurun_out/a.npz
    SWITCH=0 python tools/diag_fused.py gpurun_out/b.npz
    python tools/diag_fused.py --compare gpurun_out/a.npz gpurun_out/b.npz

Runs a 512-token prefill and 16 teacher-forced decode steps (the checker's tokens) and saves the GPU
logits and the checker's logits per step.  Used for profiles/r02_attn_dense_numerics.txt (the
attention + dense fusion of round 2, BS_ATTN_DENSE, since removed from the library).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(path):
    import torch
    from distributed_inference_demo_amd import config
    from distributed_inference_demo_amd.stage import Stage
    from oracle.oracle import OracleStage, prompt_ids

    m = config.get("bloom-1b1")
    P, STEPS = 512, 16
    g = Stage(m.hidden, m.n_head, m.n_layer, m.vocab, 0, m.n_layer, dtype="bf16", max_batch=1,
              max_ctx=P + STEPS + 1, max_tokens=P, seed=0)
    o = OracleStage(m.hidden, m.n_head, m.n_layer, m.vocab, 0, m.n_layer, bf16=True, max_batch=1,
                    max_ctx=P + STEPS + 1, seed=0)
    ids = prompt_ids(1234, 1, P, m.vocab)
    dev = torch.device("cuda", 0)
    cs = torch.cuda.Stream()
    G, O = [], []
    with torch.cuda.stream(cs):
        tin = torch.from_numpy(ids).to(dev)
        tok = torch.empty(1, dtype=torch.int32, device=dev)
        lg = torch.empty((1, m.vocab), dtype=torch.float32, device=dev)
        g.forward(tin, tok, 1, P, past_len=0, logits=lg, stream=cs.cuda_stream)
        to, lo = o.forward(ids, 1, P, want_logits=True)
        torch.cuda.synchronize()
        G.append(lg.cpu().numpy()[0]); O.append(lo[0])
        for step in range(STEPS):
            tok.copy_(torch.from_numpy(to))
            g.forward(tok, tok, 1, 1, past_len=P + step, logits=lg, stream=cs.cuda_stream)
            to, lo = o.forward(to.reshape(1, 1), 1, 1, past_len=P + step, want_logits=True)
            torch.cuda.synchronize()
            G.append(lg.cpu().numpy()[0]); O.append(lo[0])
    G, O = np.array(G), np.array(O)
    np.savez(path, gpu=G, ref=O)
    err = np.abs(G - O).max(axis=1)
    print(os.path.basename(path), "max-abs vs checker per step:", " ".join("%.4f" % e for e in err))
    print("mean-abs per step:", " ".join("%.5f" % e for e in np.abs(G - O).mean(axis=1)))


def compare(a, b):
    A, B = np.load(a), np.load(b)
    for name, x in (("A", A), ("B", B)):
        e = np.abs(x["gpu"] - x["ref"])
        print(name, "max", " ".join("%.4f" % v for v in e.max(axis=1)), "| mean", "%.5f" % e.mean())
    d = np.abs(A["gpu"] - B["gpu"])
    print("A vs B gpu: max", " ".join("%.4f" % v for v in d.max(axis=1)), "| mean", "%.5f" % d.mean())


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])
