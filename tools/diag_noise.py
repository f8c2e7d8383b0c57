"""Diagnostic: bf16 GPU-vs-checker error of one real-width block per family (S=64 / S=7 / S=1),
beside the checker's own noise floor (fp32 vs double accumulation of the same bf16-emulated math)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401
from distributed_inference_demo_amd.stage import Stage
from oracle.oracle import OracleStage, lib as olib
G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "family_blocks.npz")
f = np.load(G)
for fam in ["560m", "1b1", "3b", "7b1"]:
    h, nh, _, V, seed = (int(v) for v in f[fam + "_config"])
    res = {}
    for acc in (0, 1):
        olib().or_set_accum_double(acc)
        o = OracleStage(h, nh, 1, V, 0, 1, bf16=True, max_ctx=64, seed=seed, is_last=False)
        ids = f[fam + "_ids23"]
        r = [o.forward(f[fam + "_ids64"], 1, 64)]
        o.forward(ids[:, :15], 1, 15, past_len=0)
        r.append(o.forward(ids[:, 15:22], 1, 7, past_len=15))
        r.append(o.forward(ids[:, 22:23], 1, 1, past_len=22))
        res[acc] = r
    olib().or_set_accum_double(0)
    g = Stage(h, nh, 1, V, 0, 1, dtype="bf16", max_ctx=64, max_tokens=64, seed=seed, is_last=False)
    ids = f[fam + "_ids23"]
    gr = [g.forward_host(f[fam + "_ids64"], 1, 64)]
    g.forward_host(ids[:, :15], 1, 15, past_len=0)
    gr.append(g.forward_host(ids[:, 15:22], 1, 7, past_len=15))
    gr.append(g.forward_host(ids[:, 22:23], 1, 1, past_len=22))
    for i, name in enumerate(["S=64", "S=7", "S=1"]):
        print(f"{fam} {name}: gpu-vs-oracle {np.abs(gr[i] - res[0][i]).max():.4f}  gpu-vs-oracle(double) "
              f"{np.abs(gr[i] - res[1][i]).max():.4f}  oracle floor {np.abs(res[0][i] - res[1][i]).max():.4f}  "
              f"max|ref| {np.abs(res[0][i]).max():.2f}", flush=True)
