"""Multi-seed study of the bf16 logits distance at bloom-7b1 width (VERDICT r4 "next" #1).

Question: how far from an exact (float64-accumulating) evaluation of the same bf16-rounded math do CORRECT fp32
evaluations land, and where does the device sit in that spread?  The answer fixes the constant bound of
tests/test_gpu_7b1_width.py before any run.

Workload per seed (seeds 101..108): h = 4096, 32 heads (hd 128), V = 4096, repo-generator weights of the seed,
    L = 2 : B = 16 rows x a 16-token prompt (the test's prefill), then one decode step at position 16
    L = 30: B = 8 rows x a 16-token prompt, then one decode step
Logits of the last position of every row.  Checker variants (oracle/bloom_oracle.c knobs, bf16 storage points):
    f64        dot products accumulated in double (the reference point)
    fp32_lanes fp32, 16 lanes + tree (the checker's default order)
    fp32_seq   fp32, one sequential accumulator
    fp32_k32   fp32, 32-element chunks summed in order (the MFMA K-step grouping)
    emul_fp16  fp32_lanes + the device's current P.V roundings: V -> fp16, P -> fp16 hi + lo (unnormalised P)
    emul_bf16  fp32_lanes + P -> bf16 hi + lo, V bf16 (unnormalised P)
Device variants (GPU phase): the library's bf16 stage as built.

    python tools/parity_study.py cpu  [--layers 2,30] [--seeds 8]   # checker variants -> tools/study/ (here)
    python tools/parity_study.py gpu  [--layers 2,30] [--seeds 8]   # device logits -> gpurun_out/study/ (GPU box)
    python tools/parity_study.py report                             # -> profiles/r05_parity_study.{jsonl,txt}
"""
import argparse
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
H, NH, V, P = 4096, 32, 4096, 16
CPU_DIR = os.path.join(ROOT, "tools", "study")
GPU_DIR = os.path.join(ROOT, "gpurun_out", "study")
VARIANTS = {"f64": (1, 0), "fp32_lanes": (0, 0), "fp32_seq": (2, 0), "fp32_k32": (3, 0),
            "emul_fp16": (0, 1 | 2), "emul_bf16": (0, 4)}


BATCH = {}  # --batch override: rows per L (file tag L{L}B{B})


def shape(L):
    return (BATCH.get(L) or (16 if L == 2 else 8), P)


def tag(L):
    return f"L{L}" if L not in BATCH else f"L{L}B{BATCH[L]}"


def inputs(seed, L):
    from oracle import gen_np
    B, S = shape(L)
    return gen_np.prompt_ids(seed + 7, B, S, V).astype(np.int32), gen_np.prompt_ids(seed + 1007, B, 1, V).astype(np.int32)


def run_cpu(layers, seeds):
    from oracle.oracle import OracleStage, checker_mode
    os.makedirs(CPU_DIR, exist_ok=True)
    for L in layers:
        B, S = shape(L)
        for seed in seeds:
            out = os.path.join(CPU_DIR, f"ref_{tag(L)}_s{seed}.npz")
            if os.path.exists(out):
                continue
            ids, nxt = inputs(seed, L)
            o = OracleStage(H, NH, L, V, 0, L, bf16=True, max_batch=B, max_ctx=S + 2, seed=seed)
            res = {}
            for name, (acc, emul) in VARIANTS.items():
                with checker_mode(acc, emul):
                    _, pre = o.forward(ids, B, S, want_logits=True)
                    _, dec = o.forward(nxt, B, 1, past_len=S, want_logits=True)
                res[name + "_prefill"], res[name + "_decode"] = pre, dec
                print(f"L={L} seed={seed} {name}", flush=True)
            o.close()
            np.savez(out, **res)


def run_gpu(layers, seeds, dtag):
    import torch  # noqa: F401  (torch's HIP runtime first)
    from distributed_inference_demo_amd.stage import Stage
    os.makedirs(GPU_DIR, exist_ok=True)
    for L in layers:
        B, S = shape(L)
        for seed in seeds:
            ids, nxt = inputs(seed, L)
            g = Stage(H, NH, L, V, 0, L, dtype="bf16", max_batch=B, max_ctx=S + 2, max_tokens=B * S, seed=seed)
            _, pre = g.forward_host(ids, B, S, past_len=0, want_logits=True)
            _, dec = g.forward_host(nxt, B, 1, past_len=S, want_logits=True)
            g.close()
            np.savez(os.path.join(GPU_DIR, f"dev_{dtag}_{tag(L)}_s{seed}.npz"), prefill=pre, decode=dec)
            print(f"device {dtag} {tag(L)} seed={seed}", flush=True)


def report(out_prefix):
    rows = []
    for f in sorted(glob.glob(os.path.join(CPU_DIR, "ref_L*_s*.npz"))):
        base = os.path.basename(f)[4:-4]  # L{L}[B{B}]_s{seed}
        lt, seed = base.split("_")[0][1:], int(base.split("_")[1][1:])
        L, B = (int(lt.split("B")[0]), int(lt.split("B")[1])) if "B" in lt else (int(lt), 16 if lt == "2" else 8)
        ref = np.load(f)
        cands = {k[:-len("_prefill")]: None for k in ref.files if k.endswith("_prefill") and not k.startswith("f64")}
        for dev in sorted(glob.glob(os.path.join(GPU_DIR, f"dev_*_{base}.npz"))):
            cands["device_" + os.path.basename(dev)[4:-len(base) - 5]] = np.load(dev)
        for name, dv in cands.items():
            for ph in ("prefill", "decode"):
                got = ref[f"{name}_{ph}"] if dv is None else dv[ph]
                d = np.abs(got.astype(np.float64) - ref[f"f64_{ph}"])
                rows.append({"L": L, "B": B, "seed": seed, "phase": ph, "variant": name, "max_abs": float(d.max()),
                             "mean_abs": float(d.mean()), "max_ref": float(np.abs(ref[f"f64_{ph}"]).max()),
                             "n": int(d.size)})
    with open(out_prefix + ".jsonl", "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
    lines = ["distance to the float64-accumulating checker (same bf16 storage points), logits of the last position",
             "per (L, phase, variant): max-abs over seeds [min .. max] and mean over seeds; mean-abs max over seeds", ""]
    keys = sorted({(r["L"], r["B"], r["phase"], r["variant"]) for r in rows})
    for L, B, ph, var in keys:
        sel = [r for r in rows if (r["L"], r["B"], r["phase"], r["variant"]) == (L, B, ph, var)]
        mx = [r["max_abs"] for r in sel]
        mn = [r["mean_abs"] for r in sel]
        lines.append(f"L={L:2d} B={B:2d} {ph:7s} {var:22s} seeds={len(sel)} max-abs [{min(mx):.4f} .. {max(mx):.4f}] "
                     f"mean {np.mean(mx):.4f}   mean-abs max {max(mn):.5f}")
    open(out_prefix + ".txt", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("phase", choices=["cpu", "gpu", "report"])
    ap.add_argument("--layers", default="2,30")
    ap.add_argument("--seeds", type=int, default=8)
    ap.add_argument("--tag", default="lib")
    ap.add_argument("--batch", type=int, default=0, help="rows (default 16 at L = 2, 8 at L = 30)")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05_parity_study"))
    a = ap.parse_args()
    layers = [int(x) for x in a.layers.split(",")]
    if a.batch:
        BATCH.update({L: a.batch for L in layers})
    seeds = list(range(101, 101 + a.seeds))
    if a.phase == "cpu":
        run_cpu(layers, seeds)
    elif a.phase == "gpu":
        run_gpu(layers, seeds, a.tag)
    else:
        report(a.out)


if __name__ == "__main__":
    main()
