"""Per-shape tile GEMV sweep at batched decode (run on the GPU box): each arm sets BS_TILES_CFG for the
four block matrices of a model at once, runs bench.py under a rocprofv3 kernel trace and reports the
median duration of each shape's tile GEMV (identified by its position around the attention kernel).

    python tools/tiles_sweep.py bloom-7b1 32 "QKV T,KS,W|DENSE|FC1|FC2" ...
"""
import csv
import glob
import os
import shutil
import statistics
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_inference_demo_amd import config  # noqa: E402


def main():
    model, batch = sys.argv[1], int(sys.argv[2])
    m = config.get(model)
    h = m.hidden
    shapes = [("qkv", 3 * h, h), ("dense", h, h), ("fc1", 4 * h, h), ("fc2", h, 4 * h)]
    for arm in sys.argv[3:]:
        parts = arm.split("|")
        cfg = "/".join(f"{n},{k},{p}" for (name, n, k), p in zip(shapes, parts) if p)
        d = f"gpurun_out/tsw_{abs(hash(arm)) % 10**8}"
        shutil.rmtree(d, ignore_errors=True)
        env = dict(os.environ, **{"BS_TILES_CFG" if batch > 16 else "BS_TILES_CFG1": cfg})
        cmd = ["timeout", "-k", "10", "300", "rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", d, "-o",
               "run", "--", sys.executable, "bench.py", "--cpu-baseline", "0", "--no-pmc", "--no-profile", "--model",
               model, "--batch", str(batch), "--prompt", "128", "--steps", "24", "--warmup", "4"]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True)
        if r.returncode != 0:
            print(arm, "FAILED", r.stderr[-400:])
            sys.exit(1)
        val = r.stdout.strip().splitlines()[-1]
        f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
        rows = sorted(csv.DictReader(open(f)), key=lambda x: int(x["Start_Timestamp"]))
        names = [x["Kernel_Name"] for x in rows]
        dur = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3 for x in rows]
        got = {s[0]: [] for s in shapes}
        for i, nm in enumerate(names):
            if "attn_decode" not in nm:
                continue
            seq = [j for j in range(i - 3, min(len(rows), i + 5)) if ("gemv_tiles" in names[j] or "gemv_ldsw" in names[j])]
            before = [j for j in seq if j < i]
            after = [j for j in seq if j > i]
            if before and len(after) >= 3:
                got["qkv"].append(dur[before[-1]])
                got["dense"].append(dur[after[0]])
                got["fc1"].append(dur[after[1]])
                got["fc2"].append(dur[after[2]])
        out = []
        for (name, n, k), p in zip(shapes, parts):
            v = got[name]
            med = statistics.median(v) if v else float("nan")
            gbs = n * k * 2 / (med * 1e-6) / 1e9
            out.append(f"{name} [{p or 'table'}] {med:6.2f} us {gbs:6.0f} GB/s")
        import json
        tps = json.loads(val)["value"]
        print(f"{tps:8.1f} tok/s | " + " | ".join(out), flush=True)
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
