"""Per-launch HBM traffic of the decode weight GEMVs from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
passes (separate runs).  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per
128-B request of a wide coalesced stream, i.e. half the bytes -> x2; WRITE_SIZE exact.  Units: KB."""
import collections
import csv
import json
import sys


def load(path, counter):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return out


fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE") if len(sys.argv) > 2 else {}
res = {}
tot_f = tot_w = n_tot = 0
for (name, grid), vals in sorted(fetch.items(), key=lambda kv: -sum(kv[1])):
    if "gemv" not in name:
        continue
    vals = vals[len(vals) // 4:]  # skip warm-up dispatches
    f = sum(vals) / len(vals) * 1024 * 2
    wv = write.get((name, grid), [0.0])
    wv = wv[len(wv) // 4:] if len(wv) > 3 else wv
    w = sum(wv) / len(wv) * 1024
    res[f"{name[:40]} grid={grid}"] = {"launches": len(vals), "fetch_bytes": f, "write_bytes": w}
    tot_f += f * len(vals)
    tot_w += w * len(vals)
    n_tot += len(vals)
print(json.dumps({"per_kernel": res, "avg_hbm_bytes_per_gemv_launch": (tot_f + tot_w) / max(1, n_tot)}, indent=1))
