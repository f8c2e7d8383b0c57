"""MFMA utilisation per (shape, variant) of tools/attn_prefill_bench from one rocprofv3 --pmc pass: the bench launches
every (shape, variant) PER times in a row (1 + 7 x 20), so the attention dispatches, in dispatch order, are cut into
groups of PER and labelled with the bench log's lines in order.

    python tools/pmc_mfma_seq.py PMC_DIR BENCH_LOG [PER]"""
import csv
import os
import sys
from collections import defaultdict

d, log = sys.argv[1], sys.argv[2]
per_n = int(sys.argv[3]) if len(sys.argv) > 3 else 141
files = [os.path.join(dp, f) for dp, _, fs in os.walk(d) for f in fs if f.endswith("counter_collection.csv")]
disp = defaultdict(dict)
names = {}
for f in files:
    for r in csv.DictReader(open(f)):
        if "attn_prefill" not in r["Kernel_Name"]:
            continue
        k = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        disp[k][r["Counter_Name"]] = disp[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[k] = r["Kernel_Name"]
labels = [l.rstrip() for l in open(log) if "us/launch" in l]
ids = sorted(disp)
for gi in range(len(ids) // per_n):
    grp = ids[gi * per_n:(gi + 1) * per_n]
    mb = sum(disp[i].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for i in grp)
    ga = sum(disp[i].get("GRBM_GUI_ACTIVE", 0.0) for i in grp)
    util = mb / (ga / 8.0 * 1024.0) if ga else float("nan")
    lab = labels[gi][:75] if gi < len(labels) else "?"
    print(f"{lab:75s} util {util:.3f}  {names[grp[0]][:40]}")
