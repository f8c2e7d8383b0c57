"""Per-kernel averages of every PMC counter in a rocprofv3 --pmc output directory (one line per
kernel, counters averaged over its dispatches).  A measurement aid.

    python tools/pmc_table.py OUT [kernel-substring]
"""
import csv
import os
import sys
from collections import defaultdict

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
files = [os.path.join(dp, f) for dp, _, fs in os.walk(d) for f in fs if f.endswith("counter_collection.csv")]
rows = [r for f in files for r in csv.DictReader(open(f))]
per = defaultdict(lambda: defaultdict(float))
for r in rows:
    per[(r["Kernel_Name"], r.get("Dispatch_Id") or r.get("Correlation_Id"))][r["Counter_Name"]] += float(r["Counter_Value"])
agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(int)
for (k, _), c in per.items():
    if pat not in k:
        continue
    cnt[k] += 1
    for n, v in c.items():
        agg[k][n] += v
for k in sorted(agg, key=lambda k: -cnt[k]):
    vals = "  ".join(f"{n}={v / cnt[k]:.4g}" for n, v in sorted(agg[k].items()))
    print(f"{k[:70]:70s} n={cnt[k]}  {vals}")
