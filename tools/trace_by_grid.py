"""Average duration per (kernel, grid) from a rocprofv3 kernel_trace.csv (a measurement aid: the
prefill GEMMs of one template differ only in their grid).  python tools/trace_by_grid.py DIR [substr]"""
import csv
import os
import sys
from collections import defaultdict

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
files = [os.path.join(dp, f) for dp, _, fs in os.walk(d) for f in fs if f.endswith("kernel_trace.csv")]
agg = defaultdict(list)
for f in files:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if pat not in k:
            continue
        grid = (r.get("Grid_Size_X") or r.get("Grid_Size"), r.get("Grid_Size_Y", ""), r.get("Workgroup_Size_X") or r.get("Workgroup_Size"))
        agg[(k[:60], grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (k, grid), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{k:60s} grid {grid}  n={len(v):5d}  avg {sum(v) / len(v):8.2f} us  med {v[len(v) // 2]:8.2f}  min {v[0]:8.2f}")
