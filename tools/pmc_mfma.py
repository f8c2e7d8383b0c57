"""MFMA utilisation of the prefill GEMMs from PMC counters (one rocprofv3 --pmc pass per counter set).

    export BS_GRAPHS=0   # eager decode steps under counter collection (profiles/r06_rocprof_pmc_segv.txt)
    cd /tmp && rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d OUT -o pmc \
        --output-format csv -- python3 bench.py --cpu-baseline 0 --no-pmc --no-profile --steps 4 --warmup 1
    python tools/pmc_mfma.py OUT

SQ_VALU_MFMA_BUSY_CYCLES is summed over the chip's SIMDs (cycles a SIMD's matrix pipe is busy);
GRBM_GUI_ACTIVE over the 8 XCDs (MI355X_MICROARCH.md, DVFS note).  Utilisation of a dispatch =
MFMA_BUSY / (GUI_ACTIVE / 8 x 1024 SIMDs): the fraction of SIMD-cycles the matrix pipes were busy
while the kernel ran."""
import csv
import os
import sys
from collections import defaultdict

d = sys.argv[1]
files = [os.path.join(dp, f) for dp, _, fs in os.walk(d) for f in fs if f.endswith("counter_collection.csv")]
rows = [r for f in files for r in csv.DictReader(open(f))]
per = defaultdict(lambda: defaultdict(float))
for r in rows:
    per[(r["Kernel_Name"], r.get("Dispatch_Id") or r.get("Correlation_Id"))][r["Counter_Name"]] += float(r["Counter_Value"])
agg = defaultdict(lambda: [0.0, 0.0, 0])
for (k, _), c in per.items():
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
        a = agg[k]
        a[0] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        a[1] += c["GRBM_GUI_ACTIVE"]
        a[2] += 1
for k, (mb, ga, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    if mb <= 0:
        continue
    util = mb / (ga / 8.0 * 1024.0)
    print(f"{k[:90]:90s} dispatches {n:5d}  MFMA busy {mb / n:14.0f}  GUI_ACTIVE/8 {ga / 8 / n:10.0f}  util {util:.3f}")
