"""Per-(kernel, grid) duration summary of a rocprofv3 kernel trace (decode vs prefill split by grid).
    python tools/prof_split.py gpurun_out/prof_x [last_n_kernels]"""
import csv
import glob
import statistics
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
if len(sys.argv) > 2:
    rows = rows[-int(sys.argv[2]):]
agg = {}
for r in rows:
    key = (r["Kernel_Name"][:48], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    agg.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in agg.values())
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0]:48s} grid {k[1]:>7}x{k[2]:>3}x{k[3]:>3} n={len(v):5d} med {statistics.median(v):8.2f} us  "
          f"total {sum(v):9.1f} us ({100 * sum(v) / tot:4.1f}%)")
