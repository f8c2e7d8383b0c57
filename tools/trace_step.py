"""Summarise one graph-replayed decode step from a rocprofv3 kernel trace (set_past_kernel marks steps)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
names = [r['Kernel_Name'] for r in rows]
st = [int(r['Start_Timestamp']) for r in rows]
en = [int(r['End_Timestamp']) for r in rows]
sp = [i for i, n in enumerate(names) if n.startswith('set_past')]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(sp) // 2
i0, i1 = sp[k], sp[k + 1]
print(f"graph replays {len(sp)}; step {k}: span {(st[i1] - st[i0]) / 1e3:.1f} us, {i1 - i0} kernels")
d = collections.defaultdict(lambda: [0, 0])
for i in range(i0, i1):
    key = (names[i][:48], rows[i]['Grid_Size_X'], rows[i]['Workgroup_Size_X'])
    d[key][0] += en[i] - st[i]
    d[key][1] += 1
for key, v in sorted(d.items(), key=lambda kv: -kv[1][0]):
    print(f"  {key[0]:48s} grid {key[1]:>8s} wg {key[2]:>5s}  n={v[1]:3d}  total {v[0] / 1e3:8.1f} us  avg {v[0] / v[1] / 1e3:7.2f}")
busy = sum(en[i] - st[i] for i in range(i0, i1))
print(f"  kernel-busy {busy / 1e3:.1f} us of {(st[i1] - st[i0]) / 1e3:.1f}")
