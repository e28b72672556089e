#!/usr/bin/env python
"""Summarise a rocprofv3 kernel-trace CSV: per-kernel totals and one step's launch sequence."""
import csv
import re
import sys
from collections import defaultdict

trace = sys.argv[1]
rows = list(csv.DictReader(open(trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def nm(r):
    return re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])


def dur(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3


agg = defaultdict(lambda: [0, 0.0])
for r in rows:
    a = agg[nm(r)[:90]]
    a[0] += 1
    a[1] += dur(r)
tot = sum(v[1] for v in agg.values())
print(f"total {tot/1e3:.3f} ms over {len(rows)} launches")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"{t/tot*100:5.1f}% {n:5d} x {t/n:8.2f} us  {k}")
if len(sys.argv) > 2:
    marker = sys.argv[2]
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    s0, s1 = starts[-3], starts[-2]
    t0 = int(rows[s0]["Start_Timestamp"])
    step = 0.0
    for r in rows[s0:s1]:
        g = (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"], r["Grid_Size_Z"])
        step += dur(r)
        print(f"{(int(r['Start_Timestamp'])-t0)/1e3:9.1f} {dur(r):8.2f}us {nm(r)[:62]:62s} grid={g}")
    print(f"one step: {len(rows[s0:s1])} launches, busy {step:.1f} us, "
          f"span {(int(rows[s1]['Start_Timestamp'])-t0)/1e3:.1f} us")
