#!/usr/bin/env python
"""Per-(kernel, grid) launch counts and average durations from a rocprofv3 kernel trace CSV,
largest total first (separates the configs of one multi-config run by their grid sizes)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
d = collections.defaultdict(list)
for r in rows:
    nm = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:64]
    d[(nm, r["Grid_Size_X"], r["Grid_Size_Y"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{k[0]:64s} grid=({k[1]},{k[2]}) n={len(v):4d} avg={sum(v) / len(v):9.1f} us")
