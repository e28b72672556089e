#!/usr/bin/env python
"""Per-queue busy time and overlap of one step from a rocprofv3 kernel trace taken WITH the
side stream: tells whether the step is bound by one chain or by the sum of both."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker = "param_prep"
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
which = int(sys.argv[2]) if len(sys.argv) > 2 else 6
s0, s1 = idx[which], idx[which + 1]
t0 = int(rows[s0]["Start_Timestamp"])
t1 = int(rows[s1]["Start_Timestamp"])
busy = {}
ivals = []
for r in rows[s0:s1]:
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r["Queue_Id"]
    busy[q] = busy.get(q, 0) + (b - a)
    ivals.append((a, b))
ivals.sort()
union, cur_a, cur_b = 0, None, None
for a, b in ivals:
    if cur_b is None or a > cur_b:
        if cur_b is not None:
            union += cur_b - cur_a
        cur_a, cur_b = a, b
    else:
        cur_b = max(cur_b, b)
union += cur_b - cur_a
span = t1 - t0
print(f"step span {span / 1e3:.1f} us; any-kernel-running {union / 1e3:.1f} us; idle {(span - union) / 1e3:.1f} us")
for q, v in sorted(busy.items()):
    print(f"  queue {q}: busy {v / 1e3:.1f} us")
