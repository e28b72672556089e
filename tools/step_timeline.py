#!/usr/bin/env python
"""One step's kernel timeline from a rocprofv3 kernel trace of a normal (multi-stream) run:
per-stream busy time, the union of busy intervals, the step span and the idle gaps, and the
kernels in start order with their stream.  usage: step_timeline.py trace.csv [step]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
step = int(sys.argv[2]) if len(sys.argv) > 2 else 2
marks = [i for i, r in enumerate(rows) if "param_prep" in r["Kernel_Name"]]
s0, s1 = marks[step], marks[step + 1]
ks = rows[s0:s1]
t0 = int(ks[0]["Start_Timestamp"])
span = int(rows[s1]["Start_Timestamp"]) - t0
busy = {}
last = {}
iv = []
for r in ks:
    a, b = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    q = r["Queue_Id"]
    busy[q] = busy.get(q, 0) + b - a
    last[q] = max(last.get(q, 0), b)
    iv.append((a, b))
    nm = re.sub(r"\(anonymous namespace\)::|dsgemm::|GemmK|\(.*|void ", "", r["Kernel_Name"])[:40]
    print(f"q{q:>2s} {a / 1e3:8.2f} {b / 1e3:8.2f} {(b - a) / 1e3:7.2f}  {nm}")
iv.sort()
union, cur = 0, None
gaps = []
for a, b in iv:
    if cur is None or a > cur[1]:
        if cur is not None:
            union += cur[1] - cur[0]
            gaps.append(a - cur[1])
        cur = [a, b]
    else:
        cur[1] = max(cur[1], b)
union += cur[1] - cur[0]
print(f"step span {span / 1e3:.1f} us, kernels {len(ks)}, union busy {union / 1e3:.1f} us, "
      f"idle {(span - union) / 1e3:.1f} us in {len(gaps)} gaps (mean {sum(gaps) / max(1, len(gaps)) / 1e3:.2f} us)")
for q, v in busy.items():
    print(f"  queue {q}: busy {v / 1e3:.1f} us, last kernel ends at {last[q] / 1e3:.1f} us")
print(f"  the step's last kernel is on queue {max(last, key=last.get)}")
