#!/usr/bin/env python
"""Gap statistics of tools/fork_probe's kernel trace: per mode, the idle time on the stream
between the first and the second kernel of each pair.  usage: fork_probe.py kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "k_busy" in r["Kernel_Name"]]
names = ["nothing", "event record", "wait old event", "write value", "wait value"]
per = len(rows) // 5
for m in range(5):
    rs = rows[m * per:(m + 1) * per]
    gaps = sorted((int(rs[i + 1]["Start_Timestamp"]) - int(rs[i]["End_Timestamp"])) / 1e3 for i in range(0, len(rs) - 1, 2))
    dur = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rs)
    print(f"{names[m]:16s} gap median {gaps[len(gaps) // 2]:6.2f} us  p10 {gaps[len(gaps) // 10]:6.2f}  "
          f"p90 {gaps[9 * len(gaps) // 10]:6.2f}   (kernel {dur[len(dur) // 2]:.2f} us)")
