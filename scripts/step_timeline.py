#!/usr/bin/env python
"""One bench step from a rocprofv3 kernel trace: per-stream busy time and the main
stream's kernel sequence with gaps (window = between two consecutive tail_fwd launches,
i.e. one backward + the next forward).

    python scripts/step_timeline.py gpurun_out/prof/run_kernel_trace.csv [step_index]
"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = int(sys.argv[2]) if len(sys.argv) > 2 else -3
marks = [int(r["Start_Timestamp"]) for r in rows if "tail_fwd_kernel" in r["Kernel_Name"]]
t0, t1 = marks[idx - 1], marks[idx]
win = [r for r in rows if t0 <= int(r["Start_Timestamp"]) < t1]


def nm(r):
    s = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
    s = re.sub(r"\(.*", "", s)
    return s[:60]


print(f"window {(t1 - t0) / 1e3:.1f} us, {len(win)} kernels")
streams = sorted(set(r["Stream_Id"] for r in win))
for sid in streams:
    ks = [r for r in win if r["Stream_Id"] == sid]
    busy, last = 0, t0
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        s = max(s, last)
        if e > s:
            busy += e - s
            last = e
    print(f"stream {sid}: {len(ks)} kernels, busy {busy / 1e3:.1f} us")
main = max(streams, key=lambda sid: sum(1 for r in win if r["Stream_Id"] == sid and "tail_fwd" in r["Kernel_Name"]) * 0
           + sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win if r["Stream_Id"] == sid))
if len(sys.argv) > 3:
    main = sys.argv[3]
print(f"--- stream {main} sequence (offset us, duration us, gap before us)")
prev_end = t0
for r in win:
    if r["Stream_Id"] != main:
        continue
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {(s - prev_end) / 1e3:6.1f}  {nm(r)}")
    prev_end = e
