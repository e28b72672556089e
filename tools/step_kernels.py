#!/usr/bin/env python
"""One step's kernels in launch order from a rocprofv3 kernel trace (run with
DSTAGNN_SIDE_STREAM=0 so durations are not inflated by concurrency), GEMM calls annotated
with the DSTAGNN_GEMM_LOG host lines.  usage: step_kernels.py trace.csv gemm_log [step]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Dispatch_Id"]))
logs = [l.strip()[7:] for l in open(sys.argv[2]) if l.startswith("[gemm]")]
step = int(sys.argv[3]) if len(sys.argv) > 3 else 2
marks = [i for i, r in enumerate(rows) if "param_prep" in r["Kernel_Name"]]
s0, s1 = marks[step], marks[step + 1]
def is_gemm(name):  # a launch that consumed one "[gemm]" host log line
    return "gemm_f32" in name or "skinny_dw" in name


gi = sum(1 for r in rows[:s0] if is_gemm(r["Kernel_Name"]))
tot = 0.0
cat = {}
for r in rows[s0:s1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    nm = re.sub(r"\(anonymous namespace\)::|GemmK|\(.*", "", r["Kernel_Name"])[:44]
    extra = ""
    if is_gemm(r["Kernel_Name"]):
        extra = logs[gi] if gi < len(logs) else "?"
        gi += 1
        key = "gemm"
    else:
        key = nm.split("<")[0].replace("void ", "")
    cat[key] = cat.get(key, 0.0) + d
    print(f"{d:7.2f} {nm:44s} {extra}")
print(f"step kernels: {s1 - s0}, busy {tot:.1f} us")
for k, v in sorted(cat.items(), key=lambda kv: -kv[1]):
    print(f"  {v:7.1f} us  {k}")
