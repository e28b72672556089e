#!/usr/bin/env python
"""One training step's launch sequence from a rocprofv3 kernel-trace CSV, delimited by
consecutive launches of a marker kernel (default: param_prep_kernel, one per forward)."""
import csv
import re
import sys

trace = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "param_prep"
which = int(sys.argv[3]) if len(sys.argv) > 3 else 6
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
s0, s1 = idx[which], idx[which + 1]
t0 = int(rows[s0]["Start_Timestamp"])
busy = 0.0
for r in rows[s0:s1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy += d
    g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
    name = re.sub(r"GemmK|\(anonymous namespace\)::", "", r["Kernel_Name"])[:58]
    st = (int(r["Start_Timestamp"]) - t0) / 1e3
    print(f"{st:8.1f} {d:7.2f} {name:58s} g={g},{r['Grid_Size_Y']} q={r.get('Queue_Id', '')}")
span = (int(rows[s1]["Start_Timestamp"]) - t0) / 1e3
print(f"{s1 - s0} launches, busy {busy:.1f} us, span {span:.1f} us")
