#!/usr/bin/env python
"""Per-kernel averages of the pmc_block.sh passes (gpurun_out/pmcb/{a,b,c,d})."""
import csv
import os
import re
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcb"
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for p in "abcd":
    f = os.path.join(root, p, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(anonymous namespace\)::|GemmK|\(.*", "", r["Kernel_Name"]).replace("void ", "")[:40]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if p == "a" and r["Counter_Name"] == "SQ_WAVES":
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
cols = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_WAVE_CYCLES",
        "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
        "FETCH_SIZE", "WRITE_SIZE"]
short = ["waves", "valu/w", "lds/w", "vmr/w", "vmw/w", "cyc/w", "wait%", "iss%", "act%", "ldsconf%", "fetchMB",
         "writeMB"]
print(f"{'kernel':40s} {'n':>4s} {'us':>7s} " + " ".join(f"{s:>8s}" for s in short))
rows = []
for k, d in vals.items():
    def m(c):
        v = d.get(c)
        return sum(v) / len(v) if v else float("nan")
    w = m("SQ_WAVES")
    wc = m("SQ_WAVE_CYCLES")
    us = sum(dur[k]) / len(dur[k]) if dur[k] else float("nan")
    row = [w, m("SQ_INSTS_VALU") / w, m("SQ_INSTS_LDS") / w, m("SQ_INSTS_VMEM_RD") / w, m("SQ_INSTS_VMEM_WR") / w,
           wc / w, 100 * m("SQ_WAIT_ANY") / wc, 100 * m("SQ_WAIT_INST_ANY") / wc, 100 * m("SQ_ACTIVE_INST_ANY") / wc,
           100 * m("SQ_LDS_BANK_CONFLICT") / max(1.0, m("SQ_LDS_IDX_ACTIVE")),
           m("FETCH_SIZE") / 1024, m("WRITE_SIZE") / 1024]
    rows.append((us * len(dur[k]), k, len(dur[k]), us, row))
for tot, k, n, us, row in sorted(rows, key=lambda r: -r[0]):
    print(f"{k:40s} {n:4d} {us:7.1f} " + " ".join(f"{v:8.1f}" for v in row))
