#!/usr/bin/env python
"""One step's kernels in launch order from a rocprofv3 kernel trace (run with
DSTAGNN_SIDE_STREAM=0 so durations are not inflated by concurrency), GEMM calls annotated
with the DSTAGNN_GEMM_LOG host lines ("[gemm] ..." per GEMM launch, "[fused] kind= flops=" per
fused kernel that computes GEMM-family products).
usage: step_kernels.py trace.csv gemm_log [step] [--json out.json]

--json writes the GEMM-family roofline as rocprof measured it: every family
call of the step with its duration and algorithmic FLOP, the family's achieved TFLOP/s and
fraction of the fp32 MFMA peak, and the dominant single kernel — bench.py carries these numbers
(roofline.rocprof) when the file's build stamp matches its own library."""
import csv
import hashlib
import json
import os
import re
import sys

PEAK = 157.3  # TFLOP/s, MI355X dense fp32 MFMA (MI355X_MICROARCH.md)
args = [a for a in sys.argv[1:] if not a.startswith("--json")]
jout = None
if "--json" in sys.argv:
    jout = sys.argv[sys.argv.index("--json") + 1]
    args = [a for a in args if a != jout]
rows = sorted(csv.DictReader(open(args[0])), key=lambda r: int(r["Dispatch_Id"]))
lines = open(args[1]).read().splitlines()
logs = [l.strip()[7:] for l in lines if l.startswith("[gemm]")]
fused = [l.strip() for l in lines if l.startswith("[fused]")]
step = int(args[2]) if len(args) > 2 else 2
marks = [i for i, r in enumerate(rows) if "param_prep" in r["Kernel_Name"]]
s0, s1 = marks[step], marks[step + 1]


def is_gemm(name):  # a launch that consumed one "[gemm]" host log line
    return "gemm_f32" in name or "skinny_dw" in name


FUSED_NAMES = ("tat_fused_fwd", "tat_fused_bwd", "gtu_fwd_fused", "gtu_bwd_fused", "gtu_tconv", "gtu_conv_fwd",
               "sat_ln_bwd")


def is_fused(name):
    return any(f in name for f in FUSED_NAMES)


def gemm_flops(log):
    f = 0.0
    for part in log.split("|"):
        m = re.search(r"M=(\d+) N=(\d+) K=(\d+) batch=(\d+)", part)
        if m:
            M, N, K, b = (int(x) for x in m.groups())
            f += 2.0 * M * N * K * b
    return f


gi = sum(1 for r in rows[:s0] if is_gemm(r["Kernel_Name"]))
fi = sum(1 for r in rows[:s0] if is_fused(r["Kernel_Name"]))
tot = 0.0
cat = {}
fam = []
for r in rows[s0:s1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    nm = re.sub(r"\(anonymous namespace\)::|GemmK|\(.*", "", r["Kernel_Name"])[:44]
    extra = ""
    if is_gemm(r["Kernel_Name"]):
        extra = logs[gi] if gi < len(logs) else "?"
        gi += 1
        key = "gemm"
        fam.append({"kernel": nm.strip(), "us": d, "gflop": gemm_flops(extra) / 1e9})
    else:
        key = nm.split("<")[0].replace("void ", "")
        if is_fused(r["Kernel_Name"]):
            fl = fused[fi] if fi < len(fused) else ""
            fi += 1
            m = re.search(r"flops=([0-9.e+]+)", fl)
            extra = fl
            fam.append({"kernel": nm.strip(), "us": d, "gflop": float(m.group(1)) / 1e9 if m else 0.0})
        elif "splitk_reduce" in r["Kernel_Name"]:  # the fold of the GEMM call before it
            fam.append({"kernel": nm.strip(), "us": d, "gflop": 0.0})
    cat[key] = cat.get(key, 0.0) + d
    print(f"{d:7.2f} {nm:44s} {extra}")
print(f"step kernels: {s1 - s0}, busy {tot:.1f} us")
for k, v in sorted(cat.items(), key=lambda kv: -kv[1]):
    print(f"  {v:7.1f} us  {k}")
fus = sum(e["us"] for e in fam)
fgf = sum(e["gflop"] for e in fam)
if fam:
    print(f"GEMM family (rocprof, serialised): {len(fam)} kernels, {fus:.1f} us, {fgf:.3f} GFLOP -> "
          f"{fgf / (fus * 1e-6) / 1e3:.1f} TFLOP/s = {fgf / (fus * 1e-6) / 1e3 / PEAK:.4f} of peak")
if jout:
    def sha(path):
        h = hashlib.sha256()
        with open(path, "rb") as f:
            for chunk in iter(lambda: f.read(1 << 20), b""):
                h.update(chunk)
        return h.hexdigest()[:16]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.environ.get("DSTAGNN_STAMP_LIB", os.path.join(root, "dstagnn_drought_amd", "libdstagnn.so"))
    dom = max((e for e in fam if e["gflop"] > 0), key=lambda e: e["us"], default=None)
    out = {"source": "rocprofv3 --kernel-trace, one serialised step (DSTAGNN_SIDE_STREAM=0), tools/step_kernels.py",
           "build": {"lib_sha256": sha(lib), "ext_sha256": sha(os.path.join(root, "dstagnn_drought_amd", "_C.so"))},
           "peak_tflops": PEAK, "step_kernels": s1 - s0, "step_busy_us": round(tot, 2),
           "family": {"kernels": len(fam), "us": round(fus, 2), "gflop": round(fgf, 4),
                      "achieved_tflops": round(fgf / (fus * 1e-6) / 1e3, 3) if fus else None,
                      "frac": round(fgf / (fus * 1e-6) / 1e3 / PEAK, 4) if fus else None},
           "dominant_kernel": None if dom is None else {
               "kernel": dom["kernel"], "us": round(dom["us"], 2), "gflop": round(dom["gflop"], 4),
               "achieved_tflops": round(dom["gflop"] / (dom["us"] * 1e-6) / 1e3, 3),
               "frac": round(dom["gflop"] / (dom["us"] * 1e-6) / 1e3 / PEAK, 4)},
           "calls": [{"kernel": e["kernel"], "us": round(e["us"], 2), "gflop": round(e["gflop"], 5)} for e in fam]}
    with open(jout, "w") as f:
        json.dump(out, f, indent=1)
