#!/usr/bin/env python3
"""Summarise tools/pmc_step.sh (gpurun_out/pmcs) into profiles/<tag>_block_pmc.json.

* calibration: known bytes of tools/fetch_calib's kernels / their FETCH_SIZE / WRITE_SIZE (KiB
  x 1024) = the correction factor per access width (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2
  of a 16-B-per-lane stream; other widths must be calibrated);
* one benchmark step (the kernels between the 2nd and 3rd param_prep_kernel dispatch: the first
  timed step of `bench.py --steps 3 --warmup 1`, serialised): memory-side bytes per step, raw
  and corrected, for all kernels and for the GEMM family (gemm_f32* + splitk_reduce);
* MFMA: SQ_VALU_MFMA_BUSY_CYCLES and SQ_INSTS_VALU_MFMA_F32 per step against GRBM_GUI_ACTIVE.

usage: pmc_step_summary.py [pmcs_dir] [out_json]
"""
import collections
import csv
import glob
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CALIB_BYTES = 64 << 20
STEP = 1


def rows_of(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def by_dispatch(rows):
    """dispatch id -> (kernel name, {counter: value})"""
    d = {}
    for r in rows:
        did = int(r["Dispatch_Id"])
        nm = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        e = d.setdefault(did, [nm, collections.defaultdict(float)])
        e[1][r["Counter_Name"]] += float(r["Counter_Value"])
    return [d[k] for k in sorted(d)]


def short(nm):
    return re.sub(r"GemmK|\(.*", "", nm).replace("void ", "").split("<")[0]


def gemm_family(nm):
    return "gemm_f32" in nm or "splitk_reduce" in nm


def step_slice(disp, step=STEP):
    marks = [i for i, (nm, _) in enumerate(disp) if "param_prep" in nm]
    if len(marks) < step + 2:
        raise SystemExit(f"only {len(marks)} param_prep dispatches")
    return disp[marks[step]:marks[step + 1]]


def calib(d, counter):
    disp = by_dispatch(rows_of(d))
    f = collections.defaultdict(list)
    for nm, c in disp:
        k = short(nm)
        if c.get(counter):
            f[k].append(CALIB_BYTES / (c[counter] * 1024.0))
    return {k: round(sum(v[1:] or v) / len(v[1:] or v), 3) for k, v in f.items()}


def stamp(d):
    """Build + workload the counters belong to: the library sha the run recorded
    (pmc_step.sh writes build.json on the GPU box), else this tree's, and this tree's HEAD."""
    st = {}
    try:
        with open(os.path.join(d, "build.json")) as fh:
            st.update(json.load(fh))
    except (OSError, ValueError):
        sys.path.insert(0, ROOT)
        from dstagnn_drought_amd._lib import build_stamp
        st.update(build_stamp())
    try:
        st["git_head"] = subprocess.check_output(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"],
                                                 text=True).strip()
    except (OSError, subprocess.CalledProcessError):
        st["git_head"] = None
    return st


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmcs")
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "block_pmc.json")
    cf = calib(os.path.join(d, "calib_fetch"), "FETCH_SIZE")
    cw = calib(os.path.join(d, "calib_write"), "WRITE_SIZE")
    fx = {"x4": cf.get("read_x4"), "x1": cf.get("read_x1"), "glds": cf.get("read_glds")}
    wx = {"x4": cw.get("write_x4"), "x1": cw.get("write_x1")}
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for name, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        for nm, c in step_slice(by_dispatch(rows_of(os.path.join(d, name)))):
            per[short(nm)][ctr] += c.get(ctr, 0.0)
            if name == "fetch":
                cnt[short(nm)] += 1
    for nm, c in step_slice(by_dispatch(rows_of(os.path.join(d, "mfma")))):
        for k, v in c.items():
            per[short(nm)][k] += v
    # the GEMM stages its operands by 4-B-per-lane LDS DMA; everything else is treated with the
    # 16-B-per-lane factor (most of its traffic is wide streaming)
    f_g = fx["glds"] or 2.0
    f_o = fx["x4"] or 2.0
    w_o = wx["x4"] or 1.0

    def tot(pred):
        s = collections.defaultdict(float)
        for k, c in per.items():
            if pred(k):
                for n, v in c.items():
                    s[n] += v
        fetch_b = sum(c["FETCH_SIZE"] * 1024 * (f_g if gemm_family(k) else f_o) for k, c in per.items() if pred(k))
        write_b = sum(c["WRITE_SIZE"] * 1024 * w_o for k, c in per.items() if pred(k))
        return {"launches": sum(v for k, v in cnt.items() if pred(k)),
                "fetch_kib_raw": round(s["FETCH_SIZE"], 1), "write_kib_raw": round(s["WRITE_SIZE"], 1),
                "bytes_corrected": int(fetch_b + write_b),
                "mfma_busy_cycles": s["SQ_VALU_MFMA_BUSY_CYCLES"], "mfma_f32_insts": s["SQ_INSTS_VALU_MFMA_F32"],
                "grbm_gui_active": s["GRBM_GUI_ACTIVE"], "sq_busy_cycles": s["SQ_BUSY_CYCLES"]}

    allk = tot(lambda k: True)
    gem = tot(gemm_family)
    # SQ_VALU_MFMA_BUSY_CYCLES is summed over the 1024 SIMDs; GRBM_GUI_ACTIVE over the 8 XCDs
    # (MI355X_MICROARCH.md): busy fraction = busy / (GUI_ACTIVE / 8 * 1024)
    for t in (allk, gem):
        t["mfma_busy_frac"] = round(t["mfma_busy_cycles"] / max(1.0, t["grbm_gui_active"] / 8 * 1024), 4)
        t["mfma_cycles_per_inst"] = round(t["mfma_busy_cycles"] / max(1.0, t["mfma_f32_insts"]), 2)
    table = []
    for k, c in sorted(per.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"]):
        f = f_g if gemm_family(k) else f_o
        table.append({"kernel": k, "launches": cnt[k], "fetch_MB": round(c["FETCH_SIZE"] * 1024 * f / 1e6, 3),
                      "write_MB": round(c["WRITE_SIZE"] * 1024 * w_o / 1e6, 3),
                      "gui_active": c["GRBM_GUI_ACTIVE"], "mfma_busy_cycles": c["SQ_VALU_MFMA_BUSY_CYCLES"],
                      "mfma_busy_frac": round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, c["GRBM_GUI_ACTIVE"] / 8 * 1024),
                                              4)})
    res = {"source": "tools/pmc_step.sh: rocprofv3 --pmc passes over `bench.py --steps 3 --warmup 1` "
                     "(DSTAGNN_SIDE_STREAM=0); one step = the kernels between the 2nd and 3rd param_prep dispatch",
           "calibration": {"fetch_bytes_per_counted_byte": fx, "write_bytes_per_counted_byte": wx,
                           "applied": {"gemm_fetch": f_g, "other_fetch": f_o, "write": w_o}},
           "build": stamp(d), "workload": os.environ.get("PMC_WORKLOAD", "pems08"),
           "step": allk, "gemm_family": gem, "per_kernel": table}
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_kernel"}, indent=1))


if __name__ == "__main__":
    main()
