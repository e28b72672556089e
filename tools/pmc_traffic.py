#!/usr/bin/env python3
"""HBM traffic of the hot kernel from the separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes
(tools/pmc.sh) -> profiles/hot_kernel_traffic.json, read by bench.py's roofline.traffic.

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch (TCC_EA0 request counters).  The guide's
½-count correction (MI355X_MICROARCH.md, HBM section) is calibrated for 16-B-per-lane streaming
reads; the GEMM reads one dword per lane, a width the guide calls uncalibrated, so the raw counts
are reported as they are, with the algorithmic bytes beside them.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(pass_dir, counter, needle):
    vals = []
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter and needle in row["Kernel_Name"]:
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    pmc = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc")
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "hot_kernel_traffic.json")
    needle = "gemm_f32_hot_kernel"
    fetch = per_launch(os.path.join(pmc, "fetch"), "FETCH_SIZE", needle)
    write = per_launch(os.path.join(pmc, "write"), "WRITE_SIZE", needle)
    if not fetch or not write:
        sys.exit(f"no {needle} rows in {pmc}/fetch or {pmc}/write")
    # drop the first launch (cold caches after allocation), average the rest
    f = fetch[1:] or fetch
    w = write[1:] or write
    fk, wk = sum(f) / len(f), sum(w) / len(w)
    # pre_conv forward GEMM at the bench shape: O (B*N x F*T) . Wp^T (F*T x D) -> (B*N x D)
    B, N, FT, D = 32, 170, 32 * 12, 512
    alg = 4 * (B * N * FT + FT * D + B * N * D)
    res = {
        "kernel": needle,
        "launches": {"fetch": len(fetch), "write": len(write)},
        "fetch_kib": round(fk, 1), "write_kib": round(wk, 1),
        "bytes_per_launch": int(round((fk + wk) * 1024)),
        "algorithmic_bytes_per_launch": alg,
        "correction": "none (dword-per-lane loads: the guide's x2 FETCH_SIZE correction is for 16 B/lane streams)",
    }
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
