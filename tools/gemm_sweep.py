#!/usr/bin/env python
"""Tuning sweep for the strided f32-MFMA GEMM (dstagnn_gemm_f32) on the DSTAGNN block's
GEMM shapes (PEMS08, B=32).  Each (tile config, implementation) runs in its own subprocess
because the overrides (DSTAGNN_GEMM_CFG / DSTAGNN_GEMM_NS) are read once per process;
every run is checked against torch.bmm.

    python tools/gemm_sweep.py            # full sweep, prints a table
    python tools/gemm_sweep.py --child    # (internal) one config
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# name, M, N, K, batch, A k-contiguous?, B n-contiguous?
SHAPES = [
    ("qkv", 12288, 96, 170, 1, True, False),
    ("fc", 12288, 170, 96, 1, True, False),
    ("preconv", 5440, 512, 384, 1, False, False),
    ("sat_proj", 5440, 96, 512, 1, True, False),
    ("sat_scores", 170, 170, 32, 96, True, False),
    ("cheb_agg", 170, 384, 510, 32, False, True),
    ("gtu7", 32640, 64, 224, 1, False, False),
    ("gtu3", 54400, 64, 96, 1, False, False),
    ("fcmy", 174080, 12, 24, 1, True, False),
    ("gtu_dX7", 65280, 32, 448, 1, False, False),
    ("cheb_dW", 170, 170, 384, 96, True, False),
    ("cheb_dxth", 170, 384, 170, 96, True, True),
    ("dthcat", 32, 96, 65280, 1, False, False),
    ("sat_dW", 96, 512, 5440, 1, False, True),
    ("dZd", 5440, 512, 96, 1, True, True),
    ("dWp", 512, 384, 5440, 1, False, False),
    ("dO", 384, 5440, 512, 1, False, False),
    ("gtu_dW7", 64, 224, 32640, 1, False, False),
    ("fcmy_dW", 12, 24, 174080, 1, False, True),
]
# steady-state probes (not block shapes): large square GEMMs, all operand layouts
BIG = [
    ("big_tn", 4096, 4096, 2048, 1, True, False),
    ("big_nn", 4096, 4096, 2048, 1, False, False),
    ("big_nt", 4096, 4096, 2048, 1, False, True),
]
# occupancy probes: 64x64 tiles, N=512 (8 n-tiles), K=384 -> M/64*8 blocks
BIG += [(f"occ{m // 64 * 8}", m, 512, 384, 1, False, False) for m in (2048, 4096, 6144, 8192, 16384, 32768)]
# long-series / large-graph configs (GAMBIA B=4: N=2139, T=144; SYN B=32: N=4096, T=24)
LARGE = [
    ("gam_dX7", 1232064, 32, 448, 1, False, False),
    ("gam_fcmy", 273792, 144, 420, 1, True, False),
    ("gam_dG", 273792, 420, 144, 1, True, True),
    ("syn_dX7", 1048576, 32, 448, 1, False, False),  # M cut to keep a dense A under 2^30 floats
]
if os.environ.get("DSTAGNN_SWEEP_BIG"):
    SHAPES = SHAPES + BIG
if os.environ.get("DSTAGNN_SWEEP_LARGE"):
    SHAPES = SHAPES + LARGE


def child(iters, only=None):
    import torch
    from dstagnn_drought_amd import _lib
    ops = _lib.load()
    res = {}
    for name, M, N, K, batch, akc, bnc in SHAPES:
        if only and name not in only.split(","):
            continue
        A = torch.randn(batch, M, K, device="cuda") if akc else torch.randn(batch, K, M, device="cuda")
        B = torch.randn(batch, K, N, device="cuda") if bnc else torch.randn(batch, N, K, device="cuda")
        C = torch.empty(batch, M, N, device="cuda")
        am, ak = ((0, K), (0, 1)) if akc else ((0, 1), (0, M))
        bk, bn = ((0, N), (0, 1)) if bnc else ((0, 1), (0, K))
        maps = _lib.gemm_maps(am, ak, (0, M * K), bk, bn, (0, K * N), (0, N), (0, 1), (0, M * N))

        def run():
            ops.gemm_f32(A, B, C, [M, N, K, batch], maps, [0, 0, 0], 1.0, 0.0, None, 1, False)
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / iters * 1e3
        if os.environ.get("DSTAGNN_GEMM_CHECK"):
            ref = torch.bmm(A if akc else A.transpose(1, 2), B if bnc else B.transpose(1, 2))
            err = float((C - ref).abs().max() / ref.abs().max())
            assert err < 1e-5, (name, err)
        res[name] = us
    print(json.dumps(res))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    # spec = <tile config | auto>:<LDS pipeline stages: 2, 3, or auto>
    ap.add_argument("--configs", default="auto:auto,0:2,1:2,2:2")
    ap.add_argument("--only", default=None)
    ap.add_argument("--big", action="store_true", help="add large square steady-state probes")
    ap.add_argument("--large", action="store_true", help="add the GAMBIA / SYN large-M shapes")
    args = ap.parse_args()
    global SHAPES
    if args.big:
        os.environ["DSTAGNN_SWEEP_BIG"] = "1"
        SHAPES = SHAPES + BIG
    if args.large:
        os.environ["DSTAGNN_SWEEP_LARGE"] = "1"
        SHAPES = SHAPES + LARGE
    if args.child:
        child(args.iters, args.only)
        return
    table = {}
    for spec in args.configs.split(","):
        cfg, ns = spec.split(":")
        env = dict(os.environ)
        if ns != "auto":
            env["DSTAGNN_GEMM_NS"] = ns
        if cfg != "auto":
            env["DSTAGNN_GEMM_CFG"] = cfg
        env["DSTAGNN_GEMM_CHECK"] = "" if os.environ.get("DSTAGNN_NOCHECK") else "1"
        cmd = [sys.executable, __file__, "--child", "--iters", str(args.iters)]
        if args.only:
            cmd += ["--only", args.only]
        out = subprocess.run(cmd, env=env,
                             capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(spec, "FAILED", out.stderr[-2000:], flush=True)
            continue
        table[spec] = json.loads(out.stdout.strip().splitlines()[-1])
        print(spec, "done", flush=True)
    specs = list(table)
    print(f"{'shape':12s} {'GFLOP':>7s} " + " ".join(f"{s:>9s}" for s in specs) + "   best TF/s")
    for name, M, N, K, batch, _, _ in SHAPES:
        if args.only and name not in args.only.split(","):
            continue
        gf = 2.0 * M * N * K * batch / 1e9
        row = [table[s].get(name, float('nan')) for s in specs]
        best = min(row)
        print(f"{name:12s} {gf:7.3f} " + " ".join(f"{v:9.1f}" for v in row) + f"   {gf / best * 1e3:7.1f}")


if __name__ == "__main__":
    main()
