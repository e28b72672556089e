#!/usr/bin/env python
"""GEMM lab: time dstagnn::gemm_f32 on arbitrary shapes, optionally for several library builds
(tools/variant_build.sh <name> ...) in one box session, interleaved, each in its own process
(LD_LIBRARY_PATH=scratch/<name> makes _C.so load that build).  Also times torch.mm (hipBLASLt /
rocBLAS fp32, no TF32) on the same operands as a library reference point.

    python tools/gemm_lab.py --shapes 5440x512x384:nn,5440x512x768:nn --variants base,ns3 --rounds 3

shape = MxNxK[xbatch]:<a><b>  a: t = A k-contiguous (M x K row-major), n = m-contiguous (K x M);
                              b: n = B n-contiguous (K x N row-major), t = k-contiguous (N x K)
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse(spec):
    dims, lay = spec.split(":") if ":" in spec else (spec, "tt")
    v = [int(x) for x in dims.split("x")]
    M, N, K = v[:3]
    batch = v[3] if len(v) > 3 else 1
    return M, N, K, batch, lay[0] == "t", lay[1] == "n"


def child(shapes, iters, torch_ref):
    import torch
    from dstagnn_drought_amd import _lib
    ops = _lib.load()
    out = {}
    for spec in shapes:
        M, N, K, batch, akc, bnc = parse(spec)
        g = torch.Generator(device="cuda").manual_seed(1)
        A = torch.rand(batch, M, K, device="cuda", generator=g) * 2 - 1 if akc else \
            torch.rand(batch, K, M, device="cuda", generator=g) * 2 - 1
        B = torch.rand(batch, K, N, device="cuda", generator=g) * 2 - 1 if bnc else \
            torch.rand(batch, N, K, device="cuda", generator=g) * 2 - 1
        C = torch.empty(batch, M, N, device="cuda")
        am, ak = ((0, K), (0, 1)) if akc else ((0, 1), (0, M))
        bk, bn = ((0, N), (0, 1)) if bnc else ((0, 1), (0, K))
        maps = _lib.gemm_maps(am, ak, (0, M * K), bk, bn, (0, K * N), (0, N), (0, 1), (0, M * N))

        def run():
            ops.gemm_f32(A, B, C, [M, N, K, batch], maps, [0, 0, 0], 1.0, 0.0, None, 1, False)

        def timed(fn):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / iters * 1e3

        us = timed(run)
        ref = torch.bmm(A if akc else A.transpose(1, 2), B if bnc else B.transpose(1, 2))
        err = float((C - ref).abs().max() / ref.abs().max())
        rec = {"us": us, "err": err}
        if torch_ref:
            torch.backends.cuda.matmul.allow_tf32 = False
            a_ = A if akc else A.transpose(1, 2)
            b_ = B if bnc else B.transpose(1, 2)
            rec["torch_us"] = timed(lambda: torch.bmm(a_, b_))
        out[spec] = rec
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", required=True)
    ap.add_argument("--variants", default="base",
                    help="comma list of <lib>[+ENV=VAL...]: lib base = the in-tree library, else scratch/<lib>")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--torch-ref", action="store_true")
    a = ap.parse_args()
    shapes = a.shapes.split(",")
    if a.child:
        return child(shapes, a.iters, a.torch_ref)
    res = {}
    for r in range(a.rounds):
        for v in a.variants.split(","):
            env = dict(os.environ)
            lib, *kv = v.split("+")  # <lib dir | base>[+ENV=VAL...]
            for item in kv:
                key, val = item.split("=", 1)
                env[key] = val
            if lib != "base":
                env["LD_LIBRARY_PATH"] = os.path.join(ROOT, "scratch", lib) + ":" + env.get("LD_LIBRARY_PATH", "")
            cmd = [sys.executable, __file__, "--child", "--shapes", a.shapes, "--iters", str(a.iters)]
            if a.torch_ref and r == 0 and v == a.variants.split(",")[0]:
                cmd.append("--torch-ref")
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=150)
            if p.returncode != 0:
                print(v, "FAILED", p.stderr[-1500:], flush=True)
                continue
            d = json.loads(p.stdout.strip().splitlines()[-1])
            for s, rec in d.items():
                res.setdefault(s, {}).setdefault(v, []).append(rec["us"])
                if "torch_us" in rec:
                    res[s]["torch"] = [rec["torch_us"]]
                if not rec["err"] < 1e-5:
                    print(f"WRONG RESULT: {v} {s} rel err {rec['err']:.3e}", flush=True)
            print(f"round {r} {v} done", flush=True)
    vs = a.variants.split(",")
    for i, v in enumerate(vs):
        print(f"  v{i} = {v}")
    print(f"{'shape':28s} {'GFLOP':>7s} " + " ".join(f"{'v%d' % i:>8s}" for i in range(len(vs))) + f" {'torch':>8s}   (median us; TF/s of best)")
    for s in shapes:
        M, N, K, batch, _, _ = parse(s)
        gf = 2.0 * M * N * K * batch / 1e9
        meds = [statistics.median(res.get(s, {}).get(v, [float("nan")])) for v in vs]
        t = res.get(s, {}).get("torch", [float("nan")])[0]
        best = min(meds)
        print(f"{s:28s} {gf:7.3f} " + " ".join(f"{m:8.1f}" for m in meds) + f" {t:8.1f}   {gf / best * 1e3:6.1f}")


if __name__ == "__main__":
    main()
