#!/usr/bin/env python
"""CPU column of every BASELINE.json config (BASELINE.md "CPU-baseline plan on the MI355X box";
VERDICT r4 item 7): the oracle — oracle/dstagnn_ref.py, the literal restatement of the
reference's loops (hoist=False: the T x K Python loop of cheb_conv_withSAt :117-133) — timed on
this host's cores (torch.set_num_threads(host cores), count printed), the same synthetic graphs /
init distribution as tools/bench_configs.py, inner block fwd+bwd (d_out, d_re_At seeded), plus
the PEMS04 full model (make_model nb_block=4 + the head, SmoothL1 backward) as BASELINE.md lists.

Samples (median of >= 5 after 2 warm-ups): PEMS04 block / model B=32, PEMS08 B=32,
PEMS07 B=12 — 2 warm-ups, median of 5; GAMBIA B=1 and SYN B=1 (20-40 s per iteration, ~20 GB RSS) —
1 warm-up, median of 3 (stated in each record's "sample").  The oracle is test infrastructure:
this tool only times it, beside the GPU figures of tools/bench_configs.py.
Prints one JSON object {config: {value, unit, cores, kind, sample, B}}."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import dstagnn_ref as ref  # noqa: E402
from tools.bench_configs import CONFIGS  # noqa: E402

PLAN = {  # name: (B, warmup, iters)
    "PEMS04": (32, 2, 5), "PEMS04_model": (32, 2, 5), "PEMS08": (32, 2, 5), "PEMS07": (12, 2, 5),
    "GAMBIA": (1, 1, 3), "SYN": (1, 1, 3),
}


def host_cores():
    for k in ("OMP_NUM_THREADS", "MAX_JOBS"):  # the box's CPU share (os.cpu_count() is the machine's)
        v = os.environ.get(k)
        if v and v.isdigit() and int(v) > 0:
            return int(v)
    return os.cpu_count() or 1


def graph(N, K):
    rs = np.random.RandomState(0)
    tmd = np.eye(N)
    pa = np.zeros((N, N))
    for i in range(N):
        tmd[i, rs.choice(N, 2, replace=False)] = 1.0
        pa[i, rs.choice(N, 4, replace=False)] = 1.0
    Lt = ref.scaled_laplacian(tmd)
    cheb = [torch.from_numpy(p).float() for p in ref.cheb_polynomials(Lt, K)][:K]
    return cheb, torch.from_numpy(pa).float()


def time_it(fn, warmup, iters):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


def run(name):
    base = name.split("_")[0]
    N, T, K, h, D, dk, C, _ = CONFIGS[base]
    B, warmup, iters = PLAN[name]
    gen = torch.Generator().manual_seed(0)
    cheb, apa = graph(N, K)
    dims = dict(n_heads=h, d_k=dk, d_v=dk, K=K)
    if name.endswith("_model"):
        blocks = [ref.random_block_params(gen, 1 if i == 0 else C, 1 if i == 0 else C, K, C, N, T, D, dk, dk, h)
                  for i in range(4)]
        final = {"final_conv.weight": torch.randn(128, 4 * T, 1, C, generator=gen) * 0.02,
                 "final_conv.bias": torch.zeros(128), "final_fc.weight": torch.randn(12, 128, generator=gen) * 0.05,
                 "final_fc.bias": torch.zeros(12)}
        x = torch.randn(B, N, 1, T, generator=gen)
        y = torch.randn(B, N, 12, generator=gen)
        leaves = [v.requires_grad_(True) for p in blocks for v in p.values()] + \
                 [v.requires_grad_(True) for v in final.values()]

        def fn():
            for v in leaves:
                v.grad = None
            out = ref.model_forward(blocks, final, x, cheb, apa, dims, hoist=False)
            torch.nn.functional.smooth_l1_loss(out, y).backward()
        what = "make_model nb_block=4 (first block F=1) + head, SmoothL1 fwd+bwd"
    else:
        p = ref.random_block_params(gen, C, C, K, C, N, T, D, dk, dk, h)
        x = torch.randn(B, N, C, T, generator=gen)
        res = torch.randn(B, 1, h, T, T, generator=gen)
        go = torch.randn(B, N, C, T, generator=gen)
        gr = torch.randn(B, C, h, T, T, generator=gen)

        def fn():
            ref.block_forward_backward(p, x, res, cheb, apa, dims, go, gr, hoist=False)
        what = "inner DSTAGNN_block fwd+bwd"
    med, ts = time_it(fn, warmup, iters)
    return {"value": round(B / med, 4), "unit": "samples/s", "cores": torch.get_num_threads(), "kind": "port", "B": B,
            "sample": f"{what}, B={B}, N={N}, T={T}, K={K}, h={h}: median of {iters} timed iterations after "
                      f"{warmup} warm-up(s) (oracle, literal T x K loop); per-iteration s "
                      f"{', '.join(f'{t:.2f}' for t in ts)}"}


def main():
    torch.set_num_threads(host_cores())
    print(f"[cpu_configs] {torch.get_num_threads()} threads", file=sys.stderr, flush=True)
    names = sys.argv[1:] or list(PLAN)
    out = {}
    for n in names:
        t0 = time.time()
        out[n] = run(n)
        print(f"[cpu_configs] {n}: {out[n]['value']} samples/s ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
