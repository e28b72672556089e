#!/usr/bin/env python
"""fwd+bwd throughput of one inner DSTAGNN_block at every BASELINE.json config (SURVEY.md
§8(d) sizes and batches), train mode, synthetic graphs/inputs, inputs resident in HBM.
Prints one JSON object: samples/s, ms/step and the fraction of the fp32 block roofline
(§8(d) algorithmic FLOP per sample, sparse T_k count)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK = 157.3e12
CONFIGS = {  # name: (N, T, K, h, D, dk, C, B)
    "PEMS08": (170, 12, 3, 3, 512, 32, 32, 32),
    "PEMS04": (307, 12, 3, 3, 512, 32, 32, 32),
    "PEMS07": (883, 12, 3, 4, 512, 32, 32, 12),
    "GAMBIA": (2139, 144, 2, 2, 64, 32, 32, 4),
    "SYN": (4096, 24, 5, 8, 512, 32, 32, 32),
}


def flops(N, T, K, h, D, dk, C):
    F = C
    nnzT = 4 * N
    fwd = 2 * (3 * F * T * N * h * dk + 2 * F * h * T * T * dk + F * T * h * dk * N + N * D * T * F + 2 * N * D * K * dk
               + K * N * N * dk + K * nnzT * F * T + K * N * T * F * C
               + sum(N * (T - k + 1) * 2 * C * C * k for k in (3, 5, 7)) + C * N * (3 * T - 12) * T)
    return 3 * fwd


def run(name, steps=10, warmup=3):
    import dstagnn_drought_amd as D_
    steps = int(os.environ.get("BENCH_CONFIGS_STEPS", steps))  # short runs under the profiler
    warmup = int(os.environ.get("BENCH_CONFIGS_WARMUP", warmup))
    N, T, K, h, Dm, dk, C, B = CONFIGS[name]
    B = int(os.environ.get("BENCH_CONFIGS_B", B))  # batch override (large-batch robustness runs)
    rs = np.random.RandomState(0)
    tmd = np.eye(N)
    pa = np.zeros((N, N))
    for i in range(N):
        tmd[i, rs.choice(N, 2, replace=False)] = 1.0
        pa[i, rs.choice(N, 4, replace=False)] = 1.0
    cheb = [torch.from_numpy(c).float() for c in D_.cheb_polynomial(D_.scaled_Laplacian(tmd), K)][:K]
    torch.manual_seed(1)
    blk = D_.DSTAGNN_block("cpu", C, C, K, C, C, 1, cheb, pa, tmd, N, T, Dm, dk, dk, h)
    for p in blk.parameters():
        if p.dim() > 1:
            torch.nn.init.xavier_uniform_(p)
        else:
            torch.nn.init.uniform_(p)
    blk = D_.set_direct_grads(blk.cuda().train())
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn(B, N, C, T, device="cuda", generator=g)
    res = torch.randn(B, 1, h, T, T, device="cuda", generator=g)
    go = torch.randn(B, N, C, T, device="cuda", generator=g)
    gr = torch.randn(B, C, h, T, T, device="cuda", generator=g)
    params = list(blk.parameters())

    def step():
        for p in params:
            p.grad = None
        o, r = blk(x, res)
        torch.autograd.backward([o, r], [go, gr])

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    f = flops(N, T, K, h, Dm, dk, C)
    sps = B / dt
    out = {"B": B, "ms_per_step": round(dt * 1e3, 3), "samples_per_s": round(sps, 1),
           "alg_mflop_per_sample": round(f / 1e6, 1), "block_roofline_frac": round(sps * f / PEAK, 4),
           "sparse_cheb": bool(blk.sparse_cheb),
           "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2)}
    del blk, x, res, go, gr, params
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats()
    return out


def run_model(name, steps=10, warmup=3):
    """make_model nb_block=4 (first block F=1) + head, SmoothL1 fwd+bwd — the CPU column's
    "PEMS04 model" row."""
    import dstagnn_drought_amd as D_
    steps = int(os.environ.get("BENCH_CONFIGS_STEPS", steps))
    warmup = int(os.environ.get("BENCH_CONFIGS_WARMUP", warmup))
    N, T, K, h, Dm, dk, C, B = CONFIGS[name.split("_")[0]]
    rs = np.random.RandomState(0)
    tmd = np.eye(N)
    pa = np.zeros((N, N))
    for i in range(N):
        tmd[i, rs.choice(N, 2, replace=False)] = 1.0
        pa[i, rs.choice(N, 4, replace=False)] = 1.0
    torch.manual_seed(1)
    net = D_.make_model("cpu", 1, 4, 1, K, C, C, 1, torch.FloatTensor(tmd), torch.FloatTensor(pa),
                        torch.FloatTensor(tmd), 12, T, N, Dm, dk, dk, h)
    net = D_.set_direct_grads(net.cuda().train())
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn(B, N, 1, T, device="cuda", generator=g)
    y = torch.randn(B, N, 12, device="cuda", generator=g)
    params = list(net.parameters())

    def step():
        for p in params:
            p.grad = None
        torch.nn.functional.smooth_l1_loss(net(x), y).backward()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    out = {"B": B, "ms_per_step": round(dt * 1e3, 3), "samples_per_s": round(B / dt, 1),
           "what": "make_model nb_block=4 + head, SmoothL1 fwd+bwd (no optimiser step)"}
    del net, x, y, params
    torch.cuda.empty_cache()
    return out


def main():
    names = sys.argv[1:] or (list(CONFIGS) + ["PEMS04_model"])
    res = {}
    for n in names:
        print(f"[configs] {n}", file=sys.stderr, flush=True)
        res[n] = run_model(n) if n.endswith("_model") else run(n)
        print(f"[configs] {n}: {res[n]}", file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
