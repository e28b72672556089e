#!/usr/bin/env python
"""The bench's `extras.model_step` workload alone (make_model nb_block=4 PEMS08, B=32: forward,
SmoothL1, backward, Adam) for a kernel trace:

    rocprofv3 --kernel-trace --stats -d gpurun_out/mstep -o run --output-format csv -- \
        python3 tools/model_step_prof.py --steps 5

then `python3 tools/prof_summary.py <trace.csv>` groups the kernels (blocks, head, loss, Adam)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    import torch
    import bench
    import dstagnn_drought_amd as D
    from dstagnn_drought_amd.train import make_adam
    c = bench.CFG
    B, N, T, K, h, Dm, dk, C = c["B"], c["N"], c["T"], c["K"], c["n_heads"], c["d_model"], c["d_k"], c["C"]
    dev = torch.device("cuda:0")
    tmd, pa = bench.synth_graph(N)
    torch.manual_seed(1)
    net = D.make_model(dev, 1, 4, 1, K, C, C, 1, tmd, pa, tmd, T, T, N, Dm, dk, dk, h)
    D.set_direct_grads(net).train()
    opt = make_adam(net.parameters(), 1e-4)
    crit = torch.nn.SmoothL1Loss().to(dev)
    gen = torch.Generator(device=dev).manual_seed(5)
    xm = torch.randn(B, N, 1, T, device=dev, generator=gen)
    ym = torch.randn(B, N, T, device=dev, generator=gen)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = crit(net(xm), ym)
        loss.backward()
        opt.step()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    print(f"model step {(time.perf_counter() - t0) / a.steps * 1e3:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
