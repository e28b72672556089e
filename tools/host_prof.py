"""Host cost of one training step of the block at a tiny batch (B=1: the GPU idles, the step
time is the host's), and a cProfile of where the Python side spends it."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    bench.CFG["B"] = int(os.environ.get("HP_B", "1"))
    blk, _, _ = bench.build_block(dev)
    c = bench.CFG
    B = c["B"]
    x = torch.randn(B, c["N"], c["C"], c["T"], device=dev)
    res = torch.randn(B, 1, c["n_heads"], c["T"], c["T"], device=dev)
    g_out = torch.randn(B, c["N"], c["C"], c["T"], device=dev)
    g_re = torch.randn(B, c["C"], c["n_heads"], c["T"], c["T"], device=dev)
    params = list(blk.parameters())

    def fwd():
        return blk(x, res)

    def step():
        for p in params:
            p.grad = None
        out, re_at = fwd()
        torch.autograd.backward([out, re_at], [g_out, g_re])

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    print(f"B={B}: step {1e6 * (time.perf_counter() - t0) / n:.1f} us")
    t0 = time.perf_counter()
    for _ in range(n):
        o = fwd()
    torch.cuda.synchronize()
    print(f"B={B}: forward only {1e6 * (time.perf_counter() - t0) / n:.1f} us")
    x.requires_grad_(True)
    for p in params:
        p.requires_grad_(False)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    print(f"B={B}: step without parameter AccumulateGrad {1e6 * (time.perf_counter() - t0) / n:.1f} us")
    for p in params:
        p.requires_grad_(True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(50):
        step()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
