"""Probe: the bench step captured in a hipGraph (torch.cuda.graph) vs eager — tells the
GPU-bound step time and whether graph replay keeps the side-stream concurrency.
(Dropout seeds are baked at capture here: a measurement probe, not a training path.)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    blk, _, _ = bench.build_block(dev)
    c = bench.CFG
    B = c["B"]
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(B, c["N"], c["C"], c["T"], device=dev, generator=g)
    res = torch.randn(B, 1, c["n_heads"], c["T"], c["T"], device=dev, generator=g)
    g_out = torch.randn(B, c["N"], c["C"], c["T"], device=dev, generator=g)
    g_re = torch.randn(B, c["C"], c["n_heads"], c["T"], c["T"], device=dev, generator=g)
    params = list(blk.parameters())

    def step():
        for p in params:
            p.grad = None
        out, re_at = blk(x, res)
        torch.autograd.backward([out, re_at], [g_out, g_re])

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    n = 100
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / n * 1e3
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        graph.replay()
    ti = (time.perf_counter() - t0) / n * 1e3
    torch.cuda.synchronize()
    rep = (time.perf_counter() - t0) / n * 1e3
    print(f"eager {eager:.3f} ms/step | graph replay {rep:.3f} ms/step (host issue {ti:.3f})")


if __name__ == "__main__":
    main()
