#!/usr/bin/env python
"""Does a half-batch split on two streams pack better than one full batch?  Times the PEMS08
bench block: forward only and forward+backward at B=32, at B=16, and two B=16 halves issued on
two torch streams (each half's block op runs on its stream, the library's side stream per main
stream).  usage: split_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
blk, _, _ = bench.build_block(dev)
c = bench.CFG
B = c["B"]
g = torch.Generator(device=dev).manual_seed(5)
x = torch.randn(B, c["N"], c["C"], c["T"], device=dev, generator=g)
res = torch.randn(B, 1, c["n_heads"], c["T"], c["T"], device=dev, generator=g)
go = torch.randn(B, c["N"], c["C"], c["T"], device=dev, generator=g)
gr = torch.randn(B, c["C"], c["n_heads"], c["T"], c["T"], device=dev, generator=g)
params = list(blk.parameters())
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
h = B // 2


def fwd(lo, hi):
    return blk(x[lo:hi], res[lo:hi])


def fb(lo, hi):
    out, re = blk(x[lo:hi], res[lo:hi])
    torch.autograd.backward([out, re], [go[lo:hi], gr[lo:hi]])


def full_f():
    with torch.no_grad():
        fwd(0, B)


def half_f():
    with torch.no_grad():
        fwd(0, h)


def two_f():
    with torch.no_grad():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur); s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            fwd(0, h)
        with torch.cuda.stream(s2):
            fwd(h, B)
        cur.wait_stream(s1); cur.wait_stream(s2)


def full_fb():
    for p in params:
        p.grad = None
    fb(0, B)


def half_fb():
    for p in params:
        p.grad = None
    fb(0, h)


def two_fb():
    for p in params:
        p.grad = None
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur); s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        o1, r1 = blk(x[:h], res[:h])
    with torch.cuda.stream(s2):
        o2, r2 = blk(x[h:], res[h:])
    with torch.cuda.stream(s1):
        torch.autograd.backward([o1, r1], [go[:h], gr[:h]])
    with torch.cuda.stream(s2):
        torch.autograd.backward([o2, r2], [go[h:], gr[h:]])
    cur.wait_stream(s1); cur.wait_stream(s2)


for name, f in [("fwd B=32", full_f), ("fwd B=16", half_f), ("fwd 2x16 two streams", two_f),
                ("fwd+bwd B=32", full_fb), ("fwd+bwd B=16", half_fb), ("fwd+bwd 2x16 two streams", two_fb)]:
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        f()
    torch.cuda.synchronize()
    print(f"{name:28s} {(time.perf_counter() - t0) * 10:.3f} ms", flush=True)
