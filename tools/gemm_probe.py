#!/usr/bin/env python
"""Event timing of one strided GEMM through dstagnn::gemm_f32 (for rocprofv3 kernel traces and
PMC passes on a single shape).  usage: gemm_probe.py M N K [akc bnc [iters]]
akc: A stored k-contiguous (M x K row-major) else m-contiguous (K x M); bnc: B stored
n-contiguous (K x N) else k-contiguous (N x K).  Default: the fcmy weight gradient."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dstagnn_drought_amd import _lib  # noqa: E402

argv = [int(v) for v in sys.argv[1:]]
M, N, K = argv[:3] if len(argv) >= 3 else (12, 25, 174080)
akc = argv[3] if len(argv) > 3 else 0
bnc = argv[4] if len(argv) > 4 else 1
iters = argv[5] if len(argv) > 5 else 50
ops = _lib.load()
A = torch.randn(M * K, device="cuda")
B = torch.randn(K * N, device="cuda")
C = torch.empty(M, N, device="cuda")
am, ak = ((0, K, 0), (0, 1, 0)) if akc else ((0, 1, 0), (0, M, 0))
bk, bn = ((0, N, 0), (0, 1, 0)) if bnc else ((0, 1, 0), (0, K, 0))
maps = _lib.gemm_maps(am, ak, (0, 0, 0), bk, bn, (0, 0, 0), (0, N, 0), (0, 1, 0), (0, 0, 0))


def run():
    ops.gemm_f32(A, B, C, [M, N, K, 1], maps, [0, 0, 0], 1.0, 0.0, None, 1, False)


for _ in range(5):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    run()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / iters * 1000
print(f"M={M} N={N} K={K} akc={akc} bnc={bnc}: {us:.2f} us/call (event, includes host gaps), "
      f"{2.0 * M * N * K / us / 1e6:.1f} TF/s")
