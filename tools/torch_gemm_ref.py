"""rocBLAS/hipBLASLt (torch.mm / bmm, fp32, no TF32) timing at the block's GEMM shapes
(tools/gemm_sweep.py SHAPES), as a library reference point for the hand-written GEMM."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_sweep import SHAPES  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
for name, M, N, K, batch, akc, bnc in SHAPES:
    a = torch.randn(batch, M, K, device="cuda") if akc else torch.randn(batch, K, M, device="cuda").transpose(1, 2)
    b = torch.randn(batch, K, N, device="cuda") if bnc else torch.randn(batch, N, K, device="cuda").transpose(1, 2)
    for _ in range(5):
        torch.bmm(a, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    e0.record()
    for _ in range(n):
        torch.bmm(a, b)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / n * 1e3
    print(f"{name:12s} {M}x{N}x{K}x{batch}: {us:8.1f} us  {2 * M * N * K * batch / us / 1e6:7.1f} TF/s", flush=True)
