#!/usr/bin/env python
"""Event timing of one strided GEMM shape through dstagnn::gemm_f32 (default: the fcmy weight
gradient, 12 x 25 over 174080 rows, A m-contiguous).  usage: skinny_probe.py [M N K]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dstagnn_drought_amd import _lib  # noqa: E402

ops = _lib.load()
if len(sys.argv) > 1 and sys.argv[1] == "theta":
    # the aggregate-first dTheta: agg (B*N, K, F, T) x g (B*N, T, C) -> (K*F, C), PEMS08 B=32
    BN, KK, F, T, Cc = 5440, 3, 32, 12, 32
    M, N, K = KK * F, Cc, BN * T
    A = torch.randn(BN, KK, F, T, device="cuda")
    B = torch.randn(BN, T, Cc, device="cuda")
    maps = _lib.gemm_maps((0, T, 0), (T, 1, KK * F * T), (0, 0, 0), (0, N, 0), (0, 1, 0), (0, 0, 0), (0, N, 0), (0, 1, 0),
                          (0, 0, 0))
else:
    M, N, K = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (12, 25, 174080)
    A = torch.randn(K, M, device="cuda")
    B = torch.randn(K, N, device="cuda")
    maps = _lib.gemm_maps((0, 1, 0), (0, M, 0), (0, 0, 0), (0, N, 0), (0, 1, 0), (0, 0, 0), (0, N, 0), (0, 1, 0),
                          (0, 0, 0))
C = torch.empty(M, N, device="cuda")


def run():
    ops.gemm_f32(A, B, C, [M, N, K, 1], maps, [0, 0, 0], 1.0, 0.0, None, 1, False)


for _ in range(5):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    run()
e1.record()
torch.cuda.synchronize()
print(f"M={M} N={N} K={K} env skinny={os.environ.get('DSTAGNN_GEMM_SKINNY')} stop={os.environ.get('DSTAGNN_SKINNY_STOP')} "
      f"kpw={os.environ.get('DSTAGNN_SKINNY_KPW')} fold1={os.environ.get('DSTAGNN_SKINNY_FOLD1_KB')}: {e0.elapsed_time(e1) / 50 * 1000:.2f} us/call")
