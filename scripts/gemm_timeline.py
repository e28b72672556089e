#!/usr/bin/env python
"""Per-workgroup timeline of one GEMM launch from the STAMP build (scripts/build_abl.sh):
s_memtime at kernel entry, after index setup, after the first k-tile is in LDS, after each
k-tile, after the epilogue.  Prints the mean/min/max of each phase in cycles, and the spread
of start and end times across workgroups.

    DSTAGNN_LIB=dstagnn_drought_amd/libdstagnn_abl_STAMP.so python scripts/gemm_timeline.py M N K [cfg]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dstagnn_drought_amd import _lib  # noqa: E402


def main():
    M, N, K = (int(v) for v in sys.argv[1:4])
    lib = _lib.load()
    lib.dstagnn_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    A = torch.randn(K, M, device="cuda")
    B = torch.randn(N, K, device="cuda")
    C = torch.empty(M, N, device="cuda")
    ws = torch.empty(1 << 20, device="cuda")
    d = _lib.GemmDesc()
    d.M, d.N, d.K, d.batch = M, N, K, 1
    d.A, d.B, d.C = A.data_ptr(), B.data_ptr(), C.data_ptr()
    d.a_m, d.a_k = _lib.idx(0, 1), _lib.idx(0, M)
    d.b_k, d.b_n = _lib.idx(0, 1), _lib.idx(0, K)
    d.a_z, d.b_z, d.c_z = _lib.idx(0, 0), _lib.idx(0, 0), _lib.idx(0, 0)
    d.c_m, d.c_n = _lib.idx(0, N), _lib.idx(0, 1)
    d.alpha, d.beta, d.bias, d.bias_stride, d.relu = 1.0, 0.0, None, 1, 0
    st = _lib.stream_handle()
    for _ in range(3):
        _lib.check(lib.dstagnn_gemm_f32(ctypes.byref(d), _lib.ptr(ws), ws.numel(), st), "gemm")
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 16, dtype=np.uint64)
    rc = lib.dstagnn_debug_stamps(buf.ctypes.data, buf.size)
    assert rc == 0, rc
    s = buf.reshape(4096, 16).astype(np.int64)
    nb = int((s[:, 0] != 0).sum())
    s = s[:nb]
    t0 = s[:, 0].min()
    ntile = (K + 31) // 32
    cols = [0, 11, 12, 1, 2] + [3 + t for t in range(min(ntile, 8))] + [15]
    print(f"workgroups {nb}, start spread {s[:, 0].max() - t0} cyc, end spread {s[:, 15].max() - s[:, 15].min()} cyc,"
          f" kernel span {s[:, 15].max() - t0} cyc")
    names = {11: "tile decode", 12: "offsets", 1: "setup rest", 2: "first tile"}
    prev = 0
    for c in cols[1:]:
        dlt = s[:, c] - s[:, prev]
        nm = names.get(c, "rest+epilogue" if c == 15 else f"tile {c - 3}")
        print(f"{nm:12s} mean {dlt.mean():8.0f}  min {dlt.min():8d}  max {dlt.max():8d}")
        prev = c
    life = s[:, 15] - s[:, 0]
    print(f"{'lifetime':12s} mean {life.mean():8.0f}  min {life.min():8d}  max {life.max():8d}")
    # concurrency: how many workgroups are alive at once (sampled)
    ts = np.linspace(t0, s[:, 15].max(), 20)
    alive = [int(((s[:, 0] <= t) & (s[:, 15] >= t)).sum()) for t in ts]
    print("alive over time:", alive)


if __name__ == "__main__":
    main()
