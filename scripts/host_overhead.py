#!/usr/bin/env python
"""Host-side cost of issuing the block: raw C-ABI forward (prebuilt arguments, no sync),
a trivial ctypes call, and the full autograd step — to tell launch-bound from GPU-bound."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dstagnn_drought_amd import _lib  # noqa: E402
from dstagnn_drought_amd.block_fn import make_dims, workspace_sizes, _fill, graph_struct, use_sparse  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    blk, _, _ = bench.build_block(dev)
    c = bench.CFG
    B = c["B"]
    x = torch.randn(B, c["N"], c["C"], c["T"], device=dev)
    res = torch.randn(B, 1, c["n_heads"], c["T"], c["T"], device=dev)
    meta = dict(blk.meta, train=True, seed=1)
    graph = blk.cheb_conv_SAt.graph(blk.adj_pa)
    dims = make_dims(x, meta, _lib.RES_BCAST, True, 1, use_sparse(graph, meta, c["T"]))
    sv, sc = workspace_sizes(dims)
    save = torch.empty(sv, dtype=torch.uint8, device=dev)
    scratch = torch.empty(sc, dtype=torch.uint8, device=dev)
    names, ps = zip(*blk.named_parameters())
    pstruct = _fill(_lib.BlockParams(), names, ps)
    gstruct = graph_struct(graph)
    out = torch.empty(B, c["N"], c["C"], c["T"], device=dev)
    re_at = torch.empty(B, c["C"], c["n_heads"], c["T"], c["T"], device=dev)
    lib = _lib.load()
    st = _lib.stream_handle(dev)
    args = (ctypes.byref(dims), ctypes.byref(pstruct), ctypes.byref(gstruct), _lib.ptr(x), _lib.ptr(res),
            _lib.ptr(out), _lib.ptr(re_at), _lib.ptr(save), sv, _lib.ptr(scratch), sc, st)
    for _ in range(5):
        lib.dstagnn_block_forward(*args)
    torch.cuda.synchronize()
    n = 100
    t0 = time.perf_counter()
    for _ in range(n):
        lib.dstagnn_block_forward(*args)
    t_issue = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for _ in range(1000):
        lib.dstagnn_version()
    t_ct = (time.perf_counter() - t0) / 1000
    # raw backward (all grads requested)
    gs = [torch.empty_like(p_) for p_ in ps]
    gstr = _fill(_lib.BlockGrads(), names, gs)
    g_out = torch.randn_like(out)
    g_re = torch.randn_like(re_at)
    dxb = torch.empty_like(x)
    dres = torch.empty_like(res)
    bargs = (ctypes.byref(dims), ctypes.byref(pstruct), ctypes.byref(gstruct), _lib.ptr(x), _lib.ptr(res),
             _lib.ptr(g_out), _lib.ptr(g_re), _lib.ptr(dxb), _lib.ptr(dres), ctypes.byref(gstr), _lib.ptr(save), sv,
             _lib.ptr(scratch), sc, st)
    for _ in range(5):
        lib.dstagnn_block_backward(*bargs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        lib.dstagnn_block_backward(*bargs)
    t_bi = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    t_ba = (time.perf_counter() - t0) / n
    print(f"raw C-ABI backward: issue {t_bi * 1e6:.1f} us/call, issue+run {t_ba * 1e6:.1f} us/call")
    # full autograd step (issue)
    params = list(blk.parameters())
    t0 = time.perf_counter()
    for _ in range(20):
        for p_ in params:
            p_.grad = None
        o, r = blk(x, res)
        torch.autograd.backward([o, r], [g_out, g_re])
    t_step = (time.perf_counter() - t0) / 20
    torch.cuda.synchronize()
    print(f"autograd step: issue {t_step * 1e6:.1f} us/step")
    # autograd forward only (issue)
    t0 = time.perf_counter()
    for _ in range(n):
        o, r = blk(x, res)
    t_fwd_py = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    print(f"raw C-ABI forward: issue {t_issue * 1e6:.1f} us/call, issue+run {t_all * 1e6:.1f} us/call")
    print(f"ctypes trivial call: {t_ct * 1e6:.2f} us")
    print(f"module forward (autograd, issue): {t_fwd_py * 1e6:.1f} us/call")


if __name__ == "__main__":
    main()
