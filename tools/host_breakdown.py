"""Host cost of the pieces of one training step of the bench block, at a tiny batch (B=1: the
GPU idles, every figure is host time).  Each piece runs N times back to back between two
synchronisations; the library's own per-stage issue laps come with DSTAGNN_HOST_PROFILE=1.
usage: python tools/host_breakdown.py [B]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def timed(fn, n=300):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t = time.perf_counter() - t0
    torch.cuda.synchronize()
    return t / n * 1e6


def main():
    dev = torch.device("cuda", 0)
    bench.CFG["B"] = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    blk, _, _ = bench.build_block(dev)
    from dstagnn_drought_amd import _lib, block_fn as bf
    ops = _lib.load()
    c = bench.CFG
    B = c["B"]
    x = torch.randn(B, c["N"], c["C"], c["T"], device=dev)
    res = torch.randn(B, 1, c["n_heads"], c["T"], c["T"], device=dev)
    g_out = torch.randn(B, c["N"], c["C"], c["T"], device=dev)
    g_re = torch.randn(B, c["C"], c["n_heads"], c["T"], c["T"], device=dev)
    params = list(blk.parameters())

    def zero():
        for p in params:
            p.grad = None

    def step():
        zero()
        out, re_at = blk(x, res)
        torch.autograd.backward([out, re_at], [g_out, g_re])

    names, ps, slots = blk._param_list()
    graph = blk._graph()
    sparse = bf.use_sparse(graph, blk.meta, c["T"])
    fl = bf.use_flash(graph, blk.meta, c["T"], None, B)
    if fl:
        graph = blk._flash_graph(graph)
    gl = bf.graph_list(graph, sparse, fl)
    cfg = bf.cfg_of(blk.meta)
    flags = bf.flags_of(True, sparse, False, fl)
    save = {}

    def op_fwd():
        save["r"] = ops.block_fwd(x, res, list(ps), slots, gl, cfg, 0.05, 1, flags)

    def op_bwd():
        o, r, s = save["r"]
        ops.block_bwd(x, res, g_out, g_re, s, list(ps), slots, gl, cfg, 0.05, 1, flags)

    def fwd_only():
        with torch.no_grad():
            blk(x, res)

    def fwd_autograd():
        save["o"] = blk(x, res)

    def bwd_autograd():
        o, r = blk(x, res)
        torch.autograd.backward([o, r], [g_out, g_re])

    rows = [("zero_grad loop (%d params)" % len(params), zero), ("full step", step),
            ("op block_fwd (no autograd, no module)", op_fwd), ("op block_bwd", op_bwd),
            ("module forward, no_grad", fwd_only), ("module forward, autograd", fwd_autograd),
            ("module forward + backward", bwd_autograd)]
    for name, fn in rows:
        if name == "op block_bwd":
            op_fwd()
        print(f"B={B} {name:42s} {timed(fn):8.1f} us", flush=True)
    print(f"B={B} (op_bwd includes nothing else; fwd+bwd ops = {timed(lambda: (op_fwd(), op_bwd())):.1f} us)")


if __name__ == "__main__":
    main()
