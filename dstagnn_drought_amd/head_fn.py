"""torch.autograd.Function over the HIP model head (head.hip, C-ABI dstagnn_head_*).

Replaces the tail of DSTAGNN_submodule.forward (model/DSTAGNN_my.py:272-280):
``torch.cat(need_concat, -1)`` -> ``final_conv(...permute(0,3,1,2))[..., -1].permute(0,2,1)``
-> ``final_fc``.  The final_conv kernel (1, nb_time_filter) spans the block output's whole
C axis, so the head is one (t,c)-contraction per block output plus a Linear; the cat is
never materialised.  Parameters stay the reference's ``final_conv.{weight,bias}`` /
``final_fc.{weight,bias}`` tensors (same state_dict).
"""
import ctypes

import torch

from . import _lib

_SCRATCH = {}


def _scratch(dev):
    t = _SCRATCH.get(dev)
    if t is None:
        n = int(_lib.load().dstagnn_head_scratch_bytes())
        t = _SCRATCH[dev] = torch.empty(n, dtype=torch.uint8, device=dev)
    return t


def _ptrs(ts):
    arr = (ctypes.c_void_p * len(ts))()
    for i, t in enumerate(ts):
        arr[i] = None if t is None else t.data_ptr()
    return arr


class DSTAGNNHeadFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, w1, b1, w2, b2, *outs):
        lib = _lib.load()
        ctx.set_materialize_grads(False)
        outs = [o.contiguous() for o in outs]
        B, N, C, T = outs[0].shape
        for o in outs:
            if tuple(o.shape) != (B, N, C, T):
                raise RuntimeError(f"head: block outputs differ in shape: {tuple(o.shape)} vs {(B, N, C, T)}")
        nb = len(outs)
        O, P = w1.shape[0], w2.shape[0]
        if tuple(w1.shape) != (O, nb * T, 1, C):
            raise RuntimeError(f"Given weight of size {list(w1.shape)}, expected input[{B}, {nb * T}, {N}, {C}] "
                               f"to match final_conv (model/DSTAGNN_my.py:265)")
        if w2.shape[1] != O:
            raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({B * N}x{O} and {w2.shape[1]}x{P})")
        dev = outs[0].device
        h = torch.empty(B, N, O, device=dev)
        y = torch.empty(B, N, P, device=dev)
        sc = _scratch(dev)
        rc = lib.dstagnn_head_forward(B, N, C, T, nb, O, P, _ptrs(outs), _lib.ptr(w1), _lib.ptr(b1),
                                      _lib.ptr(w2), _lib.ptr(b2), _lib.ptr(h), _lib.ptr(y), _lib.ptr(sc),
                                      sc.numel(), _lib.stream_handle(dev))
        _lib.check(rc, "dstagnn_head_forward")
        ctx.dims = (B, N, C, T, nb, O, P)
        ctx.save_for_backward(w1, w2, h, *outs)
        return y

    @staticmethod
    def backward(ctx, dy):
        if dy is None:
            return (None,) * (4 + ctx.dims[4])
        lib = _lib.load()
        w1, w2, h, *outs = ctx.saved_tensors
        B, N, C, T, nb, O, P = ctx.dims
        dy = dy.contiguous()
        dev = dy.device
        need = ctx.needs_input_grad
        dh = torch.empty(B, N, O, device=dev)
        dw1 = torch.empty_like(w1) if need[0] else None
        db1 = torch.empty(O, device=dev) if need[1] else None
        dw2 = torch.empty_like(w2) if need[2] else None
        db2 = torch.empty(P, device=dev) if need[3] else None
        douts = [torch.empty_like(o) if need[4 + j] else None for j, o in enumerate(outs)]
        sc = _scratch(dev)
        rc = lib.dstagnn_head_backward(B, N, C, T, nb, O, P, _ptrs(outs), _lib.ptr(w1), _lib.ptr(w2),
                                       _lib.ptr(h), _lib.ptr(dy), _lib.ptr(dh), _ptrs(douts), _lib.ptr(dw1),
                                       _lib.ptr(db1), _lib.ptr(dw2), _lib.ptr(db2), _lib.ptr(sc), sc.numel(),
                                       _lib.stream_handle(dev))
        _lib.check(rc, "dstagnn_head_backward")
        return (dw1, db1, dw2, db2, *douts)


def head(final_conv, final_fc, outs):
    return DSTAGNNHeadFunction.apply(final_conv.weight, final_conv.bias, final_fc.weight, final_fc.bias, *outs)
