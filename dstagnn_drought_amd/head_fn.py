"""torch.autograd.Function over the HIP model head (head.hip through dstagnn::head_fwd/bwd).

Replaces the tail of DSTAGNN_submodule.forward (model/DSTAGNN_my.py:272-280):
``torch.cat(need_concat, -1)`` -> ``final_conv(...permute(0,3,1,2))[..., -1].permute(0,2,1)``
-> ``final_fc``.  The final_conv kernel (1, nb_time_filter) spans the block output's whole
C axis, so the head is one (t,c)-contraction per block output plus a Linear; the cat is
never materialised.  Parameters stay the reference's ``final_conv.{weight,bias}`` /
``final_fc.{weight,bias}`` tensors (same state_dict).
"""
import torch

from . import _lib


class DSTAGNNHeadFunction(torch.autograd.Function):
    """dstagnn::head_fwd / dstagnn::head_bwd (csrc/torch_ops.cpp -> head.hip)."""

    @staticmethod
    def forward(ctx, w1, b1, w2, b2, *outs):
        ops = _lib.load()
        ctx.set_materialize_grads(False)
        outs = [o.contiguous() for o in outs]
        h, y = ops.head_fwd(outs, w1, b1, w2, b2)
        ctx.nb = len(outs)
        ctx.save_for_backward(w1, w2, h, *outs)
        return y

    @staticmethod
    def backward(ctx, dy):
        if dy is None:
            return (None,) * (4 + ctx.nb)
        w1, w2, h, *outs = ctx.saved_tensors
        need = [int(bool(n)) for n in ctx.needs_input_grad]
        r = _lib.load().head_bwd(outs, w1, w2, h, dy, need)
        return tuple(t if n else None for t, n in zip(r, need))


def head(final_conv, final_fc, outs):
    return DSTAGNNHeadFunction.apply(final_conv.weight, final_conv.bias, final_fc.weight, final_fc.bias, *outs)
