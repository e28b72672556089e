"""Host side of the HIP DSTAGNN_block: the call into ``torch.ops.dstagnn.block``.

``dstagnn::block`` (csrc/torch_ops.cpp) is ONE C++ autograd node per block: its forward is
one ``dstagnn_block_forward`` call and its backward one ``dstagnn_block_backward`` call, so
every stage of model/DSTAGNN_my.py:225-253 and its gradient runs in our own gfx950 kernels
on torch's current HIP stream.  PyTorch only provides the device memory (caching
allocator), the stream and the autograd engine.  This module maps the reference's
parameter names onto the library's parameter slots and builds the call's arguments.
"""
import os

import torch

from . import _lib

# block-local state_dict name -> slot in dstagnn_block_params (include/dstagnn.h: the struct
# is an array of 44 pointers in this order)
_FIELDS = ["pre_conv.weight", "pre_conv.bias", "EmbedT.pos_embed.weight", "EmbedT.norm.weight",
           "EmbedT.norm.bias", "EmbedS.pos_embed.weight", "EmbedS.norm.weight", "EmbedS.norm.bias",
           "TAt.W_Q.weight", "TAt.W_K.weight", "TAt.W_V.weight", "TAt.fc.weight", "TAt.layer_norm.weight",
           "TAt.layer_norm.bias", "SAt.W_Q.weight", "SAt.W_K.weight"]
PARAM_SLOT = {n: i for i, n in enumerate(_FIELDS)}
for _k in range(_lib.MAX_K):
    PARAM_SLOT[f"cheb_conv_SAt.Theta.{_k}"] = 16 + _k
    PARAM_SLOT[f"cheb_conv_SAt.mask.{_k}"] = 16 + _lib.MAX_K + _k
for _q, _ks in enumerate((3, 5, 7)):
    PARAM_SLOT[f"gtu{_ks}.con2out.weight"] = 32 + _q
    PARAM_SLOT[f"gtu{_ks}.con2out.bias"] = 35 + _q
PARAM_SLOT.update({"residual_conv.weight": 38, "residual_conv.bias": 39, "fcmy.0.weight": 40, "fcmy.0.bias": 41,
                   "ln.weight": 42, "ln.bias": 43})

# parameters a block of each kind never touches (quirk 11: their .grad stays None)
UNUSED_INNER = ("EmbedT.", "residual_conv.")

# DSTAGNN_POISON=1: every buffer the library writes starts as NaN (a read of memory the
# kernels never wrote shows up as NaN instead of as whatever the allocator handed back)
_POISON = os.environ.get("DSTAGNN_POISON", "0") == "1"


def slots_of(names):
    return [PARAM_SLOT[n] for n in names]


def res_arg(res_att, F):
    """res_att as the op takes it: None for the int 0 the first block receives
    (DSTAGNN_submodule.forward:273), else a contiguous float tensor.  Shape errors are
    raised by the op with the reference's message."""
    if not torch.is_tensor(res_att):
        if res_att != 0:
            raise RuntimeError("res_att must be 0 or a tensor (model/DSTAGNN_my.py:37)")
        return None
    return res_att.float().contiguous()


FLASH_KEYS = ("csr2csc", "apa_bits", "apa_bits_t", "apa_ptr", "apa_row", "tsupp", "csc2csr", "apa_idx", "apa2t")


def graph_list(graph, sparse, flash=False):
    """[cheb (K,N,N), adj_pa (N,N)] + the int32 CSC/CSR union support for the sparse path
    + the flash-attention index data (model.flash_support) for the fused path."""
    g = [graph["cheb"], graph["adj_pa"]]
    if sparse:
        g += [graph["csc_ptr"], graph["csc_row"], graph["csr_ptr"], graph["csr_col"]]
        if flash:
            g += [graph[k] for k in FLASH_KEYS]
    return g


def use_sparse(graph, meta, T):
    """Sparse Chebyshev aggregation when the union support is <= 1/4 dense (rows of any length:
    the kernels walk C*T in 1024-element chunks)."""
    if graph.get("csc_row") is None:
        return False
    N = graph["adj_pa"].shape[0]
    return graph["csc_row"].numel() * 4 <= N * N and meta["C"] * T <= (1 << 20)


FLASH_SMALL_N = 512  # cheb_flash.hip kSmallN: graphs up to this size take the LDS-staged kernels


def use_flash(graph, meta, T, force=None, B=0):
    """Fused (flash-style) Chebyshev attention (cheb_flash.hip): the (B,K,N,N) scores, softmax
    and score gradient are never written; on the sparse path with d_k == 32 (the MFMA tile),
    automatically: small graphs (N <= 512) take the LDS-staged kernels (one workgroup per
    32-column strip, operands staged once), larger ones the streamed kernels (one wave per strip)
    — at PEMS07's N = 883 as well (1.40 -> 1.31 ms per step against the dense (B,K,N,N) softmax
    path, same box, round 6); DSTAGNN_FLASH=0/1 overrides, as does `force`; batches up to 128
    per call (the mask-gradient kernel's lanes)."""
    if not use_sparse(graph, meta, T) or meta["d_k"] != 32 or B > 128:
        return False
    if force is not None:
        return bool(force)
    env = os.environ.get("DSTAGNN_FLASH")
    if env is not None:
        return env == "1"
    return True


def cfg_of(meta):
    return [meta["n_heads"], meta["d_k"], meta["d_v"], meta["d_model"], meta["K"], meta["C"]]


SAMPLE_SHIFT = 32  # flags bits 32..: the call's first global sample index (torch_ops.cpp kSampleShift)


def flags_of(train, sparse, direct, flash=False, sample_base=0):
    if sample_base < 0:
        raise ValueError("sample_base must be >= 0")
    return ((_lib.F_TRAIN if train else 0) | (_lib.F_SPARSE if sparse else 0) | (_lib.F_DIRECT if direct else 0)
            | (_lib.F_POISON if _POISON else 0) | (_lib.F_FLASH if flash else 0) | (int(sample_base) << SAMPLE_SHIFT))


def block_call(x, res_att, params, slots, graph, meta, train, seed, direct=False, flash=None, plan_cache=None,
               sample_base=0):
    """(out, re_at) = dstagnn::block(...) — autograd-tracked.  In direct-gradient mode with a
    plan_cache dict (the module's), the block's constant arguments go to the library once, as a
    cached BlockPlan (dstagnn::block_planned): same kernels, less host work per call.
    sample_base: global index of x[0] (a data-parallel shard's offset; keys the dropout masks)."""
    ops = _lib.load()
    x = x.float().contiguous()
    sparse = use_sparse(graph, meta, x.shape[3])
    fl = use_flash(graph, meta, x.shape[3], flash, x.shape[0])
    flags = flags_of(train, sparse, direct, fl, sample_base)
    if direct and plan_cache is not None:
        key = (id(params), id(graph), sparse, fl)
        ent = plan_cache.get("plan")
        if ent is None or ent[0] != key:
            plist = list(params)
            plan = torch.classes.dstagnn.BlockPlan(plist, list(slots), graph_list(graph, sparse, fl), cfg_of(meta))
            ent = [key, plan, _anchor(plist, None), params, graph]  # params / graph kept alive: the key holds their ids
            plan_cache["plan"] = ent
        elif not ent[2].requires_grad:
            # the anchor (the autograd input that keeps the node in the graph when x needs no
            # gradient) was frozen since: re-pick among the parameters that train now
            ent[2] = _anchor(ent[3], ent[2])
        return ops.block_planned(x, res_arg(res_att, x.shape[2]), ent[1], ent[2], float(meta.get("drop_p", 0.05)),
                                 int(seed), flags)
    return ops.block(x, res_arg(res_att, x.shape[2]), list(params), slots, graph_list(graph, sparse, fl),
                     cfg_of(meta), float(meta.get("drop_p", 0.05)), int(seed), flags)


def _anchor(params, fallback):
    """A parameter that currently requires grad (the planned op's autograd anchor), else
    `fallback` (else the first parameter): with none trainable and x not requiring grad no node
    is recorded, and there is nothing to differentiate."""
    return next((p for p in params if p.requires_grad), fallback if fallback is not None else params[0])


def dropout_masks(meta, x_shape, seed, sample_base=0):
    """The exact keep-masks (scaled by 1/(1-p)) the HIP forward draws for `seed` on samples
    sample_base .. sample_base + B - 1 of the global batch: (mask after EmbedS (B,N,D), mask
    after fcmy (B,N,C,T)) — for parity tests."""
    ops = _lib.load()
    like = torch.empty(0, device="cuda")
    return ops.dropout_masks(like, list(x_shape), cfg_of(meta), float(meta.get("drop_p", 0.05)), int(seed),
                             int(sample_base))


# dstagnn_block_paths bits (include/dstagnn.h DSTAGNN_PATH_*)
PATH_BITS = {"sparse": 1, "flash": 2, "flash_small": 4, "cheb_agg": 8, "tat_fused_fwd": 16, "tat_fused_bwd": 32,
             "gtu_fused_fwd": 64, "gtu_fused_bwd": 128, "sat_ln_fused": 256}


def block_paths(blk, x, res_att, train=False):
    """The set of kernel paths (PATH_BITS names) the library takes for this block module on
    this input (dstagnn::block_paths over dstagnn_block_paths: decided from the call's dims and
    the process's DSTAGNN_* knobs; launches nothing) — parity tests assert with it that the
    kernels they hold to the oracle are the ones that ran."""
    ops = _lib.load()
    names, ps, slots = blk._param_list()
    graph = blk._graph()
    sparse = use_sparse(graph, blk.meta, x.shape[3])
    fl = use_flash(graph, blk.meta, x.shape[3], blk.flash_cheb, x.shape[0])
    if fl:
        graph = blk._flash_graph(graph)
    bits = ops.block_paths(x.detach().float().contiguous(), res_arg(res_att, x.shape[2]), list(ps), slots,
                           graph_list(graph, sparse, fl), cfg_of(blk.meta), 0.05, 0, flags_of(train, sparse, False, fl))
    return {n for n, b in PATH_BITS.items() if bits & b}
