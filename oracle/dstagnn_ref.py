"""ORACLE — CPU restatement of the reference DSTAGNN block (TEST INFRASTRUCTURE ONLY).

This module is the parity checker for the HIP path.  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import it; the product package
(dstagnn_drought_amd) never does, and fails loudly without its HIP library.

It restates, in plain PyTorch-CPU fp32 functional code, the algorithm of
Ghoul-tn/DSTAGNN_Drought model/DSTAGNN_my.py (snapshot 2025-06-14) and
lib/utils.py, line by line.  Every function cites the reference file:line it
follows.  Parameters are passed as a dict keyed by the reference's state_dict
names (block-local, e.g. "TAt.W_Q.weight"), so the same tensors feed the oracle,
the reference and the HIP path.

Pinned against golden vectors produced by the reference itself
(tests/golden/gen_golden.py -> tests/golden/*.npz, checked by
tests/test_oracle_golden.py).  Backward comes from torch autograd on this
restatement (the reference has no hand-written backward either).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------------------
# graph preprocessing — lib/utils.py:149-203
# ----------------------------------------------------------------------------------------
def scaled_laplacian(W):
    """lib/utils.py:149-177. L~ = 2(D-W)/lambda_max - I, lambda_max by ARPACK eigs(k=1,'LR').
    Tensor input -> float32 tensor (quirk 5), ndarray -> float64 ndarray."""
    from scipy.sparse.linalg import eigs
    is_t = torch.is_tensor(W)
    Wn = W.cpu().numpy() if is_t else W
    assert Wn.shape[0] == Wn.shape[1]
    D = np.diag(np.sum(Wn, axis=1))
    L = D - Wn
    lam = eigs(L, k=1, which="LR")[0].real
    Lt = (2 * L) / lam - np.identity(Wn.shape[0])
    return torch.from_numpy(Lt).float() if is_t else Lt


def cheb_polynomials(L_tilde, K):
    """lib/utils.py:180-203 — ELEMENTWISE recurrence T_k = 2 L~ * T_{k-1} - T_{k-2}."""
    N = L_tilde.shape[0]
    out = [np.identity(N), L_tilde.copy()]
    for i in range(2, K):
        out.append(2 * L_tilde * out[i - 1] - out[i - 2])
    return out


# ----------------------------------------------------------------------------------------
# block pieces — model/DSTAGNN_my.py
# ----------------------------------------------------------------------------------------
def layer_norm(x, w, b, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def embed_t(p, x):
    """Embedding 'T' (:172-176,181): LN_N(x.permute(0,2,3,1) + pos_embed[t])."""
    B, N, Fd, T = x.shape
    emb = x.permute(0, 2, 3, 1) + p["EmbedT.pos_embed.weight"][:T].unsqueeze(0).unsqueeze(0)
    return layer_norm(emb, p["EmbedT.norm.weight"], p["EmbedT.norm.bias"])


def embed_s(p, y):
    """Embedding 'S' (:178-181): LN_D(y + pos_embed[n])."""
    N = y.shape[1]
    return layer_norm(y + p["EmbedS.pos_embed.weight"][:N].unsqueeze(0),
                      p["EmbedS.norm.weight"], p["EmbedS.norm.bias"])


def temporal_attention(p, E, res_att, h, dk, dv):
    """MultiHeadAttention.forward (:84-100) + ScaledDotProductAttention.forward (:30-42).
    Softmax over dim=3 (the QUERY axis, quirk 1).  Returns (LN_N(fc(ctx)+E), scores)."""
    B, Fd, T, N = E.shape
    Q = (E @ p["TAt.W_Q.weight"].t()).view(B, Fd, T, h, dk).transpose(2, 3)
    K = (E @ p["TAt.W_K.weight"].t()).view(B, Fd, T, h, dk).transpose(2, 3)
    V = (E @ p["TAt.W_V.weight"].t()).view(B, Fd, T, h, dv).transpose(2, 3)
    scores = torch.matmul(Q, K.transpose(-1, -2)) / np.sqrt(dk) + res_att
    attn = F.softmax(scores, dim=3)
    ctx = torch.matmul(attn, V)
    ctx = ctx.transpose(2, 3).reshape(B, Fd, T, h * dv)
    out = ctx @ p["TAt.fc.weight"].t()
    return layer_norm(out + E, p["TAt.layer_norm.weight"], p["TAt.layer_norm.bias"]), scores


def pre_conv(p, O):
    """pre_conv Conv2d(T->D, kernel (1,F)) (:207,:232): O (B,F,T,N) -> (B,N,D)."""
    return F.conv2d(O.permute(0, 2, 3, 1), p["pre_conv.weight"], p["pre_conv.bias"])[:, :, :, -1].permute(0, 2, 1)


def spatial_attention_scores(p, Z, K, dk):
    """SMultiHeadAttention.forward (:55-67) + SScaledDotProductAttention (:13-22), no softmax."""
    B, N, D = Z.shape
    Q = (Z @ p["SAt.W_Q.weight"].t()).view(B, N, K, dk).transpose(1, 2)
    Kt = (Z @ p["SAt.W_K.weight"].t()).view(B, N, K, dk).transpose(1, 2)
    return torch.matmul(Q, Kt.transpose(-1, -2)) / np.sqrt(dk)


def cheb_conv_sat(x, sat, adj_pa, thetas, masks, cheb, hoist=False, relu_mask=None, pre_out=None):
    """cheb_conv_withSAt.forward (:117-133).  Softmax over dim=1 (source node i, quirk 2).
    hoist=False reproduces the reference's T x K loop literally (the softmax is recomputed
    for every timestep); hoist=True computes it once per k (exact, quirk 3).
    relu_mask (B,N,C,T), optional: the ReLU of :133 takes these decisions instead of z > 0
    (out = z * mask, gradient mask) — a parity test hands in the decisions of the
    implementation under test, valid where they agree with sign(z) or |z| is within
    rounding of 0.  pre_out (dict, optional) receives the pre-activation z under "z"."""
    B, N, Fin, T = x.shape
    Kc = len(thetas)
    C = thetas[0].shape[1]
    if hoist:
        Ws = [cheb[k] * F.softmax(sat[:, k] + adj_pa * masks[k], dim=1) for k in range(Kc)]
    outs = []
    for t in range(T):
        g = x[:, :, :, t]
        o = torch.zeros(B, N, C, dtype=x.dtype)
        for k in range(Kc):
            if hoist:
                Wk = Ws[k]
            else:
                Wk = cheb[k] * F.softmax(sat[:, k] + adj_pa * masks[k], dim=1)
            rhs = Wk.permute(0, 2, 1).matmul(g)
            o = o + rhs.matmul(thetas[k])
        outs.append(o.unsqueeze(-1))
    z = torch.cat(outs, dim=-1)
    if pre_out is not None:
        pre_out["z"] = z.detach()
    if relu_mask is not None:
        return z * relu_mask.to(z.dtype)
    return F.relu(z)


def gtu(p, name, X, k):
    """GTU.forward (:192-197): Conv2d(C->2C,(1,k)), tanh(first C) * sigmoid(last C)."""
    c = F.conv2d(X, p[name + ".con2out.weight"], p[name + ".con2out.bias"])
    C = X.shape[1]
    return torch.tanh(c[:, :C]) * torch.sigmoid(c[:, -C:])


def block_forward(p, x, res_att, cheb, adj_pa, dims, train=False, drop_masks=None, hoist=False, relu_mask=None,
                  pre_out=None, tail_masks=None):
    """DSTAGNN_block.forward (:225-253).  Returns (x_out (B,N,C,T), re_At (B,F,h,T,T)).

    dims: dict(n_heads, d_k, d_v, K).  train=True applies the two Dropout(0.05)
    (:218,:221) using drop_masks=(mask_S (B,N,D), mask_T (B,C,N,T)) already scaled by
    1/(1-p), so a test can inject the exact masks the HIP path drew.
    relu_mask / tail_masks (parity tests): the decisions of the ReLUs at :133 (see
    cheb_conv_sat) and at :245/:247 and :252 ((B,C,N,T) each) taken from the implementation
    under test instead of z > 0; pre_out also receives their pre-activations "z_tco", "z_r"."""
    B, N, Fd, T = x.shape
    h, dk, dv, K = dims["n_heads"], dims["d_k"], dims["d_v"], dims["K"]
    if Fd == 1:
        TEmx = embed_t(p, x)                                            # :227-228
    else:
        TEmx = x.permute(0, 2, 3, 1)                                    # :230
    TATout, re_at = temporal_attention(p, TEmx, res_att, h, dk, dv)    # :231
    x_TAt = pre_conv(p, TATout)                                         # :232
    SEmx = embed_s(p, x_TAt)                                            # :233
    if train and drop_masks is not None:
        SEmx = SEmx * drop_masks[0]                                     # :234
    STAt = spatial_attention_scores(p, SEmx, K, dk)                     # :235
    thetas = [p[f"cheb_conv_SAt.Theta.{k}"] for k in range(K)]
    masks = [p[f"cheb_conv_SAt.mask.{k}"] for k in range(K)]
    spatial_gcn = cheb_conv_sat(x, STAt, adj_pa, thetas, masks, cheb, hoist=hoist, relu_mask=relu_mask,
                                pre_out=pre_out)                        # :236
    X = spatial_gcn.permute(0, 2, 1, 3)                                 # :237
    tc = torch.cat([gtu(p, "gtu3", X, 3), gtu(p, "gtu5", X, 5), gtu(p, "gtu7", X, 7)], dim=-1)  # :238-242
    tc = tc @ p["fcmy.0.weight"].t() + p["fcmy.0.bias"]                 # :243
    if train and drop_masks is not None:
        tc = tc * drop_masks[1]
    relu = (lambda z, m: z * m.to(z.dtype)) if tail_masks is not None else (lambda z, m: F.relu(z))  # noqa: E731
    if Fd == 1:
        z_tco = tc                                                      # :245
        xres = F.conv2d(x.permute(0, 2, 1, 3), p["residual_conv.weight"], p["residual_conv.bias"])  # :249
    else:
        z_tco = X + tc                                                  # :247
        xres = x.permute(0, 2, 1, 3)                                    # :251
    tco = relu(z_tco, tail_masks[0] if tail_masks is not None else None)
    z_r = xres + tco
    if pre_out is not None:
        pre_out["z_tco"], pre_out["z_r"] = z_tco.detach(), z_r.detach()
    out = layer_norm(relu(z_r, tail_masks[1] if tail_masks is not None else None).permute(0, 3, 2, 1),
                     p["ln.weight"], p["ln.bias"]).permute(0, 2, 3, 1)  # :252
    return out, re_at


def model_forward(blocks, final, x, cheb, adj_pa, dims, hoist=False):
    """DSTAGNN_submodule.forward (:271-280)."""
    need = []
    res_att = 0
    for p in blocks:
        x, res_att = block_forward(p, x, res_att, cheb, adj_pa, dims, hoist=hoist)
        need.append(x)
    return model_head(final, need)


def model_head(final, need):
    """cat + final_conv + [..., -1] + final_fc (model/DSTAGNN_my.py:276-280)."""
    fx = torch.cat(need, dim=-1)
    o1 = F.conv2d(fx.permute(0, 3, 1, 2), final["final_conv.weight"], final["final_conv.bias"])[:, :, :, -1].permute(0, 2, 1)
    return o1 @ final["final_fc.weight"].t() + final["final_fc.bias"]


def split_state_dict(sd, nb_block):
    """Split a make_model state_dict into per-block dicts + final-layer dict."""
    blocks = [{} for _ in range(nb_block)]
    final = {}
    for k, v in sd.items():
        if k.startswith("BlockList."):
            _, i, rest = k.split(".", 2)
            blocks[int(i)][rest] = v
        else:
            final[k] = v
    return blocks, final


def block_forward_backward(p, x, res_att, cheb, adj_pa, dims, g_out, g_re, hoist=True, relu_mask=None, pre_out=None,
                           train=False, drop_masks=None, tail_masks=None):
    """Forward + autograd backward of one block with upstream grads (g_out, g_re).
    Returns (out, re_at, grad_x, grad_res_att or None, {param_name: grad or None}).
    relu_mask / pre_out: see cheb_conv_sat; train / drop_masks / tail_masks: see block_forward."""
    pp = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    xx = x.detach().clone().requires_grad_(True)
    ra = res_att.detach().clone().requires_grad_(True) if torch.is_tensor(res_att) else res_att
    out, re_at = block_forward(pp, xx, ra, cheb, adj_pa, dims, train=train, drop_masks=drop_masks, hoist=hoist,
                               relu_mask=relu_mask, pre_out=pre_out, tail_masks=tail_masks)
    loss = (out * g_out).sum()
    if g_re is not None:
        loss = loss + (re_at * g_re).sum()
    loss.backward()
    grads = {k: (v.grad if v.grad is not None else None) for k, v in pp.items()}
    gra = ra.grad if torch.is_tensor(ra) else None
    return out.detach(), re_at.detach(), xx.grad, gra, grads


def param_shapes(num_of_d, in_channels, K, C, Ct, N, T, D, dk, dv, h):
    """State-dict layout of one DSTAGNN_block (:199-223), in registration order."""
    return [
        ("pre_conv.weight", (D, T, 1, num_of_d)), ("pre_conv.bias", (D,)),
        ("EmbedT.pos_embed.weight", (T, N)), ("EmbedT.norm.weight", (N,)), ("EmbedT.norm.bias", (N,)),
        ("EmbedS.pos_embed.weight", (N, D)), ("EmbedS.norm.weight", (D,)), ("EmbedS.norm.bias", (D,)),
        ("TAt.W_Q.weight", (dk * h, N)), ("TAt.W_K.weight", (dk * h, N)), ("TAt.W_V.weight", (dv * h, N)),
        ("TAt.fc.weight", (N, h * dv)), ("TAt.layer_norm.weight", (N,)), ("TAt.layer_norm.bias", (N,)),
        ("SAt.W_Q.weight", (dk * K, D)), ("SAt.W_K.weight", (dk * K, D)),
    ] + [(f"cheb_conv_SAt.Theta.{k}", (in_channels, C)) for k in range(K)] \
      + [(f"cheb_conv_SAt.mask.{k}", (N, N)) for k in range(K)] + [
        ("gtu3.con2out.weight", (2 * Ct, Ct, 1, 3)), ("gtu3.con2out.bias", (2 * Ct,)),
        ("gtu5.con2out.weight", (2 * Ct, Ct, 1, 5)), ("gtu5.con2out.bias", (2 * Ct,)),
        ("gtu7.con2out.weight", (2 * Ct, Ct, 1, 7)), ("gtu7.con2out.bias", (2 * Ct,)),
        ("residual_conv.weight", (Ct, in_channels, 1, 1)), ("residual_conv.bias", (Ct,)),
        ("fcmy.0.weight", (T, 3 * T - 12)), ("fcmy.0.bias", (T,)),
        ("ln.weight", (Ct,)), ("ln.bias", (Ct,)),
    ]


def random_block_params(gen, num_of_d, in_channels, K, C, N, T, D, dk, dv, h, scale=None):
    """Random parameters with the make_model init distribution (:292-296):
    xavier-uniform for dim>1, U(0,1) for 1-D (LayerNorm gamma/beta included)."""
    p = {}
    for name, shape in param_shapes(num_of_d, in_channels, K, C, C, N, T, D, dk, dv, h):
        t = torch.empty(shape)
        if len(shape) > 1:
            fan_in = shape[1] * (int(np.prod(shape[2:])) if len(shape) > 2 else 1)
            fan_out = shape[0] * (int(np.prod(shape[2:])) if len(shape) > 2 else 1)
            a = math.sqrt(6.0 / (fan_in + fan_out))
            t.uniform_(-a, a, generator=gen)
        else:
            t.uniform_(0.0, 1.0, generator=gen)
        p[name] = t
    return p
