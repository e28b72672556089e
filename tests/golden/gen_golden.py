#!/usr/bin/env python
"""Golden-vector generator (test infrastructure, run ONLY in the build container).

Imports the read-only reference at /root/reference (Ghoul-tn/DSTAGNN_Drought
snapshot 2025-06-14) and writes small float32 fixtures into tests/golden/*.npz.
Nothing from the reference's source text is stored: only inputs, parameters and
the outputs / gradients the reference computed on them.

Fixtures:
  g1_cheb_pems04.npz   cheb_conv_withSAt (model/DSTAGNN_my.py:102-133) on the real
                       PEMS04 STAG graph (AG) + STRG adj_pa, B=1, F=C=8, T=6, K=3.
  g2_block_first.npz   DSTAGNN_block with num_of_d=1 (first block, :225-253).
  g3_block_inner.npz   inner DSTAGNN_block, res_att (B,1,h,T,T).
  g3b_block_inner_full.npz  inner block, res_att (B,F,h,T,T) (3rd block of the chain).
  g4_model.npz         make_model nb_block=3 forward + SmoothL1 + all grads.
  g5_cheb_dense.npz    cheb_conv_withSAt with dense random cheb_polynomials.
  g6_laplacian_pems04.npz  scaled_Laplacian/cheb_polynomial (lib/utils.py:149-203)
                       tensor branch on PEMS04 STAG.
  g9_gambia_error.json the in_channels=4 failure (quirk 8).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py
Skips (exit 0) when /root/reference is absent (e.g. on the GPU box).
"""
import json
import os
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _load_ref():
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    import torch  # noqa: F401
    from model.DSTAGNN_my import make_model, cheb_conv_withSAt
    from lib.utils import scaled_Laplacian, cheb_polynomial
    from lib.dataloader import load_weighted_adjacency_matrix, load_PA
    return dict(make_model=make_model, cheb_conv_withSAt=cheb_conv_withSAt,
                scaled_Laplacian=scaled_Laplacian, cheb_polynomial=cheb_polynomial,
                load_weighted_adjacency_matrix=load_weighted_adjacency_matrix,
                load_PA=load_PA)


def synth_graph(N, seed=0):
    """Synthetic graphs as SURVEY.md §8(d): adj_TMD = self loop + 2 random
    out-neighbours per row; adj_pa = 4 random nnz per row (binary, as load_PA)."""
    rs = np.random.RandomState(seed)
    tmd = np.eye(N)
    pa = np.zeros((N, N))
    for i in range(N):
        nb = rs.choice([j for j in range(N) if j != i], 2, replace=False)
        tmd[i, nb] = 1.0
        pa[i, rs.choice(N, 4, replace=False)] = 1.0
    return tmd, pa


def f32(a):
    import torch
    if torch.is_tensor(a):
        a = a.detach().cpu().numpy()
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def gen_cheb(R, torch, name, cheb_polys, adj_pa, B, F, C, T, K, seed):
    N = adj_pa.shape[0]
    torch.manual_seed(seed)
    mod = R["cheb_conv_withSAt"](K, [torch.from_numpy(np.asarray(c, np.float32)) for c in cheb_polys],
                                 F, C, N, "cpu")
    for p in mod.Theta:
        torch.nn.init.xavier_uniform_(p)
    apa = torch.from_numpy(np.asarray(adj_pa, np.float32))
    with torch.no_grad():
        for p in mod.mask:
            # only adj_pa*mask enters the forward (:126); zero the rest so the fixture compresses
            torch.nn.init.xavier_uniform_(p)
            p.mul_((apa > 0).float())
    x = torch.randn(B, N, F, T, requires_grad=True)
    # coarse-valued scores (multiples of 1/16) keep the fixture small; any real values are valid input
    sat = (torch.randint(-48, 49, (B, K, N, N)).float() / 16.0).requires_grad_(True)
    out = mod(x, sat, apa)
    g = torch.randn_like(out)
    (out * g).sum().backward()
    d = {"x": f32(x), "spatial_attention": f32(sat), "adj_pa": f32(apa), "out": f32(out), "g_out": f32(g),
         "grad_x": f32(x.grad), "grad_spatial_attention": f32(sat.grad)}
    for k in range(K):
        d[f"cheb_{k}"] = f32(cheb_polys[k])
        d[f"Theta_{k}"] = f32(mod.Theta[k])
        d[f"mask_{k}"] = f32(mod.mask[k])
        d[f"grad_Theta_{k}"] = f32(mod.Theta[k].grad)
        d[f"grad_mask_{k}"] = f32(mod.mask[k].grad)
    d["meta"] = np.array(json.dumps(dict(B=B, N=N, F=F, C=C, T=T, K=K)))
    np.savez_compressed(os.path.join(OUT, name), **d)
    print("wrote", name)


def block_fixture(torch, block, x, res_att, seed, name, meta, extra):
    torch.manual_seed(seed + 1000)
    x = x.clone().requires_grad_(True)
    if torch.is_tensor(res_att):
        res_att = res_att.clone().requires_grad_(True)
    out, re_at = block(x, res_att)
    g_out = torch.randn_like(out)
    g_re = torch.randn_like(re_at)
    ((out * g_out).sum() + (re_at * g_re).sum()).backward()
    d = dict(extra)
    d.update({"x": f32(x), "out": f32(out), "re_at": f32(re_at), "g_out": f32(g_out), "g_re": f32(g_re),
              "grad_x": f32(x.grad)})
    if torch.is_tensor(res_att):
        d["res_att"] = f32(res_att)
        d["grad_res_att"] = f32(res_att.grad)
    for n, p in block.named_parameters():
        d["param/" + n] = f32(p)
        if p.grad is not None:
            d["grad/" + n] = f32(p.grad)
    d["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(OUT, name), **d)
    print("wrote", name)


def main():
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return 0
    import torch
    torch.set_num_threads(4)
    R = _load_ref()

    # ---- G6: Laplacian / Chebyshev on PEMS04 STAG (tensor branch, quirk 5) ----
    tmd04 = R["load_weighted_adjacency_matrix"](os.path.join(REF, "data/PEMS04/stag_001_PEMS04.csv"), 307)
    pa04 = R["load_PA"](os.path.join(REF, "data/PEMS04/strg_001_PEMS04.csv"))
    Lt = R["scaled_Laplacian"](torch.FloatTensor(tmd04))
    Ltn = Lt if isinstance(Lt, np.ndarray) else Lt.cpu().numpy()
    cps = R["cheb_polynomial"](Ltn, 3)
    np.savez_compressed(os.path.join(OUT, "g6_laplacian_pems04.npz"), adj_tmd=f32(tmd04), adj_pa=f32(pa04),
                        L_tilde=f32(Ltn), cheb_0=f32(cps[0]), cheb_1=f32(cps[1]), cheb_2=f32(cps[2]))
    print("wrote g6_laplacian_pems04.npz")

    # ---- G1: cheb_conv_withSAt on real PEMS04 graph ----
    gen_cheb(R, torch, "g1_cheb_pems04.npz", cps, pa04, B=1, F=8, C=8, T=6, K=3, seed=11)

    # ---- G5: dense random cheb polynomials ----
    rs = np.random.RandomState(5)
    Nd = 24
    dense = [rs.randn(Nd, Nd) * 0.5 for _ in range(3)]
    _, pad = synth_graph(Nd, seed=3)
    gen_cheb(R, torch, "g5_cheb_dense.npz", dense, pad, B=2, F=6, C=5, T=5, K=3, seed=12)

    # ---- G2 / G3 / G3b / G4: tiny full model, nb_block=3 ----
    N, T, K, C, D, dk, h, B = 16, 12, 3, 8, 32, 8, 3, 2
    tmd, pa = synth_graph(N, seed=0)
    torch.manual_seed(1)
    model = R["make_model"]("cpu", 1, 3, 1, K, C, C, 1, torch.FloatTensor(tmd), torch.FloatTensor(pa),
                            torch.FloatTensor(tmd), 12, T, N, D, dk, dk, h)
    model.eval()
    cheb = model.BlockList[0].cheb_conv_SAt.cheb_polynomials
    graph = {"adj_tmd": f32(tmd), "adj_pa": f32(pa)}
    for k in range(K):
        graph[f"cheb_{k}"] = f32(cheb[k])
    meta = dict(N=N, T=T, K=K, C=C, D=D, d_k=dk, d_v=dk, n_heads=h, B=B, nb_block=3, in_channels=1,
                num_for_predict=12, seed=1)

    # G4 first: full model, whole state dict at init (pins make_model init RNG order)
    torch.manual_seed(21)
    x0 = torch.randn(B, N, 1, T)
    tgt = torch.randn(B, N, 12)
    xin = x0.clone().requires_grad_(True)
    # capture per-block inputs
    acts = []
    hooks = [blk.register_forward_hook(lambda m, i, o: acts.append((i[0].detach().clone(),
                                                                     i[1].detach().clone() if torch.is_tensor(i[1]) else i[1])))
             for blk in model.BlockList]
    out = model(xin)
    for hk in hooks:
        hk.remove()
    loss = torch.nn.SmoothL1Loss()(out, tgt)
    loss.backward()
    d = dict(graph)
    d.update({"x": f32(x0), "target": f32(tgt), "out": f32(out), "loss": np.float32(loss.item()),
              "grad_x": f32(xin.grad)})
    for n, p in model.named_parameters():
        d["param/" + n] = f32(p)
        d["grad/" + n] = f32(p.grad) if p.grad is not None else np.zeros(0, np.float32)
        d["hasgrad/" + n] = np.array(p.grad is not None)
    d["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(OUT, "g4_model.npz"), **d)
    print("wrote g4_model.npz")
    model.zero_grad(set_to_none=True)

    # G2: first block alone (res_att = 0 int, as DSTAGNN_submodule.forward:273)
    block_fixture(torch, model.BlockList[0], acts[0][0], 0, 2, "g2_block_first.npz",
                  dict(meta, num_of_d=1, in_channels_blk=1), graph)
    # G3: inner block, res_att (B,1,h,T,T) as received by block 2
    x1, r1 = acts[1]
    torch.manual_seed(31)
    block_fixture(torch, model.BlockList[1], torch.randn_like(x1), torch.randn_like(r1), 3,
                  "g3_block_inner.npz", dict(meta, num_of_d=C, in_channels_blk=C), graph)
    # G3b: inner block, res_att (B,F,h,T,T) as received by block 3
    x2, r2 = acts[2]
    assert r2.shape[1] == C
    torch.manual_seed(41)
    block_fixture(torch, model.BlockList[2], torch.randn_like(x2), torch.randn_like(r2), 4,
                  "g3b_block_inner_full.npz", dict(meta, num_of_d=C, in_channels_blk=C), graph)

    # ---- G9: GAMBIA in_channels=4 failure (quirk 8) ----
    try:
        torch.manual_seed(1)
        m4 = R["make_model"]("cpu", 4, 2, 4, 2, 8, 8, 1, torch.FloatTensor(tmd), torch.FloatTensor(pa),
                             torch.FloatTensor(tmd), 12, T, N, 16, 8, 8, 2)
        m4(torch.randn(1, N, 4, T))
        err = None
    except Exception as e:  # noqa: BLE001
        err = {"type": type(e).__name__, "message": str(e)}
    with open(os.path.join(OUT, "g9_gambia_error.json"), "w") as f:
        json.dump(err, f, indent=1)
    print("wrote g9_gambia_error.json", err)
    return 0


if __name__ == "__main__":
    sys.exit(main())
