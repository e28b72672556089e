"""Sparse vs dense Chebyshev path of one block on the GPU: per-tensor max |diff| of the
outputs and every gradient, for a few (N, T, K, h, D, first) shapes."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dstagnn_drought_amd as D_  # noqa: E402


def case(N, T, K, h, Dm, first, dk=32, C=32, B=1, seed=3):
    rs = np.random.RandomState(seed)
    tmd = np.eye(N)
    pa = np.zeros((N, N))
    for i in range(N):
        tmd[i, rs.choice(N, 2, replace=False)] = 1.0
        pa[i, rs.choice(N, 4, replace=False)] = 1.0
    cheb = [torch.from_numpy(c).float() for c in D_.cheb_polynomial(D_.scaled_Laplacian(tmd), K)][:K]
    F = 1 if first else C
    torch.manual_seed(1)
    apa = torch.from_numpy(pa).float()
    blk = D_.DSTAGNN_block("cpu", F, F, K, C, C, 1, cheb, apa, apa, N, T, Dm, dk, dk, h)
    for p in blk.parameters():
        if p.dim() > 1:
            torch.nn.init.xavier_uniform_(p)
        else:
            torch.nn.init.uniform_(p)
    blk = blk.cuda().eval()
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn(B, N, F, T, device="cuda", generator=g)
    res = torch.randn(B, 1, h, T, T, device="cuda", generator=g) if not first else 0
    go = torch.randn(B, N, C, T, device="cuda", generator=g)
    gr = torch.randn(B, F, h, T, T, device="cuda", generator=g)
    outs = {}
    for sp in (False, True):
        blk.sparse_cheb = sp
        for p in blk.parameters():
            p.grad = None
        xg = x.clone().requires_grad_(True)
        rg = res.clone().requires_grad_(True) if torch.is_tensor(res) else 0
        o, r = blk(xg, rg)
        ((o * go).sum() + (r * gr).sum()).backward()
        d = {"out": o.detach().clone(), "re_at": r.detach().clone(), "grad_x": xg.grad.clone()}
        if torch.is_tensor(rg):
            d["grad_res"] = rg.grad.clone()
        for n, p in blk.named_parameters():
            if p.grad is not None:
                d[n] = p.grad.clone()
        outs[sp] = d
    bad = []
    for k in outs[False]:
        a, b = outs[False][k], outs[True][k]
        e = float((a - b).abs().max()) / max(1.0, float(a.abs().max()))
        if e > 1e-4 or not np.isfinite(e):
            bad.append(f"{k}:{e:.2e}")
    print(f"N={N} T={T} K={K} h={h} D={Dm} first={first}: {'OK' if not bad else ' '.join(bad)}", flush=True)




def test_case(name="gambia", first=False, repeat=2, order=(False, True)):
    """The parity test's own case (oracle params/inputs), both Chebyshev paths vs the fp64 oracle."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    import test_gpu_parity as tp
    N, T, K, h, Dm, dk, C = tp.CONFIGS[name]
    ref, p, x, res, cheb, apa, dims, gen = tp._oracle_case(1, N, T, K, h, Dm, dk, C, first, 0 if first else 1, seed=3)
    g_out = torch.randn(1, N, C, T, generator=gen)
    g_re = torch.randn(1, x.shape[2], h, T, T, generator=gen)
    d64 = lambda t: t.double() if torch.is_tensor(t) else t  # noqa: E731
    out_r, re_r, gx_r, gra_r, grads_r = ref.block_forward_backward(
        {k: d64(v) for k, v in p.items()}, d64(x), d64(res), [d64(c) for c in cheb], d64(apa), dims, d64(g_out),
        d64(g_re))
    F = x.shape[2]
    blk = D_.DSTAGNN_block("cpu", F, F, K, C, C, 1, cheb, apa, apa, N, T, Dm, dk, dk, h)
    blk.load_state_dict(p)
    blk = blk.cuda().eval()
    for sp in list(order) * repeat:
        blk.sparse_cheb = sp
        for q in blk.parameters():
            q.grad = None
        xg = x.cuda().requires_grad_(True)
        rg = res.cuda().requires_grad_(True) if torch.is_tensor(res) else 0
        out, re_at = blk(xg, rg)
        ((out * g_out.cuda()).sum() + (re_at * g_re.cuda()).sum()).backward()
        e = lambda a, b: float((a.detach().double().cpu() - b).abs().max())  # noqa: E731
        msg = f"out {e(out, out_r):.2e} re {e(re_at, re_r):.2e} gx {e(xg.grad, gx_r):.2e}"
        for n, q in blk.named_parameters():
            if q.grad is not None and n in grads_r and grads_r[n] is not None:
                err = e(q.grad, grads_r[n]) / max(1.0, float(grads_r[n].abs().max()))
                if err > 1e-3:
                    msg += f" {n}:{err:.2e}"
        print(f"{name} first={first} sparse={sp}: {msg}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and ":" in sys.argv[1]:
        for spec in sys.argv[1:]:  # name:first:sparse
            nm, fs, sp = spec.split(":")
            test_case(nm, fs == "1", 1, (sp == "1",))
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "poison":
        test_case("pems04", False, 1, (True, False))
        test_case("gambia", False, 1, (True, False))
        test_case("gambia", True, 1, (True, False))
    elif len(sys.argv) > 1 and sys.argv[1] == "seq":
        for nm, fs in [("pems04", False), ("pems07", False), ("gambia", True), ("gambia", False)]:
            test_case(nm, fs, 1, (True,))
    elif len(sys.argv) > 1 and sys.argv[1] == "seq2":
        for nm, fs in [("gambia", True), ("gambia", False)]:
            test_case(nm, fs, 1, (True,))
    elif len(sys.argv) > 1 and sys.argv[1] == "test":
        test_case("gambia", True, 1)
        test_case("gambia", False)
    else:
        for args in [(300, 32, 2, 2, 64, False), (300, 40, 2, 2, 64, False), (300, 144, 2, 2, 64, False),
                     (300, 144, 2, 2, 64, True), (2139, 12, 2, 2, 64, False), (2139, 144, 2, 2, 64, False)]:
            case(*args)
