"""GPU parity: the HIP path (libdstagnn.so through the torch.ops.dstagnn operators)
against the reference's golden vectors and the CPU oracle.

Tolerance (north_star: "outputs matching the CPU reference within 1e-4 fp32"):
    max |hip - ref| <= 1e-4 * max(1, max |ref|)      per tensor
i.e. 1e-4 absolute for O(1) tensors and 1e-4 relative to the tensor's scale for large
gradients (sums over up to B*N*T terms in a different order than the reference).
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def close(a, b, tol=TOL, what=""):
    a = a.detach().float().cpu().numpy() if torch.is_tensor(a) else np.asarray(a, np.float32)
    b = b.detach().float().cpu().numpy() if torch.is_tensor(b) else np.asarray(b, np.float32)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    scale = max(1.0, float(np.abs(b).max()) if b.size else 1.0)
    err = float(np.abs(a - b).max()) if b.size else 0.0
    assert err <= tol * scale, f"{what}: max err {err:.3e} > {tol:.0e} * {scale:.3e}"


def load(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name), allow_pickle=False))


# ---------------------------------------------------------------------------------------
# generic strided GEMM
# ---------------------------------------------------------------------------------------
def _gemm(A, B, C, M, N, K, am, ak, bk, bn, cm, cn, batch=1, az=(0, 0, 0), bz=(0, 0, 0), cz=(0, 0, 0),
          alpha=1.0, beta=0.0, bias=None, relu=0, scratch_mb=64):
    from dstagnn_drought_amd import _lib
    _lib.load().gemm_f32(A, B, C, [M, N, K, batch], _lib.gemm_maps(am, ak, az, bk, bn, bz, cm, cn, cz), [0, 0, 0],
                         alpha, beta, bias, 1, bool(relu))
    torch.cuda.synchronize()


@pytest.mark.parametrize("M,N,K", [(64, 64, 16), (100, 70, 33), (5440, 512, 384), (300, 96, 20000), (7, 3, 1),
                                   (12, 24, 174080), (32, 32, 9000), (5, 7, 4097), (96, 32, 65280),
                                   (40, 17, 20000), (64, 32, 5000)])
def test_gemm_plain(M, N, K):
    _need_gpu()
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g)
    bias = torch.randn(N, generator=g)
    ref = (A.double() @ B.double() + bias.double()).float()
    C = torch.empty(M, N, device="cuda")
    _gemm(A.cuda(), B.cuda(), C, M, N, K, (0, K, 0), (0, 1, 0), (0, N, 0), (0, 1, 0), (0, N, 0), (0, 1, 0),
          bias=bias.cuda())
    close(C, ref, tol=1e-5 * max(1.0, K ** 0.5), what="plain")


def test_gemm_skinny_epilogue():
    """The skinny long-reduction kernel (M, N <= 32, K >= 4096: gemm.hip skinny_dw_kernel, the
    fcmy weight gradient's shape) with a transposed A map, alpha, beta * C and ReLU, and the
    tiled kernel on the same problem (DSTAGNN_GEMM_SKINNY is read once per process, so the
    comparison is against the fp64 product)."""
    _need_gpu()
    g = torch.Generator().manual_seed(11)
    M, N, K = 12, 25, 70001
    A = torch.randn(K, M, generator=g)   # A[m][k] = At[k][m]: m-contiguous, like fcmy's dtc
    B = torch.randn(K, N, generator=g)
    C0 = torch.randn(M, N, generator=g)
    ref = torch.relu(0.5 * (A.double().t() @ B.double()) + 2.0 * C0.double()).float()
    C = C0.clone().cuda()
    _gemm(A.cuda(), B.cuda(), C, M, N, K, (0, 1, 0), (0, M, 0), (0, N, 0), (0, 1, 0), (0, N, 0), (0, 1, 0),
          alpha=0.5, beta=2.0, relu=1)
    close(C, ref, tol=1e-5 * K ** 0.5, what="skinny")
    # deterministic: a second run gives the same bits
    C2 = C0.clone().cuda()
    _gemm(A.cuda(), B.cuda(), C2, M, N, K, (0, 1, 0), (0, M, 0), (0, N, 0), (0, 1, 0), (0, N, 0), (0, 1, 0),
          alpha=0.5, beta=2.0, relu=1)
    assert torch.equal(C, C2)


def test_gemm_skinny_two_level_fold():
    """The skinny kernel with a two-level partial fold (M*N = 3072 outputs over 256 workgroups:
    the aggregate-first dTheta shape, A = agg[b,j,k,f,t] read with a two-level k map) — fp64
    product, and bit-identical reruns (fixed summation order whichever workgroup arrives last)."""
    _need_gpu()
    g = torch.Generator().manual_seed(12)
    BN, K, F, T, C = 5440, 3, 32, 12, 32
    agg = torch.randn(BN, K, F, T, generator=g)
    gp = torch.randn(BN, T, C, generator=g)
    ref = torch.einsum("jkft,jtc->kfc", agg.double(), gp.double()).reshape(K * F, C).float()
    KFT = K * F * T
    outs = []
    for _ in range(3):
        Cd = torch.empty(K * F, C, device="cuda")
        _gemm(agg.cuda(), gp.cuda(), Cd, K * F, C, BN * T, (0, T, 0), (T, 1, KFT), (0, C, 0), (0, 1, 0),
              (0, C, 0), (0, 1, 0))
        outs.append(Cd)
    close(outs[0], ref, tol=1e-5 * (BN * T) ** 0.5, what="skinny two-level")
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


def test_gemm_transposed_batched_two_level():
    """A = x viewed (b,n,f,t) -> rows (b,i,t), k = f (two-level m); C scattered with relu + beta."""
    _need_gpu()
    g = torch.Generator().manual_seed(3)
    Bn, Nn, Fd, T, KC = 3, 17, 5, 12, 9
    x = torch.randn(Bn, Nn, Fd, T, generator=g)
    th = torch.randn(Fd, KC, generator=g)
    C0 = torch.randn(Bn, Nn, KC, T, generator=g)
    ref = torch.relu(torch.einsum("bift,fk->bikt", x, th) * 0.5 + 2.0 * C0)
    C = C0.clone().cuda()
    FT, KCT = Fd * T, KC * T
    _gemm(x.cuda(), th.cuda(), C, Bn * Nn * T, KC, Fd, (T, 1, FT), (0, T, 0), (0, KC, 0), (0, 1, 0),
          (T, 1, KCT), (0, T, 0), alpha=0.5, beta=2.0, relu=1)
    close(C, ref, tol=1e-5, what="two-level")
    # batched over (b,k) with a two-level batch map: C[b,k] = X[b,:,k*4:(k+1)*4] @ Y[b,:,k*4:(k+1)*4]^T
    Kh, dk = 3, 4
    X = torch.randn(Bn, Nn, Kh * dk, generator=g)
    Y = torch.randn(Bn, Nn, Kh * dk, generator=g)
    ref2 = torch.einsum("bikd,bjkd->bkij", X.view(Bn, Nn, Kh, dk), Y.view(Bn, Nn, Kh, dk))
    C2 = torch.empty(Bn, Kh, Nn, Nn, device="cuda")
    ld = Kh * dk
    _gemm(X.cuda(), Y.cuda(), C2, Nn, Nn, dk, (0, ld, 0), (0, 1, 0), (0, 1, 0), (0, ld, 0), (0, Nn, 0), (0, 1, 0),
          batch=Bn * Kh, az=(Kh, dk, Nn * ld), bz=(Kh, dk, Nn * ld), cz=(0, Nn * Nn, 0))
    close(C2, ref2, tol=1e-5, what="batched")


# ---------------------------------------------------------------------------------------
# cheb_conv_withSAt operator vs the reference's golden vectors
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["g1_cheb_pems04.npz", "g5_cheb_dense.npz", "g15_cheb_prod.npz"])
@pytest.mark.parametrize("sparse", [0, 1])
def test_cheb_sat_golden(golden_dir, name, sparse):
    _need_gpu()
    from dstagnn_drought_amd import _lib
    from dstagnn_drought_amd.model import support_index
    ops = _lib.load()
    g = load(golden_dir, name)
    m = json.loads(str(g["meta"]))
    B, N, F, T, K, C = m["B"], m["N"], m["F"], m["T"], m["K"], m["C"]
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    x, sat = cu(g["x"]), cu(g["spatial_attention"])
    thcat = cu(np.concatenate([g[f"Theta_{k}"] for k in range(K)], axis=1))
    mcat = cu(np.stack([g[f"mask_{k}"] for k in range(K)]))
    cheb = cu(np.stack([g[f"cheb_{k}"] for k in range(K)]))
    apa = cu(g["adj_pa"])
    csc_ptr, csc_row, csr_ptr, csr_col = [t.cuda() for t in support_index(cheb.cpu())]
    graph = [cheb, apa, csc_ptr, csc_row, csr_ptr, csr_col]
    out, P, W, xth = ops.cheb_sat_fwd(x, sat, thcat, mcat, graph, C, bool(sparse))
    torch.cuda.synchronize()
    assert tuple(out.shape) == (B, N, C, T) and (W.numel() == 0) == bool(sparse)
    close(out, g["out"], what="out")
    dout = cu(g["g_out"])
    dx, dsat, dth, dm = ops.cheb_sat_bwd(x, thcat, graph, out, P, W, xth, dout, C, bool(sparse))
    torch.cuda.synchronize()
    close(dx, g["grad_x"], what="grad_x")
    close(dsat, g["grad_spatial_attention"], what="grad_sat")
    for k in range(K):
        close(dth[:, k * C:(k + 1) * C], g[f"grad_Theta_{k}"], what=f"grad_Theta_{k}")
        close(dm[k], g[f"grad_mask_{k}"], what=f"grad_mask_{k}")


# ---------------------------------------------------------------------------------------
# DSTAGNN_block (module + autograd Function) vs golden
# ---------------------------------------------------------------------------------------
def _block_from_golden(g, m, num_of_d):
    import dstagnn_drought_amd as D
    cheb = [torch.from_numpy(g[f"cheb_{k}"]) for k in range(m["K"])]
    blk = D.DSTAGNN_block("cpu", num_of_d, num_of_d, m["K"], m["C"], m["C"], 1, cheb, g["adj_pa"], g["adj_tmd"],
                          m["N"], m["T"], m["D"], m["d_k"], m["d_v"], m["n_heads"])
    sd = {k[6:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("param/")}
    blk.load_state_dict(sd)
    return blk.cuda().eval()


@pytest.mark.parametrize("name", ["g2_block_first.npz", "g3_block_inner.npz", "g3b_block_inner_full.npz",
                                  "g13_block_inner_prod.npz", "g14_block_first_prod.npz"])
def test_block_golden(golden_dir, name):
    """The block against the reference's own outputs and gradients (tests/golden/gen_golden.py,
    gen_golden_prod.py).  g13 / g14 are at the production geometry (N=170, F=C=32, T=12, K=3,
    d_k=32): the default path there is the one bench.py times — flash_small_* (fused small-graph
    attention), cheb_agg_* (aggregate-first Chebyshev), tat_fused_* (the temporal-attention stage
    as one kernel per direction), gtu_*_fused (the GTU stage as one kernel per direction) —
    asserted below through the library's own path query (dstagnn_block_paths), so the timed
    kernels are pinned to reference-written vectors directly."""
    _need_gpu()
    from dstagnn_drought_amd import block_fn as bf
    g = load(golden_dir, name)
    m = json.loads(str(g["meta"]))
    blk = _block_from_golden(g, m, m["num_of_d"])
    x = torch.from_numpy(g["x"]).cuda().requires_grad_(True)
    res = torch.from_numpy(g["res_att"]).cuda().requires_grad_(True) if "res_att" in g else 0
    if "_prod" in name:
        assert m["N"] <= bf.FLASH_SMALL_N and m["C"] == 32 and m["T"] == 12 and m["d_k"] == 32
        took = bf.block_paths(blk, x, res)
        want = {"sparse", "flash", "flash_small", "cheb_agg", "tat_fused_fwd", "tat_fused_bwd", "gtu_fused_fwd",
                "gtu_fused_bwd"}
        assert want <= took, f"{name}: kernel path {sorted(took)} lacks {sorted(want - took)}"
    out, re_at = blk(x, res)
    close(out, g["out"], what="out")
    close(re_at, g["re_at"], what="re_at")
    ((out * torch.from_numpy(g["g_out"]).cuda()).sum() + (re_at * torch.from_numpy(g["g_re"]).cuda()).sum()).backward()
    close(x.grad, g["grad_x"], what="grad_x")
    if "grad_res_att" in g:
        close(res.grad, g["grad_res_att"], what="grad_res_att")
    for n, p in blk.named_parameters():
        if "grad/" + n in g:
            assert p.grad is not None, n
            close(p.grad, g["grad/" + n], what=n)
        else:
            assert p.grad is None, f"{n} should keep grad None (quirk 11)"


def test_model_golden(golden_dir):
    _need_gpu()
    import dstagnn_drought_amd as D
    g = load(golden_dir, "g4_model.npz")
    m = json.loads(str(g["meta"]))
    torch.manual_seed(0)
    model = D.make_model("cpu", 1, m["nb_block"], 1, m["K"], m["C"], m["C"], 1, torch.FloatTensor(g["adj_tmd"]),
                         torch.FloatTensor(g["adj_pa"]), torch.FloatTensor(g["adj_tmd"]), m["num_for_predict"],
                         m["T"], m["N"], m["D"], m["d_k"], m["d_k"], m["n_heads"])
    model.load_state_dict({k[6:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("param/")})
    cheb = torch.from_numpy(np.stack([g[f"cheb_{k}"] for k in range(m["K"])]))
    for b in model.BlockList:  # pin the reference's ARPACK lambda_max exactly
        b.cheb_conv_SAt.cheb_stack.copy_(cheb)
    model = model.cuda().eval()
    x = torch.from_numpy(g["x"]).cuda().requires_grad_(True)
    out = model(x)
    close(out, g["out"], what="out")
    loss = torch.nn.SmoothL1Loss()(out, torch.from_numpy(g["target"]).cuda())
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    loss.backward()
    close(x.grad, g["grad_x"], what="grad_x")
    for n, p in model.named_parameters():
        if bool(g["hasgrad/" + n]):
            close(p.grad, g["grad/" + n], what=n)
        else:
            assert p.grad is None, n


# ---------------------------------------------------------------------------------------
# larger shapes vs the CPU oracle (PEMS08 geometry, small batch)
# ---------------------------------------------------------------------------------------
def _scaled_laplacian_fixed_start(W):
    """scaled_Laplacian (lib/utils.py:149-177) with a run-independent lambda_max.  ARPACK's
    default start vector comes from its own RNG, whose state persists across calls, and on
    these non-symmetric L its "LR" answer depends on the start (GAMBIA: 3.392-0.212j vs the
    true 3.4115), so lambda_max (hence T_k) would depend on which tests ran before; at GAMBIA size a
    1e-3 change in T_k moves a pre-ReLU Chebyshev output across 0 and flips one grad_x entry
    by O(1) between an fp32 and an fp64 evaluation.  A fixed start makes each case the same
    case in every run."""
    from scipy.sparse.linalg import eigs
    Lap = np.diag(W.sum(axis=1)) - W
    if W.shape[0] <= 2500:  # exact: ARPACK's "LR" pick on these non-symmetric L is start-dependent
        ev = np.linalg.eigvals(Lap)
        lam = ev[np.argmax(ev.real)].real
    else:
        lam = eigs(Lap, k=1, which="LR", v0=np.random.RandomState(0).rand(W.shape[0]))[0].real
    return (2.0 * Lap) / lam - np.eye(W.shape[0])


def _oracle_case(B, N, T, K, h, D, dk, C, first, res_kind, seed, train=False):
    from oracle import dstagnn_ref as ref
    import dstagnn_drought_amd as D_
    gen = torch.Generator().manual_seed(seed)
    rs = np.random.RandomState(seed)
    tmd = np.eye(N)
    pa = np.zeros((N, N))
    for i in range(N):
        tmd[i, rs.choice(N, 2, replace=False)] = 1.0
        pa[i, rs.choice(N, 4, replace=False)] = 1.0
    Lt = _scaled_laplacian_fixed_start(tmd)
    cheb = [torch.from_numpy(c).float() for c in D_.cheb_polynomial(Lt, K)][:K]
    F = 1 if first else C
    p = ref.random_block_params(gen, F, F, K, C, N, T, D, dk, dk, h)
    x = torch.randn(B, N, F, T, generator=gen)
    if res_kind == 0:
        res = 0
    else:
        res = torch.randn(B, 1 if res_kind == 1 else F, h, T, T, generator=gen)
    return ref, p, x, res, cheb, torch.from_numpy(pa).float(), dict(n_heads=h, d_k=dk, d_v=dk, K=K), gen


@pytest.mark.parametrize("first,res_kind,sparse", [(False, 1, True), (True, 0, True), (False, 2, True),
                                                   (False, 1, False)])
def test_block_vs_oracle_pems08_geometry(first, res_kind, sparse):
    _need_gpu()
    import dstagnn_drought_amd as D_
    B, N, T, K, h, D, dk, C = 2, 170, 12, 3, 3, 512, 32, 32
    ref, p, x, res, cheb, apa, dims, gen = _oracle_case(B, N, T, K, h, D, dk, C, first, res_kind, seed=7)
    g_out = torch.randn(B, N, C, T, generator=gen)
    g_re = torch.randn(B, x.shape[2], h, T, T, generator=gen)
    F = x.shape[2]
    blk = D_.DSTAGNN_block("cpu", F, F, K, C, C, 1, cheb, apa, apa, N, T, D, dk, dk, h)
    blk.load_state_dict(p)
    blk = blk.cuda().eval()
    blk.sparse_cheb = sparse
    xg = x.cuda().requires_grad_(True)
    rg = res.cuda().requires_grad_(True) if torch.is_tensor(res) else 0
    masks = hip_relu_masks(blk, xg, rg)
    relu_aware_mask(ref, p, x, res, cheb, apa, dims, masks, "pems08-geometry")
    out_r, re_r, gx_r, gra_r, grads_r = ref.block_forward_backward(p, x, res, cheb, apa, dims, g_out, g_re,
                                                                   relu_mask=masks[0], tail_masks=masks[1:])
    out, re_at = blk(xg, rg)
    close(out, out_r, what="out")
    close(re_at, re_r, what="re_at")
    ((out * g_out.cuda()).sum() + (re_at * g_re.cuda()).sum()).backward()
    close(xg.grad, gx_r, what="grad_x")
    if torch.is_tensor(res):
        close(rg.grad, gra_r, what="grad_res_att")
    for n, prm in blk.named_parameters():
        if grads_r[n] is None:
            assert prm.grad is None, n
        else:
            close(prm.grad, grads_r[n], what=n)


def test_block_train_mode_dropout_vs_oracle():
    """Train mode: both Dropout(0.05) active; the oracle gets the exact masks the HIP path drew."""
    _need_gpu()
    import dstagnn_drought_amd as D_
    from dstagnn_drought_amd.block_fn import dropout_masks
    B, N, T, K, h, D, dk, C = 2, 40, 12, 3, 3, 64, 16, 32
    ref, p, x, res, cheb, apa, dims, gen = _oracle_case(B, N, T, K, h, D, dk, C, False, 1, seed=11)
    blk = D_.DSTAGNN_block("cpu", C, C, K, C, C, 1, cheb, apa, apa, N, T, D, dk, dk, h)
    blk.load_state_dict(p)
    blk = blk.cuda().train()
    torch.manual_seed(1234)
    xg = x.cuda().requires_grad_(True)
    out, re_at = blk(xg, res.cuda())
    torch.manual_seed(1234)
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    m0, m1 = dropout_masks(blk.meta, x.shape, seed)
    keep = float((m0 > 0).float().mean())
    assert 0.93 < keep < 0.97, keep  # p = 0.05
    pp = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    xx = x.clone().requires_grad_(True)
    out_r, re_r = ref.block_forward(pp, xx, res, cheb, apa, dims, train=True,
                                    drop_masks=(m0.cpu(), m1.cpu().permute(0, 2, 1, 3)), hoist=True)
    close(out, out_r, what="out(train)")
    g_out = torch.randn(out.shape, generator=gen)
    (out * g_out.cuda()).sum().backward()
    (out_r * g_out).sum().backward()
    close(xg.grad, xx.grad, what="grad_x(train)")
    for n, prm in blk.named_parameters():
        if pp[n].grad is not None:
            close(prm.grad, pp[n].grad, what=n + "(train)")


# ---------------------------------------------------------------------------------------
# the other BASELINE configs as parity cases (B=1)
# ---------------------------------------------------------------------------------------
CONFIGS = {
    # name: (N, T, K, h, D, dk, C)
    "pems08": (170, 12, 3, 3, 512, 32, 32),   # the bench geometry
    "pems04": (307, 12, 3, 3, 512, 32, 32),
    "pems07": (883, 12, 3, 4, 512, 32, 32),
    "gambia": (2139, 144, 2, 2, 64, 32, 32),   # long series: sparse Chebyshev rows in 1024-element chunks
    "syn": (4096, 24, 5, 8, 512, 32, 32),
    "t24": (64, 24, 3, 2, 64, 32, 32),         # small graph, T >= 20: the split GTU tail
    # K = 3 at a long series: the aggregate-first backward's LDS image (16 K F T bytes = 221 KB)
    # does not fit, so cheb_agg_ok sends the block down the Theta-first sparse path
    "t144k3": (48, 144, 3, 2, 64, 32, 32),
    # T = 8 / 16 with d_k = 32: the other tile fills of the matrix-core TAt kernels (T = 12 above)
    "t8": (40, 8, 3, 2, 64, 32, 32),
    "t16": (40, 16, 3, 2, 64, 32, 32),
    # h = 3, d_k = 32 at every T the fused temporal-attention kernels admit (tat_fused.hip: the
    # 48-row tile holds 48 / T problems), plus their LDS bound N = 320 and an odd N (no float2 /
    # float4 row loads, a partial 16-node tile)
    "t8h3": (40, 8, 3, 3, 64, 32, 32),
    "t16h3": (40, 16, 3, 3, 64, 32, 32),
    "n320": (320, 12, 3, 3, 64, 32, 32),
    "n101": (101, 12, 3, 3, 64, 32, 32),
    # an odd number of 32-node strips (5): the two-strip small-graph dQ'/dK' kernel's last pair
    # holds one strip (its second pair of waves idle), with N <= 192 so that kernel runs
    "n150": (150, 12, 3, 3, 64, 32, 32),
    # Chebyshev orders 2 and 5 at T <= 16: the sample-pair aggregate-first kernels' other order
    # templates (KM = 2: 8 dot products a batch; KM = 5: 20, reduced as 32)
    "k2t12": (64, 12, 2, 3, 64, 32, 32),
    "k5t8": (40, 8, 5, 3, 64, 32, 32),
}
RELU_EPS = 1e-5  # ReLU decisions may differ from the fp64 oracle's only where |z| <= RELU_EPS * max|z|


def hip_relu_masks(blk, x, res, train=False, seed=0):
    """The HIP forward's decisions at the block's three ReLUs (dstagnn::block_relu_out: the
    sign patterns of the ReLU outputs the forward keeps): model/DSTAGNN_my.py:133 (the
    Chebyshev output, (B,N,C,T) like the oracle's z), :245/:247 and :252 ((B,C,N,T), the
    oracle's tail layout).  train=True with the dropout seed of the run under test."""
    from dstagnn_drought_amd import _lib, block_fn as bf
    names, ps, slots = blk._param_list()
    graph = blk._graph()
    sparse = bf.use_sparse(graph, blk.meta, x.shape[3])
    fl = bf.use_flash(graph, blk.meta, x.shape[3], blk.flash_cheb, x.shape[0])
    if fl:
        graph = blk._flash_graph(graph)
    args = (x.detach().float().contiguous(), bf.res_arg(res, x.shape[2]), list(ps), slots,
            bf.graph_list(graph, sparse, fl), bf.cfg_of(blk.meta), 0.05, int(seed), bf.flags_of(train, sparse, False, fl))
    ops = _lib.load()
    X = ops.block_relu_out(*args, 0)
    tco = ops.block_relu_out(*args, 1)
    r = ops.block_relu_out(*args, 2)
    return ((X > 0).permute(0, 1, 3, 2).contiguous().cpu(), (tco > 0).permute(0, 2, 1, 3).contiguous().cpu(),
            (r > 0).permute(0, 2, 1, 3).contiguous().cpu())


def hip_cheb_relu_mask(blk, x, res, train=False, seed=0):
    """(B,N,C,T) bool: the HIP forward's ReLU decisions at model/DSTAGNN_my.py:133."""
    return hip_relu_masks(blk, x, res, train, seed)[0]


def relu_aware_mask(ref, p, x, res, cheb, apa, dims, mask_hip, what, eps=RELU_EPS, drop_masks=None):
    """Check that the HIP's ReLU decisions differ from the fp64 oracle's only where the fp64
    pre-activation is within RELU_EPS * scale of 0; returns the number of such flips (the
    oracle then evaluates with the HIP's decisions, so a flip cannot fail the value checks
    and a kernel bug cannot hide behind one).  mask_hip: the :133 decisions, or the triple of
    hip_relu_masks (then the tail ReLUs :245/:247 and :252 are checked the same way, each
    given the HIP's earlier decisions).  drop_masks: train mode with these masks."""
    d64 = lambda t: t.double() if torch.is_tensor(t) else t  # noqa: E731
    masks = mask_hip if isinstance(mask_hip, tuple) else (mask_hip,)
    dm = None if drop_masks is None else tuple(d64(m) for m in drop_masks)
    flips = 0
    names = ("z", "z_tco", "z_r")
    for q, m in enumerate(masks):
        # each ReLU's fp64 pre-activation given the HIP's decisions at the ReLUs before it
        kw = {}
        if q >= 1:
            kw["relu_mask"] = masks[0]
        if q >= 2:
            kw["tail_masks"] = (masks[1], torch.ones_like(masks[1]))  # z_r is recorded before its own ReLU
        pre = {}
        with torch.no_grad():
            ref.block_forward({k: d64(v) for k, v in p.items()}, d64(x), d64(res), [d64(c) for c in cheb], d64(apa),
                              dims, train=dm is not None, drop_masks=dm, hoist=True, pre_out=pre, **kw)
        z = pre[names[q]]
        flip = m != (z > 0)
        scale = float(z.abs().max())
        if bool(flip.any()):
            worst = float(z[flip].abs().max())
            assert worst <= eps * scale, \
                f"{what}: ReLU decision ({names[q]}) differs at |z| = {worst:.3e} > {eps} * {scale:.3e}"
        flips += int(flip.sum())
    return flips


TRAIN_SEED = 1234  # torch.manual_seed before a train-mode forward: the block draws its dropout seed from it


def _train_seed():
    """The dropout seed DSTAGNN_block.forward draws after torch.manual_seed(TRAIN_SEED)
    (model.py: torch.randint(0, 2**62) from the global CPU generator)."""
    torch.manual_seed(TRAIN_SEED)
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def _run_config_vs_oracle(name, first, B, seed=3, flash=None, tol=TOL, relu_eps=RELU_EPS, errs=None, normwise=False,
                          train=False, owns=None, res_kind=None, paths=None):
    """paths: a set of block_fn.PATH_BITS names the library must take for this case (asserted
    before the comparison), or a (must, must_not) pair of sets."""
    import dstagnn_drought_amd as D_
    from dstagnn_drought_amd.block_fn import dropout_masks, block_paths
    N, T, K, h, D, dk, C = CONFIGS[name]
    if res_kind is None:
        res_kind = 0 if first else 1
    ref, p, x, res, cheb, apa, dims, gen = _oracle_case(B, N, T, K, h, D, dk, C, first, res_kind, seed=seed)
    g_out = torch.randn(B, N, C, T, generator=gen)
    g_re = torch.randn(B, x.shape[2], h, T, T, generator=gen)
    F = x.shape[2]
    blk = D_.DSTAGNN_block("cpu", F, F, K, C, C, 1, cheb, apa, apa, N, T, D, dk, dk, h)
    blk.load_state_dict(p)
    blk = blk.cuda().train(train)
    blk.flash_cheb = flash
    xg = x.cuda().requires_grad_(True)
    rg = res.cuda().requires_grad_(True) if torch.is_tensor(res) else 0
    if paths is not None:
        must, must_not = paths if isinstance(paths, tuple) else (paths, set())
        took = block_paths(blk, xg, rg, train=train)
        assert must <= took and not (must_not & took), f"{name}: kernel path {sorted(took)}, expected " \
                                                       f"{sorted(must)} and none of {sorted(must_not)}"
    dseed = _train_seed() if train else 0
    dm = None
    if train:
        # the exact keep-masks (0 or 1/(1-p)) the HIP forward draws for this seed, handed to
        # the oracle: EmbedS (B,N,D) as drawn, fcmy (B,N,C,T) -> the oracle's (B,C,N,T)
        m0, m1 = dropout_masks(blk.meta, x.shape, dseed)
        keep = float((m0 > 0).float().mean())
        assert 0.94 < keep < 0.96, keep  # p = 0.05 over B*N*D draws
        dm = (m0.cpu(), m1.cpu().permute(0, 2, 1, 3).contiguous())
    masks = hip_relu_masks(blk, xg, rg, train=train, seed=dseed)  # all three ReLUs (:133, :247, :252)
    flips = relu_aware_mask(ref, p, x, res, cheb, apa, dims, masks, name, eps=relu_eps, drop_masks=dm)
    d64 = lambda t: t.double() if torch.is_tensor(t) else t  # noqa: E731
    out_r, re_r, gx_r, gra_r, grads_r = ref.block_forward_backward(
        {k: d64(v) for k, v in p.items()}, d64(x), d64(res), [d64(c) for c in cheb], d64(apa), dims, d64(g_out),
        d64(g_re), relu_mask=masks[0], tail_masks=masks[1:], train=train,
        drop_masks=None if dm is None else tuple(d64(m) for m in dm))
    o32 = ref.block_forward_backward(p, x, res, cheb, apa, dims, g_out, g_re, relu_mask=masks[0], tail_masks=masks[1:],
                                     train=train, drop_masks=dm)
    ref32 = {"out": o32[0], "re_at": o32[1], "grad_x": o32[2], "grad_res_att": o32[3], **o32[4]}

    def close_cal(a, b, key):
        b32 = ref32[key]
        scale = max(1.0, float(b.abs().max()))
        own = float((b32.double() - b).abs().max()) if b32 is not None else 0.0
        d = a.detach().double().cpu() - b
        if normwise:  # ||a - b||_2 / ||b||_2 (reduced-precision variants)
            nb = max(float(b.norm()), 1e-30)
            err, own_n = float(d.norm()) / nb, (float((b32.double() - b).norm()) / nb if b32 is not None else 0.0)
            if errs is not None:
                errs[key] = err
            assert err <= max(tol, 2.0 * own_n), f"{name} {key}: normwise err {err:.3e} > {tol:.1e}"
            return
        bound = max(tol * scale, 2.0 * own)
        err = float(d.abs().max())
        if errs is not None:
            errs[key] = err / scale
        if owns is not None:
            owns[key] = own / scale
        assert err <= bound, f"{name} {key}: max err {err:.3e} > bound {bound:.3e} (fp32 reference's own {own:.3e})"

    if train:
        torch.manual_seed(TRAIN_SEED)  # the forward draws dseed again
    out, re_at = blk(xg, rg)
    close_cal(out, out_r, "out")
    close_cal(re_at, re_r, "re_at")
    ((out * g_out.cuda()).sum() + (re_at * g_re.cuda()).sum()).backward()
    close_cal(xg.grad, gx_r, "grad_x")
    if torch.is_tensor(res):
        close_cal(rg.grad, gra_r, "grad_res_att")
    for n, prm in blk.named_parameters():
        if grads_r[n] is None:
            assert prm.grad is None, n
        else:
            close_cal(prm.grad, grads_r[n], n)
    return flips


@pytest.mark.parametrize("name,first,B,flash", [
    ("pems04", False, 1, None), ("pems07", False, 1, None), ("gambia", True, 1, None), ("gambia", False, 1, None),
    ("syn", False, 1, None), ("t24", True, 1, None), ("t24", False, 1, None), ("pems08", False, 32, None),
    # the fused (flash) Chebyshev attention is automatic on the sparse path: N <= 512 the
    # LDS-staged small-graph kernels (pems08, pems04, t24 above), larger N the streamed kernels
    # (pems07, gambia, syn); forced off at small, middle and large N, so the dense softmax path
    # is held to the oracle everywhere too
    ("pems07", False, 2, False), ("pems08", False, 4, False), ("pems08", True, 2, False), ("pems04", False, 2, False),
    ("t24", False, 2, False), ("gambia", False, 1, False), ("t144k3", False, 2, None), ("t144k3", True, 1, None),
    ("t8", False, 3, None), ("t16", False, 2, None), ("t16", True, 2, None),
    ("n150", False, 3, None), ("n150", True, 2, None), ("k2t12", False, 3, None), ("k2t12", True, 2, None),
    ("k5t8", False, 3, None), ("k5t8", True, 2, None)])
def test_block_vs_oracle_configs(name, first, B, flash):
    """Held against the oracle evaluated in float64 (pems08 at B=32: the bench configuration
    itself).  Bound per tensor: the stated 1e-4 (scaled by max(1, max|ref|)), or twice the
    error of the reference's own fp32 arithmetic (the fp32 oracle vs fp64) where that is larger
    — at these sizes a gradient summed over up to 3e5 terms (GAMBIA dTheta: B*N*T) carries
    ~1.5e-4 of fp32 rounding in the reference itself, so no fp32 implementation meets a flat
    1e-4 there.  ReLU-aware: the Chebyshev ReLU (:133) decisions of the HIP forward may differ
    from the fp64 oracle's only where |z| <= 1e-5 * max|z| (checked, counted); the oracle then
    takes the HIP's decisions, so such a flip cannot fail the value checks."""
    _need_gpu()
    flips = _run_config_vs_oracle(name, first, B, flash=flash)
    print(f"{name} B={B} flash={flash}: {flips} ReLU decision(s) within rounding of 0")


TF_FWD, TF_BWD = "tat_fused_fwd", "tat_fused_bwd"


@pytest.mark.parametrize("name,first,res_kind,B,train,fwd,bwd", [
    # T = 8 / 16 (the other row tilings of the 48-row tile: 6 / 3 problems per workgroup)
    ("t8h3", True, 0, 2, False, True, True), ("t8h3", False, 2, 2, False, True, True),
    ("t8h3", False, 2, 3, True, True, True), ("t8h3", True, 0, 7, True, True, True),
    ("t16h3", True, 0, 2, False, True, True), ("t16h3", False, 2, 2, False, True, True),
    ("t16h3", False, 2, 3, True, True, True), ("t16h3", True, 0, 4, True, True, True),
    # broadcast res_att at T = 8 / 16: F T is not a multiple of 48, so the in-kernel res_att fold
    # cannot own whole samples — fused forward, unfused backward (the mixed pairing)
    ("t8h3", False, 1, 2, False, True, False), ("t16h3", False, 1, 2, True, True, False),
    # T = 12 at the LDS bound N = 320 and at an odd N (scalar row loads, partial node tile)
    ("n320", False, 1, 2, False, True, True), ("n320", True, 0, 2, True, True, True),
    ("n101", False, 1, 2, False, True, True), ("n101", False, 2, 2, True, True, True),
    ("n101", True, 0, 3, False, True, True)])
def test_tat_fused_variants_vs_oracle(name, first, res_kind, B, train, fwd, bwd):
    """every fused temporal-attention instantiation the gate admits
    (tat_fused_fwd_ok: h = 3, d_k = 32, T in {8, 12, 16}, N <= 320) held to the fp64 oracle,
    first and inner block, eval and train, with the path asserted (block_fn.block_paths)."""
    _need_gpu()
    must = ({TF_FWD} if fwd else set()) | ({TF_BWD} if bwd else set())
    must_not = set() if bwd else {TF_BWD}
    flips = _run_config_vs_oracle(name, first, B, train=train, res_kind=res_kind, paths=(must, must_not))
    print(f"{name} first={first} res={res_kind} B={B} train={train}: {flips} ReLU decision(s) within rounding of 0")


@pytest.mark.parametrize("name,first,B,flash", [("pems08", False, 32, None), ("pems08", True, 32, None),
                                                ("pems08", False, 4, False), ("pems07", False, 2, None)])
def test_block_train_mode_vs_oracle_configs(name, first, B, flash):
    """TRAIN mode at the bench's own size (PEMS08 inner block, B=32: the timed path of
    bench.py, both Dropout(0.05) of model/DSTAGNN_my.py:218,221 active at :234,:243): the
    fp64 oracle gets the exact keep-masks the HIP forward drew (dstagnn::dropout_masks for the
    same seed), then out, re_At, grad_x, grad_res_att and every parameter gradient are held to
    the same bound as the eval-mode cases above (1e-4 * max(1, max|ref|), or twice the fp32
    reference's own error where larger).  Also the first block and the fused attention."""
    _need_gpu()
    flips = _run_config_vs_oracle(name, first, B, flash=flash, train=True)
    print(f"train {name} first={first} B={B} flash={flash}: {flips} ReLU decision(s) within rounding of 0")


@pytest.mark.parametrize("name,B,flash", [("pems08", 96, True), ("pems07", 66, True)])
def test_flash_large_batch_vs_oracle(name, B, flash):
    """The fused Chebyshev attention at a batch in (64, 128] against the fp64 oracle: the
    large-graph mask-gradient kernel gives every lane two batch elements there (b and b + 64),
    a lane group no B <= 64 case reaches, and the small-graph kernels sum the batch in one
    thread.  (A direct flash-vs-unfused comparison is not a sound test: the two paths round
    the Chebyshev pre-activation differently, so a ReLU decision within rounding of 0 may
    differ between them — the oracle comparison is ReLU-aware.)"""
    _need_gpu()
    flips = _run_config_vs_oracle(name, False, B, flash=flash)
    print(f"{name} B={B} flash={flash}: {flips} ReLU decision(s) within rounding of 0")


BF16_TOL = 3e-2      # bf16-operand GEMM variant: normwise ||err||_2 / ||ref||_2 <= BF16_TOL per tensor
BF16_RELU_EPS = 2e-2  # ... and its ReLU decisions may differ where |z| <= BF16_RELU_EPS * max|z|


@pytest.mark.parametrize("name,first,B", [("pems08", False, 32), ("pems08", True, 2), ("pems04", False, 2)])
def test_bf16_gemm_variant(name, first, B):
    """The opt-in bf16 GEMM variant (dstagnn::set_gemm_bf16(1): every contraction on
    v_mfma_f32_32x32x16_bf16 with operands rounded to bf16, fp32 accumulation; softmax,
    LayerNorm, fused attention and reductions in fp32) against the fp64 oracle, forward and
    every gradient, at the stated normwise BF16_TOL (a max-abs bound is meaningless here: the
    block's second ReLU (:252) flips wherever its input is within bf16 rounding of 0, an O(1)
    change of one gradient element).  The default fp32 path is held to 1e-4 max-abs above.
    Scope: the PEMS geometries (BASELINE config 2 is PEMS08).  Measured worst cases: PEMS08
    B=32 1.5e-2, first block 2.1e-2 (LayerNorm bias grads, cancelling sums); on the synthetic
    T=24 graph the attention-mask gradient (a softmax-backward sum) reaches 8e-2, outside the
    stated bound, so the variant is not claimed there."""
    _need_gpu()
    from dstagnn_drought_amd import _lib
    ops = _lib.load()
    prev = ops.set_gemm_bf16(1)
    errs = {}
    try:
        flips = _run_config_vs_oracle(name, first, B, tol=BF16_TOL, relu_eps=BF16_RELU_EPS, errs=errs, normwise=True)
    finally:
        ops.set_gemm_bf16(prev)
    worst = max(errs.items(), key=lambda kv: kv[1])
    print(f"bf16 {name} B={B}: worst normwise err {worst[1]:.2e} ({worst[0]}), {flips} ReLU flips; "
          + " ".join(f"{k}={v:.1e}" for k, v in sorted(errs.items())))
    assert prev == 0


# ---------------------------------------------------------------------------------------
# full-batch code paths: samples are independent (no BatchNorm, per-sample softmax / LN), so
# out[b], re_At[b], grad_x[b], grad_res_att[b] of a full-batch run must equal a B=1 run on
# x[b:b+1].  Reaches what the B<=2 oracle cases cannot: the bench batch, GAMBIA's row-chunked
# fcmy GEMM (B*N*C > 2^28 / (3T-12) rows), SYN's (B,K,N,N) score tensor of > 2^31 elements.
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("name,B,samples", [("pems08", 32, (0, 13, 31)), ("pems07", 12, (0, 7, 11)),
                                            ("gambia", 12, (0, 10, 11)), ("syn", 32, (0, 31))])
def test_batch_consistency(name, B, samples):
    """With split-K off (dstagnn::set_splitk_target(1): every reduction in one fixed order)
    the per-sample results (out, re_At, grad_x, grad_res_att) must be BIT-identical; with the
    default split-K policy (a B=1 GEMM may split a reduction the B=32 one does not) the
    forward outputs within the stated 1e-4 * scale."""
    _need_gpu()
    import dstagnn_drought_amd as D_
    from dstagnn_drought_amd import _lib
    ops = _lib.load()
    N, T, K, h, D, dk, C = CONFIGS[name]
    ref, p, x, res, cheb, apa, dims, gen = _oracle_case(B, N, T, K, h, D, dk, C, False, 1, seed=5)
    g_out = torch.randn(B, N, C, T, generator=gen)
    g_re = torch.randn(B, C, h, T, T, generator=gen)
    blk = D_.DSTAGNN_block("cpu", C, C, K, C, C, 1, cheb, apa, apa, N, T, D, dk, dk, h)
    blk.load_state_dict(p)
    blk = blk.cuda().eval()

    def run(sl):
        xg = x[sl].cuda().requires_grad_(True)
        rg = res[sl].cuda().requires_grad_(True)
        out, re_at = blk(xg, rg)
        ((out * g_out[sl].cuda()).sum() + (re_at * g_re[sl].cuda()).sum()).backward()
        r = [t.detach() for t in (out, re_at, xg.grad, rg.grad)]
        for prm in blk.parameters():
            prm.grad = None
        return r

    for exact in (True, False):
        prev = ops.set_splitk_target(1 if exact else 0)
        try:
            full = run(slice(0, B))
            torch.cuda.synchronize()
            assert all(bool(torch.isfinite(t).all()) for t in full), "non-finite values in the full-batch run"
            for b in samples:
                one = run(slice(b, b + 1))
                for what, a, o in zip(("out", "re_at", "grad_x", "grad_res_att"), full, one):
                    a = a[b:b + 1]
                    if exact:
                        assert torch.equal(a, o), f"{name} B={B} sample {b} {what}: not bit-identical " \
                                                  f"(max diff {float((a - o).abs().max()):.3e})"
                    elif what in ("out", "re_at"):
                        # gradients only in the exact pass: with a different summation order a
                        # Chebyshev pre-activation within rounding of 0 may take the other ReLU
                        # branch (an O(1) change of a few grad_x entries, see relu_aware_mask)
                        scale = max(1.0, float(o.abs().max()))
                        err = float((a - o).abs().max())
                        assert err <= TOL * scale, f"{name} B={B} sample {b} {what}: {err:.3e} > {TOL} * {scale:.3e}"
        finally:
            ops.set_splitk_target(prev)


@pytest.mark.parametrize("name,B,samples", [("pems08", 32, (0, 13, 30)), ("pems07", 12, (0, 5, 10))])
def test_batch_consistency_train(name, B, samples):
    """Train mode (both dropouts on, one seed): the keep-mask of sample b depends only on
    (seed, b, position), never on the batch size, and sample b's results do not depend on the
    other samples.  So a run on the prefix x[:b+1] with the same seed must give sample b
    BIT-identically to the full-batch run (split-K off: every reduction in one fixed order),
    and its masks must equal the full batch's masks of sample b."""
    _need_gpu()
    import dstagnn_drought_amd as D_
    from dstagnn_drought_amd import _lib
    from dstagnn_drought_amd.block_fn import dropout_masks
    ops = _lib.load()
    N, T, K, h, D, dk, C = CONFIGS[name]
    ref, p, x, res, cheb, apa, dims, gen = _oracle_case(B, N, T, K, h, D, dk, C, False, 1, seed=9)
    g_out = torch.randn(B, N, C, T, generator=gen)
    g_re = torch.randn(B, C, h, T, T, generator=gen)
    blk = D_.DSTAGNN_block("cpu", C, C, K, C, C, 1, cheb, apa, apa, N, T, D, dk, dk, h)
    blk.load_state_dict(p)
    blk = blk.cuda().train()
    dseed = _train_seed()
    full_m = dropout_masks(blk.meta, x.shape, dseed)

    def run(n):
        xg = x[:n].cuda().requires_grad_(True)
        rg = res[:n].cuda().requires_grad_(True)
        torch.manual_seed(TRAIN_SEED)
        out, re_at = blk(xg, rg)
        ((out * g_out[:n].cuda()).sum() + (re_at * g_re[:n].cuda()).sum()).backward()
        r = [t.detach() for t in (out, re_at, xg.grad, rg.grad)]
        for prm in blk.parameters():
            prm.grad = None
        return r

    prev = ops.set_splitk_target(1)
    try:
        full = run(B)
        torch.cuda.synchronize()
        assert all(bool(torch.isfinite(t).all()) for t in full), "non-finite values in the full-batch run"
        for b in samples:
            pre_m = dropout_masks(blk.meta, (b + 1,) + tuple(x.shape[1:]), dseed)
            for a, o in zip(full_m, pre_m):
                assert torch.equal(a[b], o[b]), f"{name}: dropout mask of sample {b} depends on the batch size"
            one = run(b + 1)
            for what, a, o in zip(("out", "re_at", "grad_x", "grad_res_att"), full, one):
                assert torch.equal(a[b], o[b]), f"{name} train B={B} sample {b} {what}: not bit-identical " \
                                                f"(max diff {float((a[b] - o[b]).abs().max()):.3e})"
    finally:
        ops.set_splitk_target(prev)


# ---------------------------------------------------------------------------------------
# model head (final_conv + final_fc over the block outputs, head.hip) vs the oracle
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("B,N,C,T,nb,P", [(8, 170, 32, 12, 4, 12), (3, 37, 16, 12, 2, 5), (2, 883, 32, 12, 4, 12)])
def test_head_vs_oracle(B, N, C, T, nb, P):
    _need_gpu()
    from oracle import dstagnn_ref as ref
    from dstagnn_drought_amd.head_fn import DSTAGNNHeadFunction
    gen = torch.Generator().manual_seed(B * 1000 + N)
    O = 128
    outs = [torch.randn(B, N, C, T, generator=gen) for _ in range(nb)]
    final = {"final_conv.weight": torch.randn(O, nb * T, 1, C, generator=gen) * 0.05,
             "final_conv.bias": torch.randn(O, generator=gen),
             "final_fc.weight": torch.randn(P, O, generator=gen) * 0.1,
             "final_fc.bias": torch.randn(P, generator=gen)}
    dy = torch.randn(B, N, P, generator=gen)
    # oracle forward + autograd
    fr = {k: v.clone().requires_grad_(True) for k, v in final.items()}
    orr = [o.clone().requires_grad_(True) for o in outs]
    y_ref = ref.model_head(fr, orr)
    y_ref.backward(dy)
    # HIP
    fg = {k: v.cuda().requires_grad_(True) for k, v in final.items()}
    og = [o.cuda().requires_grad_(True) for o in outs]
    y = DSTAGNNHeadFunction.apply(fg["final_conv.weight"], fg["final_conv.bias"], fg["final_fc.weight"],
                                  fg["final_fc.bias"], *og)
    y.backward(dy.cuda())
    close(y, y_ref, what="y")
    for k in final:
        close(fg[k].grad, fr[k].grad, what=k)
    for j in range(nb):
        close(og[j].grad, orr[j].grad, what=f"d out_{j}")


def test_direct_grads_equal_autograd_grads():
    """set_direct_grads: the block's backward writes .grad itself; values identical to the
    AccumulateGrad path, accumulation across two backward passes included."""
    _need_gpu()
    import dstagnn_drought_amd as D
    B, N, T, K, h, Dm, dk, C = 2, 24, 12, 3, 2, 32, 8, 8
    rs = np.random.RandomState(3)
    tmd = np.eye(N)
    pa = np.zeros((N, N))
    for i in range(N):
        tmd[i, rs.choice(N, 2, replace=False)] = 1.0
        pa[i, rs.choice(N, 3, replace=False)] = 1.0
    cheb = [torch.from_numpy(c_).float() for c_ in D.cheb_polynomial(D.scaled_Laplacian(tmd), K)]
    torch.manual_seed(0)
    blk = D.DSTAGNN_block("cpu", C, C, K, C, C, 1, cheb, pa, tmd, N, T, Dm, dk, dk, h)
    for p in blk.parameters():  # make_model's init (Theta / mask are allocated uninitialised)
        if p.dim() > 1:
            torch.nn.init.xavier_uniform_(p)
        else:
            torch.nn.init.uniform_(p)
    blk = blk.cuda().eval()
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(B, N, C, T, device="cuda", generator=g)
    res = torch.randn(B, 1, h, T, T, device="cuda", generator=g)
    go = torch.randn(B, N, C, T, device="cuda", generator=g)
    gr = torch.randn(B, C, h, T, T, device="cuda", generator=g)

    def grads(direct, passes):
        D.set_direct_grads(blk, direct)
        for p in blk.parameters():
            p.grad = None
        for _ in range(passes):
            o, r = blk(x, res)
            torch.autograd.backward([o, r], [go, gr])
        return {n: (None if p.grad is None else p.grad.clone()) for n, p in blk.named_parameters()}

    for passes in (1, 2):
        a, b = grads(False, passes), grads(True, passes)
        for n in a:
            assert (a[n] is None) == (b[n] is None), n
            if a[n] is not None:
                assert torch.equal(a[n], b[n]), n
    D.set_direct_grads(blk, False)


@pytest.mark.parametrize("N,T,first,sparse", [(170, 12, False, True), (170, 12, True, True), (170, 12, False, False),
                                              (64, 24, False, True), (64, 24, True, True)])
def test_block_never_reads_unwritten_memory(N, T, first, sparse):
    """Every buffer the library writes (save / scratch workspaces, outputs, the flat gradient
    buffer) starts as NaN (block_fn._POISON): the results must be bit-identical to a run on
    whatever the allocator hands back.  Guards the no-memset paths (sparse dW written on the
    support only, split-K slabs, the split GTU tail's dG scratch at T=24)."""
    _need_gpu()
    import dstagnn_drought_amd as D
    from dstagnn_drought_amd import block_fn
    K, h, Dm, dk, C, B = 3, 3, 64, 16, 32, 4
    rs = np.random.RandomState(5)
    tmd = np.eye(N)
    pa = np.zeros((N, N))
    for i in range(N):
        tmd[i, rs.choice(N, 2, replace=False)] = 1.0
        pa[i, rs.choice(N, 4, replace=False)] = 1.0
    cheb = [torch.from_numpy(c_).float() for c_ in D.cheb_polynomial(_scaled_laplacian_fixed_start(tmd), K)][:K]
    F = 1 if first else C
    torch.manual_seed(0)
    blk = D.DSTAGNN_block("cpu", F, F, K, C, C, 1, cheb, pa, tmd, N, T, Dm, dk, dk, h)
    for p in blk.parameters():
        if p.dim() > 1:
            torch.nn.init.xavier_uniform_(p)
        else:
            torch.nn.init.uniform_(p)
    blk = blk.cuda().eval()
    blk.sparse_cheb = sparse
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(B, N, F, T, device="cuda", generator=g)
    res = 0 if first else torch.randn(B, 1, h, T, T, device="cuda", generator=g)
    go = torch.randn(B, N, C, T, device="cuda", generator=g)
    gr = torch.randn(B, F, h, T, T, device="cuda", generator=g)

    def run():
        for p in blk.parameters():
            p.grad = None
        xg = x.clone().requires_grad_(True)
        o, r = blk(xg, res)
        torch.autograd.backward([o, r], [go, gr])
        out = {"out": o.detach().clone(), "re_at": r.detach().clone(), "grad_x": xg.grad.clone()}
        out.update({n: p.grad.clone() for n, p in blk.named_parameters() if p.grad is not None})
        return out

    saved = block_fn._POISON
    try:
        block_fn._POISON = False
        plain = run()
        block_fn._POISON = True
        poisoned = run()
    finally:
        block_fn._POISON = saved
    assert plain.keys() == poisoned.keys()
    for k in plain:
        assert torch.isfinite(poisoned[k]).all(), f"{k}: NaN from an unwritten buffer"
        assert torch.equal(plain[k], poisoned[k]), f"{k}: differs with poisoned buffers"


def test_frozen_anchor_keeps_other_grads():
    """in direct-gradient mode the planned op's only parameter input is one anchor;
    freezing the parameter that was the anchor when the plan was built must not drop the node
    (x needs no gradient, res_att = 0: the first block on raw input) — every other trainable
    parameter still gets its gradient, equal to the unfrozen run's."""
    _need_gpu()
    import dstagnn_drought_amd as D
    B, N, T, K, h, Dm, dk, C = 2, 24, 12, 3, 2, 32, 8, 8
    rs = np.random.RandomState(4)
    tmd = np.eye(N)
    pa = np.zeros((N, N))
    for i in range(N):
        tmd[i, rs.choice(N, 2, replace=False)] = 1.0
        pa[i, rs.choice(N, 3, replace=False)] = 1.0
    cheb = [torch.from_numpy(c_).float() for c_ in D.cheb_polynomial(D.scaled_Laplacian(tmd), K)]
    torch.manual_seed(0)
    blk = D.DSTAGNN_block("cpu", 1, 1, K, C, C, 1, cheb, pa, tmd, N, T, Dm, dk, dk, h)
    for p in blk.parameters():
        if p.dim() > 1:
            torch.nn.init.xavier_uniform_(p)
        else:
            torch.nn.init.uniform_(p)
    blk = D.set_direct_grads(blk.cuda().eval())
    x = torch.randn(B, N, 1, T, device="cuda")
    go = torch.randn(B, N, C, T, device="cuda")

    def run():
        for p in blk.parameters():
            p.grad = None
        out, _ = blk(x, 0)
        out.backward(go)
        return {n: p.grad.clone() for n, p in blk.named_parameters() if p.grad is not None}

    full = run()                       # builds the plan (anchor = first trainable parameter)
    first = next(iter(blk.parameters()))
    first.requires_grad_(False)
    try:
        part = run()
    finally:
        first.requires_grad_(True)
    name0 = next(iter(blk.state_dict()))
    assert name0 not in part
    assert sorted(part) == sorted(k for k in full if k != name0), sorted(set(full) ^ set(part))
    for k in part:
        assert torch.equal(part[k], full[k]), k


def test_dropout_masks_keyed_by_global_sample():
    """Data-parallel shards draw the masks of the concatenated batch: the masks of samples
    [base, base + b) (sample_base = base) are rows [base, base + b) of the full batch's masks."""
    _need_gpu()
    from dstagnn_drought_amd.block_fn import dropout_masks
    meta = dict(n_heads=3, d_k=32, d_v=32, d_model=64, K=3, C=32, drop_p=0.05)
    full = dropout_masks(meta, (8, 30, 32, 12), 12345)
    for base, b in ((0, 3), (3, 5), (6, 2)):
        part = dropout_masks(meta, (b, 30, 32, 12), 12345, sample_base=base)
        for f, q in zip(full, part):
            assert torch.equal(f[base:base + b], q)
