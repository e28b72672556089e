"""CPU, world_size 2 over gloo: the data-parallel exchange step (dstagnn_drought_amd.dp).

Each rank takes a disjoint shard of the global batch, computes block gradients (with the
CPU oracle standing in for the device compute), and GradAllReducer averages them —
bucketed, None grads skipped, cheb mask grads sent as adj_pa-support nnz only.  The
result must equal the full-batch gradient.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(seed=5):
    from oracle import dstagnn_ref as ref
    import dstagnn_drought_amd as D
    B, N, T, K, h, Dm, dk, C = 4, 12, 12, 3, 2, 16, 8, 8
    gen = torch.Generator().manual_seed(seed)
    rs = np.random.RandomState(seed)
    tmd = np.eye(N)
    pa = np.zeros((N, N))
    for i in range(N):
        tmd[i, rs.choice(N, 2, replace=False)] = 1.0
        pa[i, rs.choice(N, 3, replace=False)] = 1.0
    cheb = [torch.from_numpy(c).float() for c in D.cheb_polynomial(D.scaled_Laplacian(tmd), K)][:K]
    p = ref.random_block_params(gen, C, C, K, C, N, T, Dm, dk, dk, h)
    x = torch.randn(B, N, C, T, generator=gen)
    res = torch.randn(B, 1, h, T, T, generator=gen)
    tgt = torch.randn(B, N, C, T, generator=gen)
    dims = dict(n_heads=h, d_k=dk, d_v=dk, K=K)
    return ref, p, x, res, tgt, cheb, torch.from_numpy(pa).float(), dims


def _grads(ref, p, x, res, tgt, cheb, apa, dims):
    pp = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    out, _ = ref.block_forward(pp, x, res, cheb, apa, dims, hoist=True)
    loss = torch.nn.functional.smooth_l1_loss(out, tgt)  # mean over the (local) batch
    loss.backward()
    return {k: v.grad for k, v in pp.items()}


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dstagnn_drought_amd.dp import GradAllReducer, shard_batch
        torch.set_num_threads(1)
        ref, p, x, res, tgt, cheb, apa, dims = _setup()
        full = _grads(ref, p, x, res, tgt, cheb, apa, dims)
        local = _grads(ref, p, shard_batch(x, rank, world), shard_batch(res, rank, world),
                       shard_batch(tgt, rank, world), cheb, apa, dims)
        params = {k: torch.nn.Parameter(v.clone()) for k, v in p.items()}
        for k, prm in params.items():
            prm.grad = None if local[k] is None else local[k].clone()
        sup = {f"cheb_conv_SAt.mask.{k}": apa > 0 for k in range(dims["K"])}
        red = GradAllReducer(params.items(), mask_support=sup, bucket_bytes=4 << 10)
        nb = red.all_reduce()
        errs = {}
        for k, prm in params.items():
            if full[k] is None:
                errs[k] = 0.0 if prm.grad is None else 1.0
            else:
                errs[k] = float((prm.grad - full[k]).abs().max() / max(1.0, float(full[k].abs().max())))
        dense = 4 * sum(v.numel() for v in p.values())
        q.put((rank, nb, max(errs.values()), red.payload_bytes(), dense))
    finally:
        dist.destroy_process_group()


def test_dp_allreduce_matches_full_batch():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank, nb, err, payload, dense in res:
        assert nb >= 2, "expected several buckets with a 4 KB bucket size"
        assert err < 1e-5, err
        assert payload < dense  # sparse mask payload


def test_shard_batch_partitions():
    from dstagnn_drought_amd.dp import shard_batch
    t = torch.arange(10)
    parts = [shard_batch(t, r, 3) for r in range(3)]
    assert torch.equal(torch.cat(parts), t)


def _flat_worker(rank, world, port, q, early=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dstagnn_drought_amd.dp import GradAllReducer
        shapes = [(4, 3), (5,), (2, 2, 2)]
        params = [torch.nn.Parameter(torch.zeros(s)) for s in shapes]
        extra = torch.nn.Parameter(torch.zeros(7))  # a separate gradient: bucketed path
        flat = torch.arange(25, dtype=torch.float32) * (rank + 1)
        for p, g in zip(params, torch._utils._unflatten_dense_tensors(flat, params)):
            p.grad = g
        extra.grad = torch.full((7,), float(rank + 1))
        named = [(f"p{i}", p) for i, p in enumerate(params)] + [("extra", extra)]
        red = GradAllReducer(named)
        if early:  # a direct-grad block's backward node handing its gradients over (attach)
            blk = torch.nn.Module()
            blk.ps = torch.nn.ParameterList(params)
            blk.direct_grads = True
            assert GradAllReducer.block_flat_grad(blk) is flat
            red.on_grads_ready(blk)
            red.on_grads_ready(blk)  # a second hand-over of the same buffer is ignored
            assert len(red._inflight) == 1
            blk.direct_grads = False
            assert GradAllReducer.block_flat_grad(blk) is None
        n = red.all_reduce()
        assert not red._inflight
        mean = sum(r + 1 for r in range(world)) / world
        ok = torch.allclose(flat, torch.arange(25, dtype=torch.float32) * mean) and \
            torch.allclose(extra.grad, torch.full((7,), mean)) and params[0].grad.data_ptr() == flat.data_ptr()
        q.put((rank, n, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("early", [False, True])
def test_flat_gradient_buffer_reduced_in_place(early):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_flat_worker, args=(r, world, port, q, early)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank, n, ok in res:
        assert ok, rank
        assert n == 2  # one flat collective + one bucket
