"""Worker of tests/test_gpu_dp.py (one rank; launched by torch.distributed.run, world 2, both
ranks on cuda:0, gloo over device tensors): a real DSTAGNN_block forward + backward in
direct-gradient mode with GradAllReducer.attach — the overlap path of dp.py that the
driver's RCCL scaling bench runs — against the same gradients reduced without attach.
Writes one JSON record per rank into $DSTAGNN_DP_OUT."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    import dstagnn_drought_amd as D
    from dstagnn_drought_amd.dp import GradAllReducer, mask_support_of
    B, N, T, K, h, Dm, dk, C = 4, 40, 12, 3, 3, 64, 32, 32
    rs = np.random.RandomState(0)
    tmd, pa = np.eye(N), np.zeros((N, N))
    for i in range(N):
        tmd[i, rs.choice([j for j in range(N) if j != i], 2, replace=False)] = 1.0
        pa[i, rs.choice(N, 4, replace=False)] = 1.0
    cheb = [torch.from_numpy(c).float() for c in D.cheb_polynomial(D.scaled_Laplacian(torch.FloatTensor(tmd)).numpy(), K)]
    torch.manual_seed(1)  # identical parameters on both ranks
    blk = D.DSTAGNN_block("cpu", C, C, K, C, C, 1, cheb, pa, tmd, N, T, Dm, dk, dk, h)
    for p in blk.parameters():
        if p.dim() > 1:
            torch.nn.init.xavier_uniform_(p)
        else:
            torch.nn.init.uniform_(p)
    blk = D.set_direct_grads(blk.to(dev).eval())
    gen = torch.Generator(device=dev).manual_seed(100 + rank)  # each rank its own shard
    x = torch.randn(B, N, C, T, device=dev, generator=gen)
    res = torch.randn(B, 1, h, T, T, device=dev, generator=gen)
    g_out = torch.randn(B, N, C, T, device=dev, generator=gen)
    g_re = torch.randn(B, C, h, T, T, device=dev, generator=gen)

    def run(attach):
        for p in blk.parameters():
            p.grad = None
        red = GradAllReducer(blk.named_parameters(), mask_support=mask_support_of(blk))
        blk.grads_ready = None
        if attach:
            red.attach(blk)
        out, re_at = blk(x, res)
        torch.autograd.backward([out, re_at], [g_out, g_re])
        inflight = len(red._inflight)
        flat = GradAllReducer.block_flat_grad(blk)
        red.all_reduce()
        torch.cuda.synchronize()
        grads = {n: p.grad.detach().clone() for n, p in blk.named_parameters() if p.grad is not None}
        return inflight, flat is not None, grads

    n_on, flat_on, g_on = run(True)
    n_off, flat_off, g_off = run(False)
    err = max(float((g_on[k] - g_off[k]).abs().max()) for k in g_off)
    same_keys = sorted(g_on) == sorted(g_off)
    # the reduced gradients are the mean over ranks: all ranks must hold the same values
    probe = torch.stack([g_on[k].abs().sum() for k in sorted(g_on)]).cpu()
    allp = [torch.zeros_like(probe) for _ in range(world)]
    dist.all_gather(allp, probe)
    ranks_agree = all(torch.equal(allp[0], a) for a in allp)
    rec = {"rank": rank, "inflight_with_attach": n_on, "inflight_without": n_off, "flat": flat_on,
           "max_err": err, "same_keys": same_keys, "ranks_agree": ranks_agree}
    with open(os.path.join(os.environ["DSTAGNN_DP_OUT"], f"rank{rank}.json"), "w") as f:
        json.dump(rec, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
