"""Worker of tests/test_gpu_dp.py::test_dp_step_equals_one_gpu_step (one rank; launched by
torch.distributed.run, world 2, both ranks on cuda:0, gloo over device tensors).

SURVEY.md §4.4 / VERDICT r3 item 8: a data-parallel step must be the 1-GPU step on the
concatenated batch (train_DSTAGNN_my.py:148,158: xm.optimizer_step = all-reduce + Adam).  Every
rank builds the same 2-block make_model, then for eval and train mode:
  * DP:  rank r runs its shard x[rB:(r+1)B] (model.DSTAGNN_block keys the dropout masks by the
         global sample index, rank * B + b), SmoothL1, backward with GradAllReducer.attach (the
         RCCL path of the driver's scaling bench), mean all-reduce, Adam step;
  * ref: the same model copy on the whole batch, sample base 0, backward, Adam step.
Both use the driver's optimiser (train.make_adam -> HipAdam, one launch) and take TWO steps, so the
second runs HipAdam's cached fast path on the all-reduced gradients; the second step's
parameters are compared like the first's.
Split-K off (every tiled reduction in one fixed order).  Writes one JSON record per rank."""
import copy
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
    from dstagnn_drought_amd import _lib
    from dstagnn_drought_amd.dp import GradAllReducer, mask_support_of
    from dstagnn_drought_amd.train import make_adam
    ops = _lib.load()
    ops.set_splitk_target(1)
    Bl, N, T, K, h, Dm, dk, C, P = 2, 40, 12, 3, 3, 64, 32, 32, 12
    B = Bl * world
    rs = np.random.RandomState(0)
    adj = np.zeros((N, N))
    for i in range(N):
        for j in rs.choice([q for q in range(N) if q != i], 3, replace=False):
            adj[i, j] = adj[j, i] = 1.0
    pa = (rs.rand(N, N) < 0.1).astype(np.float64)
    torch.manual_seed(1)  # identical parameters on every rank
    base = D.make_model("cpu", 1, 2, 1, K, C, C, 1, adj, pa, adj, P, T, N, Dm, dk, dk, h).to(dev)
    gen = torch.Generator(device=dev).manual_seed(100)  # the same global batch on every rank
    x = torch.randn(B, N, 1, T, device=dev, generator=gen)
    y = torch.randn(B, N, P, device=dev, generator=gen)
    sl = slice(rank * Bl, (rank + 1) * Bl)
    rec = {"rank": rank}
    for mode in ("eval", "train"):
        nets = {}
        for kind in ("dp", "ref"):
            net = D.set_direct_grads(copy.deepcopy(base))
            net.train(mode == "train")
            if kind == "ref":
                D.set_sample_base(net, 0)  # the whole batch on one device
            nets[kind] = net
        red = GradAllReducer(nets["dp"].named_parameters(), mask_support=mask_support_of(nets["dp"])).attach(nets["dp"])
        outs, losses, grads, params, grads2, params2, kinds = {}, {}, {}, {}, {}, {}, {}
        for kind, xb, yb in (("dp", x[sl], y[sl]), ("ref", x, y)):
            net = nets[kind]
            opt = make_adam(net.parameters(), 1e-4)
            kinds[kind] = type(opt).__name__
            for it in range(2):
                opt.zero_grad()
                torch.manual_seed(77 + it)  # the blocks draw the same dropout seeds in both runs
                out = net(xb if it == 0 else xb.flip(-1))
                loss = torch.nn.functional.smooth_l1_loss(out, yb)
                loss.backward()
                if kind == "dp":
                    red.all_reduce()
                    lt = loss.detach().clone()
                    dist.all_reduce(lt)
                    loss = lt / world
                opt.step()
                torch.cuda.synchronize()
                g = {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.grad is not None}
                pr = {n: p.detach().clone() for n, p in net.named_parameters()}
                if it == 0:
                    outs[kind] = out.detach()
                    losses[kind] = float(loss)
                    grads[kind], params[kind] = g, pr
                else:
                    grads2[kind], params2[kind] = g, pr
        fwd_exact = bool(torch.equal(outs["dp"], outs["ref"][sl]))
        fwd_err = float((outs["dp"] - outs["ref"][sl]).abs().max())
        gerr = {n: float((grads["dp"][n] - g).abs().max()) / max(1.0, float(g.abs().max()))
                for n, g in grads["ref"].items()}
        perr = {}
        for n, p in params["ref"].items():
            if n.endswith("fcmy.0.bias"):
                continue
            d = (params["dp"][n] - p).abs()
            g = grads["ref"].get(n)
            if g is not None:
                # Adam's first step moves an element by lr * g / (|g| + eps): where |g| is at the
                # rounding level of the two summation orders its sign is not determined, so the
                # update is compared where |g| > 1e-3 * max|g| of the tensor
                d = d[g.abs() > 1e-3 * float(g.abs().max())]
            perr[n] = (float(d.max()) if d.numel() else 0.0) / max(1.0, float(p.abs().max()))
        perr2 = {}  # after the second (cached-plan) HipAdam step
        for n, p in params2["ref"].items():
            if n.endswith("fcmy.0.bias"):
                continue
            d = (params2["dp"][n] - p).abs()
            g1, g2 = grads["ref"].get(n), grads2["ref"].get(n)
            if g1 is not None and g2 is not None:
                d = d[(g1.abs() > 1e-3 * float(g1.abs().max())) & (g2.abs() > 1e-3 * float(g2.abs().max()))]
            perr2[n] = (float(d.max()) if d.numel() else 0.0) / max(1.0, float(p.abs().max()))
        rec[mode] = {"fwd_exact": fwd_exact, "fwd_err": fwd_err, "loss_dp": losses["dp"], "loss_ref": losses["ref"],
                     "same_grad_keys": sorted(grads["dp"]) == sorted(grads["ref"]),
                     "grad_err": max(gerr.values()), "grad_worst": max(gerr, key=gerr.get),
                     "param_err": max(perr.values()), "param_worst": max(perr, key=perr.get),
                     "param_err2": max(perr2.values()), "param_worst2": max(perr2, key=perr2.get),
                     "optimizer": kinds}
    with open(os.path.join(os.environ["DSTAGNN_DP_OUT"], f"equiv_rank{rank}.json"), "w") as f:
        json.dump(rec, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
