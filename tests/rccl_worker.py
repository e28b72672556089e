"""Worker of tests/test_gpu_dp.py::test_rccl_world1_reducer: the RCCL path of
the driver's scaling bench, exercised on the one GPU a lease has — world size 1, backend "nccl"
(RCCL on ROCm), `init_process_group(..., device_id=cuda:local)` exactly as bench.py's init_ranks
does for world > 1 (reference: xm.optimizer_step's all-reduce, train_DSTAGNN_my.py:148,158).

The bench block (PEMS08 geometry, B=32, train mode, direct gradients) runs:
  * plain: forward + backward, no reducer;
  * rccl:  the same step with GradAllReducer.attach — the block's flat gradient buffer is
           all-reduced asynchronously from the post-hook on the dstagnn::block autograd node, on
           RCCL's stream beside the library's side stream — then reducer.all_reduce();
and checks that the hook issued the collective, that the collective completed and that the
reduced gradients equal the plain ones bit for bit (a sum over one rank, divided by 1).  The
per-step cost of the reducer is the timed difference of the two loops.  One JSON record."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    import bench
    from dstagnn_drought_amd.dp import GradAllReducer, mask_support_of
    blk, _, _ = bench.build_block(dev)
    c = bench.CFG
    B = c["B"]
    gen = torch.Generator(device=dev).manual_seed(100)
    x = torch.randn(B, c["N"], c["C"], c["T"], device=dev, generator=gen)
    res = torch.randn(B, 1, c["n_heads"], c["T"], c["T"], device=dev, generator=gen)
    g_out = torch.randn(B, c["N"], c["C"], c["T"], device=dev, generator=gen)
    g_re = torch.randn(B, c["C"], c["n_heads"], c["T"], c["T"], device=dev, generator=gen)
    params = list(blk.parameters())
    red = GradAllReducer(blk.named_parameters(), mask_support=mask_support_of(blk))
    seen = {"inflight": []}

    def step(reducer):
        for p in params:
            p.grad = None
        torch.manual_seed(5)  # the same dropout seed in both variants
        out, re_at = blk(x, res)
        torch.autograd.backward([out, re_at], [g_out, g_re])
        if reducer is not None:
            seen["inflight"].append(len(reducer._inflight))
            reducer.all_reduce()

    def grads():
        torch.cuda.synchronize()
        return {n: p.grad.detach().clone() for n, p in blk.named_parameters() if p.grad is not None}

    blk.grads_ready = None
    step(None)
    g_plain = grads()
    red.attach(blk)
    step(red)
    g_rccl = grads()
    exact = sorted(g_plain) == sorted(g_rccl) and all(torch.equal(g_plain[k], g_rccl[k]) for k in g_plain)
    # a plain collective on RCCL as well: world 1 sum of a known tensor
    t = torch.arange(8, device=dev, dtype=torch.float32)
    dist.all_reduce(t)
    coll_ok = bool(torch.equal(t.cpu(), torch.arange(8, dtype=torch.float32)))

    def timed(reducer, n=30, w=5):
        if reducer is None:
            blk.grads_ready = None
        else:
            reducer.attach(blk)
        for _ in range(w):
            step(reducer)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            step(reducer)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    ms = {}
    for rnd in range(2):  # interleaved
        ms.setdefault("plain", []).append(timed(None))
        ms.setdefault("rccl", []).append(timed(red))
    plain, rccl = min(ms["plain"]), min(ms["rccl"])
    rec = {"backend": dist.get_backend(), "world": dist.get_world_size(), "exact": exact, "collective_ok": coll_ok,
           "hook_inflight": seen["inflight"][0] if seen["inflight"] else 0,
           "grad_bytes": int(sum(g.numel() for g in g_plain.values()) * 4),
           "ms_per_step_plain": round(plain, 4), "ms_per_step_rccl": round(rccl, 4),
           "reducer_ms_per_step": round(rccl - plain, 4), "rounds": ms}
    print(json.dumps(rec), flush=True)
    with open(os.path.join(os.environ["DSTAGNN_DP_OUT"], "rccl_world1.json"), "w") as f:
        json.dump(rec, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
