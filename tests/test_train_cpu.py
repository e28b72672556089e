"""Training-driver logic (dstagnn_drought_amd.train) on CPU with a small
stand-in model: the compute path is the HIP library (GPU tests), the loop is model-agnostic.

* the epoch order equals iterating the reference's shuffled DataLoader;
* fit() == a direct statement of train_DSTAGNN_my.py:141-159 (double optimizer step,
  zero_grad after the first step, SmoothL1, Adam) on the same data;
* world_size 2 over gloo: sharded data + gradient all-reduce == one process on the
  union batch (weak-scaling DP), same checkpoints and validation losses.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from dstagnn_drought_amd import train as TR


class Tiny(nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = nn.Linear(12, 12)
        self.unused = nn.Linear(2, 2)  # grad stays None, like the inner blocks' EmbedT (quirk 11)

    def forward(self, x):                # (B, N, 1, T) -> (B, N, T)
        return self.lin(x[:, :, 0, :])


def _data(n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, 5, 1, 12, generator=g), torch.randn(n, 5, 12, generator=g)


def _reference_loop(net, x, y, vx, vy, epochs, bs, lr):
    """train_DSTAGNN_my.py:141-172 restated with torch's own DataLoader (single process)."""
    crit = nn.SmoothL1Loss()
    opt = torch.optim.Adam(net.parameters(), lr=lr)
    tl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(x, y), batch_size=bs, shuffle=True)
    vl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(vx, vy), batch_size=bs, shuffle=False)
    vals = []
    for _ in range(epochs):
        net.train()
        for xb, yb in tl:
            opt.step()          # xm.optimizer_step(optimizer, barrier=True)  (:148)
            opt.zero_grad()
            loss = crit(net(xb), yb)
            loss.backward()
            opt.step()          # xm.optimizer_step(optimizer)  (:158)
        net.eval()
        with torch.no_grad():
            vals.append(sum(crit(net(a), b).item() for a, b in vl) / len(vl))
    return vals


def test_epoch_order_matches_dataloader():
    x, y = _data(37, 0)
    torch.manual_seed(11)
    ref = [int(i) for _, b in torch.utils.data.DataLoader(
        torch.utils.data.TensorDataset(x, torch.arange(37)), batch_size=5, shuffle=True) for i in b]
    torch.manual_seed(11)
    got = TR.DeviceBatches(x, torch.arange(37), 5, True)
    assert [int(i) for _, b in got for i in b] == ref


def test_fit_matches_reference_loop(tmp_path):
    x, y = _data(40, 1)
    vx, vy = _data(13, 2)
    torch.manual_seed(3)
    a = Tiny()
    b = Tiny()
    b.load_state_dict(a.state_dict())
    torch.manual_seed(5)
    vals_ref = _reference_loop(a, x, y, vx, vy, 3, 8, 1e-2)
    torch.manual_seed(5)
    best, best_val, hist = TR.fit(b, x, y, vx, vy, epochs=3, batch_size=8, lr=1e-2, params_path=str(tmp_path),
                                  log=lambda *_: None)
    assert [h["val_loss"] for h in hist] == pytest.approx(vals_ref, rel=1e-6)
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        assert torch.allclose(p, q, atol=1e-6), n
    assert b.unused.weight.grad is None
    assert best == min(range(3), key=lambda e: vals_ref[e])
    sd = torch.load(os.path.join(tmp_path, f"epoch_{best}.params"), weights_only=True)
    assert set(sd) == set(b.state_dict())


def test_single_step_mode_differs():
    x, y = _data(16, 1)
    vx, vy = _data(8, 2)
    torch.manual_seed(3)
    a = Tiny()
    b = Tiny()
    b.load_state_dict(a.state_dict())
    torch.manual_seed(5)
    TR.fit(a, x, y, vx, vy, epochs=1, batch_size=8, lr=1e-2, params_path=_tmp(), log=lambda *_: None)
    torch.manual_seed(5)
    TR.fit(b, x, y, vx, vy, epochs=1, batch_size=8, lr=1e-2, params_path=_tmp(), log=lambda *_: None,
           double_step=False)
    assert not torch.allclose(a.lin.weight, b.lin.weight)


def _tmp():
    import tempfile
    return tempfile.mkdtemp()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, bs, q, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        x, y = _data(32, 1)
        vx, vy = _data(12, 2)
        torch.manual_seed(3)
        net = Tiny()
        torch.manual_seed(5)
        best, bv, hist = TR.fit(net, x, y, vx, vy, epochs=2, batch_size=bs, lr=1e-2, params_path=outdir,
                                log=lambda *_: None)
        final = {k: v.numpy().copy() for k, v in net.state_dict().items()}
        # the best checkpoint: rank 0 reads the file, rank 1 gets it by broadcast
        if rank == 1:
            with torch.no_grad():
                for p in net.parameters():
                    p.zero_()
        TR.load_best(net, os.path.join(outdir, f"epoch_{best}.params"))
        loaded = {k: v.numpy().copy() for k, v in net.state_dict().items()}
        q.put((rank, final, [h["val_loss"] for h in hist], best, loaded))
    finally:
        dist.destroy_process_group()


def test_dp_world2_equals_single_process(tmp_path):
    """world 2 x batch 4 (rank r: permutation positions r, r+2, ...) == world 1 x batch 8."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 4, q, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x, y = _data(32, 1)
    vx, vy = _data(12, 2)
    torch.manual_seed(3)
    net = Tiny()
    torch.manual_seed(5)
    best, bv, hist = TR.fit(net, x, y, vx, vy, epochs=2, batch_size=8, lr=1e-2, params_path=_tmp(),
                            log=lambda *_: None)
    for rank, sd, vals, b, loaded in res:
        for k, v in net.state_dict().items():
            assert torch.allclose(torch.from_numpy(sd[k]), v, atol=2e-6), (rank, k)
        assert b == best
        ck = torch.load(os.path.join(str(tmp_path), f"epoch_{b}.params"), weights_only=True)
        for k, v in ck.items():
            assert torch.equal(torch.from_numpy(loaded[k]), v), (rank, k)
    # validation batches are split over the ranks and reduced: both ranks report the same
    # mean (batch size 4 there vs 8 here, so only the two ranks are compared)
    assert res[0][2] == pytest.approx(res[1][2], rel=1e-12)


def test_hip_adam_state_dict_round_trips_torch_format():
    """HipAdam keeps ``step`` as an int (its by-step grouping keys on the value); a
    torch.optim.Adam state_dict (tensor steps) loads as ints, and HipAdam's own state_dict has
    torch's tensor steps without touching the live state."""
    p = [nn.Parameter(torch.randn(3, 2)), nn.Parameter(torch.randn(4))]
    ref = torch.optim.Adam(p, lr=1e-3)
    for q in p:
        q.grad = torch.ones_like(q)
    ref.step()
    ref.step()
    ha = TR.HipAdam(p, lr=1e-3)  # (CPU parameters: state handling only, no step here)
    ha.load_state_dict(ref.state_dict())
    steps = [ha.state[q]["step"] for q in p]
    assert steps == [2, 2] and all(type(s) is int for s in steps)
    sd = ha.state_dict()
    assert all(torch.is_tensor(s["step"]) and float(s["step"]) == 2.0 for s in sd["state"].values())
    assert all(type(ha.state[q]["step"]) is int for q in p)  # the live state keeps ints
    ref2 = torch.optim.Adam(p, lr=1e-3)
    ref2.load_state_dict(sd)  # and torch takes it back
    assert all(float(ref2.state[q]["step"]) == 2.0 for q in p)


def test_shard_batch_sets_true_sample_base():
    """a short last shard keys its dropout masks from its true global offset."""
    from dstagnn_drought_amd.dp import shard_batch, shard_start

    from dstagnn_drought_amd import model as M
    blk = M.DSTAGNN_block.__new__(M.DSTAGNN_block)
    nn.Module.__init__(blk)
    blk.sample_base = None
    t = torch.arange(5)
    assert [shard_start(5, r, 2) for r in range(2)] == [0, 3]
    part = shard_batch(t, 1, 2, model=blk)
    assert part.tolist() == [3, 4] and blk.sample_base == 3
    assert shard_batch(t, 0, 2, model=blk).tolist() == [0, 1, 2] and blk.sample_base == 0


def test_sharded_scope_restores_default_sample_base():
    """dp.sharded sets the shard's base for the block only and restores the previous
    base (None: the default rank * B) on exit, exceptions included."""
    from dstagnn_drought_amd.dp import sharded

    from dstagnn_drought_amd import model as M
    blk = M.DSTAGNN_block.__new__(M.DSTAGNN_block)
    nn.Module.__init__(blk)
    blk.sample_base = None
    t = torch.arange(5)
    with sharded(t, 1, 2, blk) as part:
        assert part.tolist() == [3, 4] and blk.sample_base == 3
    assert blk.sample_base is None
    blk.sample_base = 7
    try:
        with sharded(t, 0, 2, blk):
            assert blk.sample_base == 0
            raise KeyError("x")
    except KeyError:
        pass
    assert blk.sample_base == 7
