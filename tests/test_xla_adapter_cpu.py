"""The torch_xla-API adapter under dstagnn_drought_amd/refpaths (VERDICT r4 item 8;
train_DSTAGNN_my.py:16-18, :25, :33, :113-115, :127, :148-161, :180, :195-197) on CPU: the
reference's import lines resolve, the world-1 calls behave as torch_xla's, xla_device refuses
a machine without a HIP device (no CPU fallback), and xmp.spawn + xm.optimizer_step form the
data-parallel step over gloo (world 2: the reduced gradients are the mean, a master-only xm.save
between steps as the reference does it, an unreduced step refused).  The HIP-device
loop is tests/test_gpu_xla_adapter.py.  Subprocesses keep the top-level names out of the
other tests."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import os, sys, tempfile
import dstagnn_drought_amd.refpaths as r
r.install()
from tensorboardX import SummaryWriter
import torch_xla.core.xla_model as xm
import torch_xla.distributed.parallel_loader as pl
import torch_xla.distributed.xla_multiprocessing as xmp
import torch
assert xm.__file__.startswith(r.PATH), xm.__file__
w = SummaryWriter("runs/x"); w.add_scalar("a", 1.0, 0); w.flush(); w.close()
assert xm.xrt_world_size() == 1 and xm.get_ordinal() == 0 and xm.is_master_ordinal()
xm.master_print("MASTER_PRINT_OK")
try:
    xm.xla_device()
    raise SystemExit("xla_device must raise without a HIP device")
except RuntimeError as e:
    assert "no HIP device" in str(e)
ds = torch.utils.data.TensorDataset(torch.arange(10.).reshape(5, 2), torch.arange(5))
dl = torch.utils.data.DataLoader(ds, batch_size=2)
ml = pl.MpDeviceLoader(dl, torch.device("cpu"))
assert len(ml) == 3 and [b[1].tolist() for b in ml] == [[0, 1], [2, 3], [4]]
lin = torch.nn.Linear(3, 2)
ref = torch.nn.Linear(3, 2); ref.load_state_dict(lin.state_dict())
o1, o2 = torch.optim.Adam(lin.parameters(), lr=0.1), torch.optim.Adam(ref.parameters(), lr=0.1)
for m in (lin, ref):
    m(torch.ones(4, 3)).sum().backward()
xm.optimizer_step(o1, barrier=True)
o2.step()
assert all(torch.equal(a, b) for a, b in zip(lin.parameters(), ref.parameters()))
p = os.path.join(tempfile.mkdtemp(), "e.params")
xm.save(lin.state_dict(), p)
sd = torch.load(p, weights_only=True)
assert set(sd) == {"weight", "bias"}
xm.mark_step(); xm.rendezvous("x")
print("ADAPTER_OK")
'''

SPAWN = r'''
import os, sys, json, tempfile
import dstagnn_drought_amd.refpaths as r
r.install()
import torch
import torch.distributed as dist
import torch_xla.core.xla_model as xm
import torch_xla.distributed.xla_multiprocessing as xmp
OUT = sys.argv[1]

def fn(index, out):
    torch.manual_seed(0)
    lin = torch.nn.Linear(3, 1, bias=False)
    opt = torch.optim.SGD(lin.parameters(), lr=1.0)
    try:  # WORLD_SIZE = 2 without a process group: the all-reduce must not be skipped silently
        xm.optimizer_step(opt)
        raise SystemExit("optimizer_step without a process group must raise")
    except RuntimeError as e:
        assert "not initialised" in str(e), e
    dist.init_process_group("gloo")  # (on a GPU box xm.xla_device() does this on RCCL)
    assert xm.xrt_world_size() == 2 and xm.get_ordinal() == index
    x = torch.full((1, 3), float(index + 1))   # rank 0: ones, rank 1: twos
    deltas = []
    for epoch in range(2):
        opt.zero_grad()
        lin(x).sum().backward()                     # grad = x
        w0 = lin.weight.detach().clone()
        xm.optimizer_step(opt)                      # mean all-reduce + step
        deltas.append((w0 - lin.weight.detach()).tolist())
        if xm.is_master_ordinal():                  # train_DSTAGNN_my.py:173-180: master-only save
            xm.save(lin.state_dict(), os.path.join(out, f"epoch_{epoch}.params"))
    with open(os.path.join(out, f"r{index}.json"), "w") as f:
        json.dump({"grad": lin.weight.grad.tolist(), "delta": deltas}, f)

if __name__ == "__main__":
    xmp.spawn(fn, args=(OUT,), nprocs=2, start_method="fork")
    print("SPAWN_OK")
'''


def _run(code, *args):
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, "-c", code, *args], cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=240)


def test_xla_adapter_world1():
    r = _run(SCRIPT)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "MASTER_PRINT_OK" in r.stdout and "ADAPTER_OK" in r.stdout


def test_xmp_spawn_optimizer_step_means_gradients(tmp_path):
    import json
    r = _run(SPAWN, str(tmp_path))
    assert r.returncode == 0 and "SPAWN_OK" in r.stdout, r.stderr[-3000:]
    recs = [json.loads((tmp_path / f"r{i}.json").read_text()) for i in (0, 1)]
    for rec in recs:  # mean of ones and twos, in both epochs (the master's save between them is no collective)
        assert rec["grad"] == [[1.5, 1.5, 1.5]], rec
        assert all(abs(v - 1.5) < 1e-6 for d in rec["delta"] for v in d[0]) and len(rec["delta"]) == 2, rec
    assert (tmp_path / "epoch_0.params").exists() and (tmp_path / "epoch_1.params").exists()
