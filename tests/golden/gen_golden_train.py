#!/usr/bin/env python
"""Golden trajectory of the reference TRAINING SCRIPT, made by running
/root/reference/train_DSTAGNN_my.py itself (test infrastructure, build container only).

The script imports torch_xla and tensorboardX, absent here.  It is run unmodified under
minimal single-process stand-ins for exactly the calls it makes (xla_device -> cpu,
optimizer_step -> optimizer.step(), MpDeviceLoader -> the loader, save -> torch.save,
is_master_ordinal -> True, ...), written to a temporary directory on PYTHONPATH.
Dropout is forced to p=0 (torch.nn.Dropout patched in the launcher) so the trajectory is
deterministic and comparable across implementations; everything else — the double
optimizer step per batch (quirk 14), the DataLoader shuffles, SmoothL1, Adam, the
best-val checkpoints, the final test loss — is the script's own.

Writes tests/golden/g12_train.npz: the synthetic inputs (series, graph CSV texts, config
text), the epochs the script checkpointed, each checkpoint's state_dict, and the
validation / test losses it printed (4 decimals).
Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_train.py
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

STUBS = {
    "torch_xla/__init__.py": "",
    "torch_xla/core/__init__.py": "",
    "torch_xla/core/xla_model.py": (
        "import torch\n"
        "def xla_device(): return torch.device('cpu')\n"
        "def xrt_world_size(): return 1\n"
        "def is_master_ordinal(): return True\n"
        "def optimizer_step(optimizer, barrier=False, optimizer_args={}):\n"
        "    return optimizer.step(**optimizer_args)\n"
        "def master_print(*a, **k): print(*a, **k)\n"
        "def get_memory_info(device): return {}\n"
        "def save(obj, path): torch.save(obj, path)\n"),
    "torch_xla/distributed/__init__.py": "",
    "torch_xla/distributed/parallel_loader.py": "def MpDeviceLoader(loader, device): return loader\n",
    "tensorboardX/__init__.py": "class SummaryWriter:\n    def __init__(self, *a, **k): pass\n"
                                "    def add_scalar(self, *a, **k): pass\n",
}

LAUNCHER = """import runpy, sys, torch
_init = torch.nn.Dropout.__init__
def _nodrop(self, p=0.5, inplace=False):
    _init(self, 0.0, inplace)
torch.nn.Dropout.__init__ = _nodrop
sys.argv = ['train_DSTAGNN_my.py', '--config', sys.argv[1]]
sys.path.insert(0, {ref!r})
runpy.run_path({script!r}, run_name='__main__')
"""

CONF = """[Data]
adj_filename = {td}/adj.csv
graph_signal_matrix_filename = {td}/SYN.npz
stag_filename = {td}/stag.csv
strg_filename = {td}/strg.csv
num_of_vertices = {N}
period = 12
points_per_hour = 12
num_for_predict = 12
len_input = 12
dataset_name = SYN

[Training]
ctx = 0
in_channels = 1
nb_block = 2
n_heads = 2
K = 3
d_k = 8
d_model = 16
nb_chev_filter = 8
nb_time_filter = 8
batch_size = 8
graph = AG
model_name = dstagnn
dataset_name = SYN
num_of_weeks = 0
num_of_days = 0
num_of_hours = 1
start_epoch = 0
epochs = 4
learning_rate = 0.001
"""

PREP_CONF = """[Data]
adj_filename = unused
graph_signal_matrix_filename = {td}/SYN.npz
stag_filename = unused
strg_filename = unused
num_of_vertices = {N}
points_per_hour = 12
num_for_predict = 12
len_input = 12
dataset_name = SYN

[Training]
num_of_weeks = 0
num_of_days = 0
num_of_hours = 1
"""


def dense_csv(a):
    return "\n".join(",".join(repr(float(v)) for v in row) for row in a) + "\n"


def main():
    if not os.path.isdir(REF):
        print("reference absent: nothing to do")
        return
    N, T = 10, 100
    rs = np.random.RandomState(7)
    t = np.arange(T)
    series = (np.sin(t[:, None] / 6.0 + rs.rand(N)[None, :] * 6) * 2 + rs.randn(T, N) * 0.3)[:, :, None]
    tmd = np.eye(N)
    pa = np.zeros((N, N))
    for i in range(N):
        tmd[i, rs.choice([j for j in range(N) if j != i], 2, replace=False)] = rs.rand(2) + 0.1
        pa[i, rs.choice(N, 3, replace=False)] = 1.0
    adj = (rs.rand(N, N) < 0.3).astype(float)
    texts = {"adj.csv": dense_csv(adj), "stag.csv": dense_csv(tmd), "strg.csv": dense_csv(pa)}
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    with tempfile.TemporaryDirectory() as td:
        for k, v in texts.items():
            with open(os.path.join(td, k), "w") as f:
                f.write(v)
        np.savez(os.path.join(td, "SYN.npz"), data=series)
        with open(os.path.join(td, "prep.conf"), "w") as f:
            f.write(PREP_CONF.format(td=td, N=N))
        subprocess.run([sys.executable, os.path.join(REF, "prepareData.py"), "--config", os.path.join(td, "prep.conf")],
                       check=True, env=env, cwd=td, stdout=subprocess.DEVNULL)
        stubdir = os.path.join(td, "stubs")
        for rel, src in STUBS.items():
            p = os.path.join(stubdir, rel)
            os.makedirs(os.path.dirname(p), exist_ok=True)
            with open(p, "w") as f:
                f.write(src)
        conf_text = CONF.format(td="@DIR@", N=N)
        with open(os.path.join(td, "train.conf"), "w") as f:
            f.write(conf_text.replace("@DIR@", td))
        with open(os.path.join(td, "launch.py"), "w") as f:
            f.write(LAUNCHER.format(ref=REF, script=os.path.join(REF, "train_DSTAGNN_my.py")))
        env["PYTHONPATH"] = stubdir
        r = subprocess.run([sys.executable, os.path.join(td, "launch.py"), os.path.join(td, "train.conf")], env=env,
                           cwd=td, capture_output=True, text=True)
        if r.returncode != 0:
            print(r.stdout[-3000:], r.stderr[-3000:])
            raise SystemExit("reference training script failed")
        val = [float(m.group(2)) for m in re.finditer(r"Epoch (\d+) Val Loss: ([0-9.]+)", r.stdout)]
        test = float(re.search(r"Final Test Loss: ([0-9.]+)", r.stdout).group(1))
        import torch
        ckpts = sorted(glob.glob(os.path.join(td, "myexperiments", "SYN", "*", "epoch_*.params")))
        saved = sorted(int(re.search(r"epoch_(\d+)\.params", p).group(1)) for p in ckpts)
        out = {"series": series, "config_text": np.array(conf_text), "val_losses": np.array(val),
               "test_loss": np.array(test), "saved_epochs": np.array(saved),
               "folder": np.array(os.path.basename(os.path.dirname(ckpts[0])))}
        out.update({f"{k}_text": np.array(v) for k, v in texts.items()})
        for e in saved:
            sd = torch.load(os.path.join(os.path.dirname(ckpts[0]), f"epoch_{e}.params"), weights_only=True)
            for k, v in sd.items():
                out[f"ep{e}/{k}"] = v.numpy()
    np.savez_compressed(os.path.join(OUT, "g12_train.npz"), **out)
    print("g12_train.npz: val", val, "test", test, "saved", saved)


if __name__ == "__main__":
    main()
