"""The reference's own import paths, as thin re-exports of dstagnn_drought_amd.

Put this directory on sys.path (``PYTHONPATH=$(python -c 'import dstagnn_drought_amd.refpaths as r;
print(r.PATH)')``, or ``dstagnn_drought_amd.refpaths.install()``) and the reference's unmodified
imports resolve to the MI355X build:

    from model.DSTAGNN_my import make_model                          # train_DSTAGNN_my.py:13
    from lib.dataloader import load_weighted_adjacency_matrix, ...   # train_DSTAGNN_my.py:14
    from lib.utils1 import load_graphdata_channel1, ...              # train_DSTAGNN_my.py:15
    from tensorboardX import SummaryWriter                           # train_DSTAGNN_my.py:16 (no-op)
    import torch_xla.core.xla_model as xm                            # train_DSTAGNN_my.py:17
    import torch_xla.distributed.parallel_loader as pl               # train_DSTAGNN_my.py:18
    import torch_xla.distributed.xla_multiprocessing as xmp          # train_DSTAGNN_my.py:196

(the torch_xla adapter maps the device, the optimiser step's all-reduce, the loaders and the
process spawn onto the HIP device and torch.distributed / RCCL: torch_xla/__init__.py).

Nothing here computes; every model / data name is the package's own object.
"""
import os
import sys

PATH = os.path.dirname(os.path.abspath(__file__))


def install():
    """Prepend this directory to sys.path (idempotent) so `model` / `lib` resolve here."""
    if PATH not in sys.path:
        sys.path.insert(0, PATH)
    return PATH
