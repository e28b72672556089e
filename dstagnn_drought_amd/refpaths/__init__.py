"""The reference's own import paths, as thin re-exports of dstagnn_drought_amd.

Put this directory on sys.path (``PYTHONPATH=$(python -c 'import dstagnn_drought_amd.refpaths as r;
print(r.PATH)')``, or ``dstagnn_drought_amd.refpaths.install()``) and the reference's unmodified
imports resolve to the MI355X build:

    from model.DSTAGNN_my import make_model                          # train_DSTAGNN_my.py:13
    from lib.dataloader import load_weighted_adjacency_matrix, ...   # train_DSTAGNN_my.py:14
    from lib.utils1 import load_graphdata_channel1, ...              # train_DSTAGNN_my.py:15

Nothing here computes; every name is the package's own object.
"""
import os
import sys

PATH = os.path.dirname(os.path.abspath(__file__))


def install():
    """Prepend this directory to sys.path (idempotent) so `model` / `lib` resolve here."""
    if PATH not in sys.path:
        sys.path.insert(0, PATH)
    return PATH
