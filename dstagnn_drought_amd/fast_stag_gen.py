"""fast_STAG_gen graph builder on MI355X (mirrors data/fast_STAG_gen.py).

  euclidean_distance(a, b)                                   :11-14
  calculate_distances(coords, data_reduced, max_distance=10) :16-35  (upper triangle, as the reference)
  pca_reduce(data, n_components=12)                          :42-45
  process_dataset(data_path, dataset_name, sparsity=0.01)    :37-86

Device work: dstagnn_fast_stag_distances (windowed cosine distance, fp64, written symmetric
with a zero diagonal — the reference's :57-59) and dstagnn_graph_topk (per-row k smallest,
:66-74).  PCA is a library SVD (torch.linalg on the device, rocSOLVER) of the centred
(N, T*F) matrix: exact, where the reference's sklearn PCA picks its randomized solver for
this shape with random_state=None (not reproducible run to run); cosine distances do not
depend on the components' signs.

Reference quirks kept: the "coords" are node indices from a 1-D mask, so
the window is |i - j| <= 10; pairs outside the window keep distance 0 and are picked first by
the top-k.  Not kept: the hard-coded 2139 (N comes from the data).  Ties in the top-k go to
the lower index (the reference's quicksort order is unspecified).
"""
import os
import time

import numpy as np
import torch

from . import _lib
from .stag_gen import _dev, _topk


def euclidean_distance(a, b):
    return np.sqrt(np.sum((np.asarray(a) - np.asarray(b)) ** 2))


def distances_device(coords, feats, max_distance=10.0, device=None):
    """Symmetric (N, N) fp64 device tensor: 1 - x.y / ((|x| + 1e-12)(|y| + 1e-12)) for
    pairs within `max_distance`, 0 elsewhere and on the diagonal."""
    dev = _dev(device)
    c = torch.as_tensor(np.asarray(coords, dtype=np.float64) if not torch.is_tensor(coords) else coords,
                        dtype=torch.float64).to(dev)
    f = torch.as_tensor(np.asarray(feats, dtype=np.float64) if not torch.is_tensor(feats) else feats,
                        dtype=torch.float64).to(dev)
    if c.dim() == 1:
        c = c[:, None]
    c, f = c.contiguous(), f.contiguous()
    if f.shape[0] != c.shape[0]:
        raise ValueError("coords and features disagree on the node count")
    return _lib.load().fast_stag_distances(c, f, float(max_distance))


def calculate_distances(coords, data_reduced, max_distance=10.0, device=None):
    """data/fast_STAG_gen.py:16-35: the upper triangle (i < j) only, zeros elsewhere."""
    sta = distances_device(coords, data_reduced, max_distance, device)
    return torch.triu(sta, 1).cpu().numpy()


def pca_reduce(data, n_components=12, device=None):
    """(T, N, F) -> (N, n_components) principal-component scores of the (N, T*F) node matrix."""
    dev = _dev(device)
    d = torch.as_tensor(np.asarray(data, dtype=np.float64) if not torch.is_tensor(data) else data,
                        dtype=torch.float64).to(dev)
    T, N, F = d.shape
    X = d.permute(1, 0, 2).reshape(N, T * F)
    if not bool(torch.isfinite(X).all()):
        raise ValueError("Input X contains NaN or infinity.")  # sklearn's validation error
    Xc = X - X.mean(dim=0, keepdim=True)
    U, S, _ = torch.linalg.svd(Xc, full_matrices=False)
    return (U[:, :n_components] * S[:n_components]).contiguous()


def adjacency(sta, sparsity, device=None):
    """data/fast_STAG_gen.py:66-74: k = max(1, int(N * sparsity)) smallest per row ->
    A_adj = 1, R_adj = 1 - sta there.  Returns (A, R, neighbours)."""
    dev = _dev(device)
    s = sta if torch.is_tensor(sta) else torch.as_tensor(np.ascontiguousarray(sta, dtype=np.float64))
    s = s.to(device=dev, dtype=torch.float64).contiguous()
    return _topk(s, max(1, int(s.shape[0] * sparsity)), 0)


def process_dataset(data_path, dataset_name, sparsity=0.01, device=None):
    """data/fast_STAG_gen.py:37-86: writes stag_001_{name}.npy (sta), stag_001_{name}.csv
    (A_adj) and strg_001_{name}.csv (R_adj) next to the input (the reference's fixed 001
    tag).  Returns (sta, A_adj, R_adj)."""
    import pandas as pd
    with np.load(data_path) as f:
        data = f["data"]
    t0 = time.time()
    feats = pca_reduce(data, 12, device)
    valid = ~np.isnan(data[0, :, 0])
    coords = np.array(np.where(valid)).T
    sta_d = distances_device(coords, feats, 10.0, device)
    A, R, _ = adjacency(sta_d, sparsity, device)
    sta = sta_d.cpu().numpy()
    out = os.path.dirname(data_path)
    np.save(os.path.join(out, f"stag_001_{dataset_name}.npy"), sta)
    pd.DataFrame(A).to_csv(os.path.join(out, f"stag_001_{dataset_name}.csv"), header=False, index=False)
    pd.DataFrame(R).to_csv(os.path.join(out, f"strg_001_{dataset_name}.csv"), header=False, index=False)
    print(f"fast STAG graph for {dataset_name}: N={sta.shape[0]}, {time.time() - t0:.2f} s")
    return sta, A, R
