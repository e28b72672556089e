"""Init-time graph preprocessing and graph-file loaders (host side, numpy/scipy).

Same API and semantics as the reference's lib/utils.py and lib/dataloader.py,
which make_model and the training script call:

  scaled_Laplacian(W)         lib/utils.py:149-177   (tensor in -> float32 tensor out, quirk 5)
  cheb_polynomial(L, K)       lib/utils.py:180-203   (ELEMENTWISE recurrence, quirk 4)
  load_weighted_adjacency_matrix / load_PA / load_weighted_adjacency_matrix2
                              lib/dataloader.py:5-23 (CSV -> binary (N,N))
  get_adjacency_matrix2       lib/utils1.py:92-145   (edge list -> connectivity)

These run once when a model is built; they are not part of the hot path.
"""
import numpy as np
import torch


def scaled_Laplacian(W):
    """L~ = 2 (D - W) / lambda_max - I with lambda_max = Re(largest-real-part eigenvalue)."""
    from scipy.sparse.linalg import eigs
    as_tensor = torch.is_tensor(W)
    Wn = W.detach().cpu().numpy() if as_tensor else np.asarray(W)
    if Wn.ndim != 2 or Wn.shape[0] != Wn.shape[1]:
        raise AssertionError("adjacency must be square")
    Lap = np.diag(Wn.sum(axis=1)) - Wn
    lam = eigs(Lap, k=1, which="LR")[0].real
    Lt = (2.0 * Lap) / lam - np.eye(Wn.shape[0])
    if as_tensor:
        return torch.from_numpy(Lt).float().to(W.device)
    return Lt


def cheb_polynomial(L_tilde, K):
    """[T_0 .. T_{K-1}] with T_0 = I, T_1 = L~, T_k = 2 L~ * T_{k-1} - T_{k-2} (elementwise, as
    the reference; list length is max(K, 2) like the reference)."""
    L = np.asarray(L_tilde)
    polys = [np.eye(L.shape[0]), L.copy()]
    for _ in range(2, K):
        polys.append(2 * L * polys[-1] - polys[-2])
    return polys


# graph-file loaders live with the rest of the data I/O (data.py); re-exported here
from .data import (get_adjacency_matrix2, load_PA, load_weighted_adjacency_matrix,  # noqa: E402,F401
                   load_weighted_adjacency_matrix2)
