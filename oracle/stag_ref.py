"""CPU oracle for the two graph builders (TEST INFRASTRUCTURE ONLY: imported by tests/,
never by the product path).  numpy/scipy restatements, each citing the reference lines it
follows.  Pinned by tests/golden/g7_stag_pairs.npz, g7b_stag_dataset.npz and
g8_fast_stag.npz (generated from the reference by tests/golden/gen_golden_stag.py).

STAG_gen (data/STAG_gen.py, exact earth mover's distance between per-timestep norm
distributions of two nodes) and fast_STAG_gen (data/fast_STAG_gen.py, windowed cosine
distance on PCA features + top-k adjacency).
"""
import numpy as np


# ------------------------------------------------------------------------------------
# STAG_gen
# ------------------------------------------------------------------------------------
def pair_problem(x, y):
    """Marginals and cost of one node pair (data/STAG_gen.py:40-57).
    x, y: (T, F) series of the two nodes.  Returns p (T), q (T), D (T, T)."""
    x_norm = np.linalg.norm(x, axis=1, keepdims=True)
    y_norm = np.linalg.norm(y, axis=1, keepdims=True)
    x_norm[x_norm == 0] = 1e-12
    y_norm[y_norm == 0] = 1e-12
    p = x_norm[:, 0] / (x_norm.sum() + 1e-12)
    q = y_norm[:, 0] / (y_norm.sum() + 1e-12)
    with np.errstate(divide="ignore", invalid="ignore"):
        D = 1 - np.dot(x / x_norm, (y / y_norm).T)
    D = np.nan_to_num(D, nan=1.0)
    D = np.clip(D, 0, 1)
    return p, q, D


def emd_linprog(p, q, D):
    """Exact transport cost by scipy linprog(method='highs') with the dense row/column
    equality constraints (data/STAG_gen.py:17-38); 1.0 when the solver fails."""
    from scipy.optimize import linprog
    try:
        n = len(p)
        A_eq = np.zeros((2 * n, n * n))
        for i in range(n):
            A_eq[i, i * n:(i + 1) * n] = 1
        for j in range(n):
            A_eq[n + j, j::n] = 1
        b_eq = np.concatenate([p, q])
        c = np.nan_to_num(D.reshape(-1), nan=0.0, posinf=1e12, neginf=-1e12)
        r = linprog(c, A_eq=A_eq, b_eq=b_eq, method="highs")
        return r.fun if r.success else 1.0
    except Exception:  # noqa: BLE001
        return 1.0


def process_node_pair(i, j, data):
    """data/STAG_gen.py:40-59; data (T, N, F)."""
    p, q, D = pair_problem(data[:, i, :], data[:, j, :])
    return emd_linprog(p, q, D)


def sta_matrix(data):
    """All pairs i<j, symmetrised (data/STAG_gen.py:78-99)."""
    n = data.shape[1]
    sta = np.zeros((n, n))
    for i in range(n):
        for j in range(i + 1, n):
            sta[i, j] = process_node_pair(i, j, data)
    return sta + sta.T


def stag_adjacency(sta, sparsity):
    """data/STAG_gen.py:103-122 (which the reference never reaches: quirk 18): adj = 1 - sta
    + I, per row the `top` smallest entries (argsort ascending) -> A = 1, R = adj value."""
    n = sta.shape[0]
    adj = 1 - sta + np.identity(n)
    top = max(1, int(n * sparsity))
    A = np.zeros_like(adj)
    R = np.zeros_like(adj)
    for i in range(n):
        nb = np.argsort(adj[i, :], kind="stable")[:top]
        A[i, nb] = 1
        R[i, nb] = adj[i, nb]
    return A, R


# ------------------------------------------------------------------------------------
# fast_STAG_gen
# ------------------------------------------------------------------------------------
def calculate_distances(coords, feats, max_distance=10.0):
    """data/fast_STAG_gen.py:16-35: for i<j within max_distance (Euclidean on `coords`),
    1 - x.y / ((|x| + 1e-12)(|y| + 1e-12)); upper triangle only, zeros elsewhere."""
    n = coords.shape[0]
    sta = np.zeros((n, n))
    for i in range(n):
        for j in range(i + 1, n):
            if np.sqrt(np.sum((coords[i] - coords[j]) ** 2)) <= max_distance:
                x, y = feats[i], feats[j]
                nx = np.sqrt(np.sum(x ** 2)) + 1e-12
                ny = np.sqrt(np.sum(y ** 2)) + 1e-12
                sta[i, j] = 1 - np.dot(x, y) / (nx * ny)
    return sta


def fast_stag_graph(coords, feats, sparsity=0.01, max_distance=10.0):
    """data/fast_STAG_gen.py:55-74: symmetrise, zero diagonal, k = max(1, int(N*sparsity))
    smallest per row (ties by index here: the reference's quicksort leaves their order
    unspecified, quirk 19) -> A = 1, R = 1 - sta."""
    sta = calculate_distances(coords, feats, max_distance)
    sta = sta + sta.T
    np.fill_diagonal(sta, 0)
    n = sta.shape[0]
    k = max(1, int(n * sparsity))
    A = np.zeros_like(sta)
    R = np.zeros_like(sta)
    for i in range(n):
        nb = np.argsort(sta[i], kind="stable")[:k]
        A[i, nb] = 1
        R[i, nb] = 1 - sta[i, nb]
    return sta, A, R
