"""STAG_gen graph builder on MI355X: exact earth mover's distance between every node pair.

Mirrors data/STAG_gen.py (same function names, arguments and outputs):

  validate_path(path)                          :12-15
  wasserstein_distance(p, q, D)                :17-38   exact LP optimum, 1.0 on failure
  process_node_pair((i, j, data)) -> (i,j,d)   :40-59
  process_dataset(data_path, dataset_name, period=12, sparsity=0.01) -> (sta, A_adj)   :61-137

The reference solves one dense 2T x T^2 linprog/HiGHS LP per pair on a process pool
(~1.0 s/pair at T=287: 3.3 days for GAMBIA's 2.29 M pairs on 8 cores) and then crashes while
pickling a local function before it writes the CSVs.  Here:
  * dstagnn_stag_prep      per-node unit rows + marginals, once per node (not per pair);
  * dstagnn_stag_emd_pairs one wavefront per pair runs a network simplex with its whole
                           workspace in LDS, costs recomputed from the unit rows (no D, no A_eq);
  * dstagnn_graph_topk     the adjacency step (:103-116) as a per-row sort in LDS;
and the CSVs are written (the reference's intended output).  Results equal the LP optimum to
~1e-12 (pinned against scipy linprog and the reference's golden vectors); pairs whose LP the
reference's solver reports infeasible (marginal totals differing by > 1e-7, e.g. all-zero
nodes) get the reference's 1.0.  There is no CPU fallback: the HIP library must load.
"""
import os
import time

import numpy as np
import torch

from . import _lib


def validate_path(path):
    if not os.path.exists(path):
        raise FileNotFoundError(f"Input file not found: {path}")
    return path


def _dev(device):
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError("the graph builders run on the HIP device only (no CPU fallback)")
    return device


def _raise_status(status, what):
    bad = int((status >= 2).sum())
    if bad:
        raise RuntimeError(f"{what}: solver pivot cap hit on {bad} pair(s)")


def wasserstein_distance(p, q, D, device=None):
    """Exact min <D, P> s.t. P1 = p, P^T1 = q, P >= 0 (data/STAG_gen.py:17-38).
    p, q (T,) and D (T, T) -> float; or batched p, q (B, T), D (B, T, T) -> (B,) array.
    Infeasible problems (negative mass, totals differing by > 1e-7) return 1.0 like the
    reference's failure path."""
    dev = _dev(device)
    p = torch.as_tensor(np.asarray(p, dtype=np.float64) if not torch.is_tensor(p) else p, dtype=torch.float64)
    q = torch.as_tensor(np.asarray(q, dtype=np.float64) if not torch.is_tensor(q) else q, dtype=torch.float64)
    D = torch.as_tensor(np.asarray(D, dtype=np.float64) if not torch.is_tensor(D) else D, dtype=torch.float64)
    single = p.dim() == 1
    if single:
        p, q, D = p[None], q[None], D.reshape(1, p.shape[-1], p.shape[-1])
    B, T = p.shape
    if q.shape != (B, T) or D.numel() != B * T * T:
        raise ValueError("wasserstein_distance: p, q must be (B,T) and D (B,T,T)")
    p, q = p.to(dev).contiguous(), q.to(dev).contiguous()
    D = D.reshape(B, T, T).to(dev).contiguous()
    out, st = _lib.load().emd_dense(p, q, D)
    _raise_status(st.cpu().numpy(), "wasserstein_distance")
    r = out.cpu().numpy()
    return float(r[0]) if single else r


class NodeData:
    """Device-resident per-node prep of a (T, N, F) series: unit rows xhat (N,T,F), marginals
    p (N,T) and their totals (N) — data/STAG_gen.py:47-54 hoisted out of the pair loop."""

    def __init__(self, data, device=None):
        dev = _dev(device)
        d = data if torch.is_tensor(data) else torch.from_numpy(np.ascontiguousarray(data, dtype=np.float64))
        d = d.to(device=dev, dtype=torch.float64).contiguous()
        if d.dim() != 3:
            raise ValueError("data must be (T, N, F)")
        self.T, self.N, self.F = (int(s) for s in d.shape)
        self.device = dev
        self.xhat, self.p, self.psum = _lib.load().stag_prep(d)

    def emd_pairs(self, pairs, with_pivots=False):
        """EMD of node pairs (P, 2) int (numpy or tensor) -> device fp64 (P,), status (P,)."""
        pr = pairs if torch.is_tensor(pairs) else torch.from_numpy(np.asarray(pairs, dtype=np.int64))
        pr = pr.to(device=self.device, dtype=torch.int32).reshape(-1, 2).contiguous()
        if pr.numel() and (int(pr.min()) < 0 or int(pr.max()) >= self.N):
            raise IndexError("node pair index out of range")
        out, st, piv = _lib.load().stag_emd_pairs(self.xhat, self.p, self.psum, pr, bool(with_pivots))
        return (out, st, piv) if with_pivots else (out, st)


def process_node_pair(args, device=None):
    """(i, j, data) -> (i, j, emd) exactly as data/STAG_gen.py:40-59 (data (T, N, F))."""
    i, j, data = args
    nd = NodeData(np.asarray(data)[:, [i, j], :], device)
    out, st = nd.emd_pairs(np.array([[0, 1]]))
    _raise_status(st.cpu().numpy(), "process_node_pair")
    return (i, j, float(out.cpu()[0]))


def sta_matrix(data, device=None, chunk=1 << 20, progress=None):
    """All pairs i<j, symmetrised (data/STAG_gen.py:77-97) -> (N, N) fp64 numpy."""
    nd = data if isinstance(data, NodeData) else NodeData(data, device)
    N = nd.N
    iu = torch.triu_indices(N, N, 1, device=nd.device)
    P = iu.shape[1]
    vals = torch.empty(P, dtype=torch.float64, device=nd.device)
    for s in range(0, P, chunk):
        e = min(P, s + chunk)
        out, st = nd.emd_pairs(iu[:, s:e].t())
        _raise_status(st.cpu().numpy(), "sta_matrix")
        vals[s:e] = out
        if progress:
            progress(e, P)
    sta = torch.zeros(N, N, dtype=torch.float64, device=nd.device)
    sta[iu[0], iu[1]] = vals
    sta = sta + sta.t()
    return sta.cpu().numpy()


def adjacency(sta, sparsity, device=None):
    """data/STAG_gen.py:103-116: adj = 1 - sta + I; per row the `top` smallest adj entries
    (top = max(1, int(N * sparsity))) -> A_adj = 1, R_adj = adj there.  Ties: lower index."""
    dev = _dev(device)
    s = torch.as_tensor(np.ascontiguousarray(sta, dtype=np.float64)).to(dev)
    return _topk(s, max(1, int(s.shape[0] * sparsity)), 1)


def _topk(s, k, mode):
    A, R, nbr = _lib.load().graph_topk(s.contiguous(), int(k), int(mode))
    return A.cpu().numpy(), R.cpu().numpy(), nbr.cpu().numpy()


def process_dataset(data_path, dataset_name, period=12, sparsity=0.01, device=None):
    """data/STAG_gen.py:61-137: writes stag_{sss}_{name}.npy (symmetric sta), and — where the
    reference crashes first (quirk 18) — stag_{sss}_{name}.csv (A_adj) and strg_{sss}_{name}.csv
    (R_adj).  `period` is accepted and unused, as in the reference.  Returns (sta, A_adj)."""
    import pandas as pd
    data_path = validate_path(data_path)
    dir_path = os.path.dirname(data_path)
    with np.load(data_path) as f:
        data = f["data"]
    t0 = time.time()
    sta = sta_matrix(data, device)
    tag = f"{int(sparsity * 100):03d}"
    np.save(os.path.join(dir_path, f"stag_{tag}_{dataset_name}.npy"), sta)
    A, R, _ = adjacency(sta, sparsity, device)
    pd.DataFrame(A).to_csv(os.path.join(dir_path, f"stag_{tag}_{dataset_name}.csv"), header=False, index=False)
    pd.DataFrame(R).to_csv(os.path.join(dir_path, f"strg_{tag}_{dataset_name}.csv"), header=False, index=False)
    print(f"STAG graph for {dataset_name}: N={sta.shape[0]}, {time.time() - t0:.1f} s")
    return sta, A
