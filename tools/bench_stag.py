#!/usr/bin/env python
"""Timing of the graph builders on the device, beside the
reference algorithm on the host (oracle/stag_ref.py = scipy linprog/HiGHS per pair, the
reference's own solver call).  Prints one JSON line.

  STAG_gen:      GAMBIA shape T=287, F=4; `--pairs` node pairs of a synthetic N-node series
                 (all pairs of the first nodes), timed with HIP events around one launch.
  fast_STAG_gen: N=2139 (GAMBIA) and N=4096 (SYN): distances + top-k.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=287)
    ap.add_argument("--F", type=int, default=4)
    ap.add_argument("--nodes", type=int, default=200)
    ap.add_argument("--cpu-pairs", type=int, default=8)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from dstagnn_drought_amd import fast_stag_gen as fg
    from dstagnn_drought_amd import stag_gen as sg
    from oracle import stag_ref as ref

    dev = torch.device("cuda", 0)
    rs = np.random.RandomState(0)
    data = rs.randn(a.T, a.nodes, a.F)
    nd = sg.NodeData(data, dev)
    iu = torch.triu_indices(a.nodes, a.nodes, 1, device=dev).t().contiguous()
    P = iu.shape[0]
    nd.emd_pairs(iu[:256])  # warm-up (module load, LDS attribute)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out, st, piv = nd.emd_pairs(iu, with_pivots=True)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    piv = piv.cpu().numpy()
    assert int(st.max()) == 0
    # CPU: the reference's solver (linprog/HiGHS with the dense A_eq), 1 thread per pair as its
    # process pool runs it
    idx = iu[: a.cpu_pairs].cpu().numpy()
    t0 = time.time()
    cpu_vals = [ref.process_node_pair(int(i), int(j), data) for i, j in idx]
    cpu_s = (time.time() - t0) / len(idx)
    err = float(np.max(np.abs(np.array(cpu_vals) - out[: a.cpu_pairs].cpu().numpy())))
    res = {
        "stag_gen": {"T": a.T, "F": a.F, "pairs": P, "ms": ms, "pairs_per_s": P / (ms / 1e3),
                     "mean_pivots": float(piv.mean()), "max_pivots": int(piv.max()),
                     "ns_per_pivot_per_pair": ms * 1e6 / max(1, piv.sum()),
                     "cpu_reference_s_per_pair": cpu_s, "cpu_sample_pairs": len(idx), "max_abs_err_vs_cpu": err,
                     "gambia_all_pairs_est_s": 2139 * 2138 / 2 / (P / (ms / 1e3))},
    }
    for N in (2139, 4096):
        feats = torch.randn(N, 12, dtype=torch.float64, device=dev)
        coords = torch.arange(N, dtype=torch.float64, device=dev)[:, None]
        fg.adjacency(fg.distances_device(coords, feats, device=dev), 0.01, dev)
        torch.cuda.synchronize()
        t0 = time.time()
        reps = 5
        for _ in range(reps):
            s = fg.distances_device(coords, feats, device=dev)
            fg.adjacency(s, 0.01, dev)
        torch.cuda.synchronize()
        res[f"fast_stag_N{N}_ms"] = (time.time() - t0) * 1e3 / reps
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
