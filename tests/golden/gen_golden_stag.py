#!/usr/bin/env python
"""Golden vectors for the graph builders (test infrastructure, build container only).

Imports the read-only reference at /root/reference and stores inputs and the outputs the
reference computed on them (no reference source text):
  g7_stag_pairs.npz     data/STAG_gen.py:40-59 process_node_pair (cosine cost, norm
                        marginals, exact EMD by scipy linprog/HiGHS) on 20 pairs at
                        T=12 and 20 at T=48, F=4, with zero rows hitting the 1e-12 guards.
  g7b_stag_dataset.npz  data/STAG_gen.py:61-100 process_dataset on N=6, T=12: the
                        symmetrised sta matrix it saves before its pickling crash (quirk 18).
  g8_fast_stag.npz      data/fast_STAG_gen.py:16-35 calculate_distances on N=40 with the
                        1-D index "coords" the reference builds (quirk 19) and PCA-12-like
                        features, including duplicated rows (exact ties).

data/fast_STAG_gen.py imports numba, which is absent here: a no-op stand-in module
(jit -> identity decorator, prange -> range) is registered in sys.modules first, which
keeps the function's semantics.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_stag.py
"""
import os
import shutil
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def numba_standin():
    m = types.ModuleType("numba")

    def jit(*a, **k):
        if a and callable(a[0]) and not k:
            return a[0]
        return lambda f: f
    m.jit = jit
    m.njit = jit
    m.prange = range
    sys.modules["numba"] = m


def main():
    if not os.path.isdir(REF):
        print("reference absent; skipping")
        return 0
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    numba_standin()
    from data.STAG_gen import process_node_pair, process_dataset
    from data.fast_STAG_gen import calculate_distances

    rs = np.random.RandomState(7)
    out = {}
    for T in (12, 48):
        N, F = 8, 4
        data = rs.randn(T, N, F)
        data[3, 2, :] = 0.0        # zero row -> 1e-12 norm guard
        data[:, 5, :] = 0.0        # all-zero node
        data[:, 6, :] = np.abs(data[:, 6, :])
        pairs, res = [], []
        for i in range(N):
            for j in range(i + 1, N):
                if len(pairs) < 20:
                    pairs.append((i, j))
                    res.append(process_node_pair((i, j, data))[2])
        out[f"data_T{T}"] = data
        out[f"pairs_T{T}"] = np.array(pairs, dtype=np.int64)
        out[f"emd_T{T}"] = np.array(res, dtype=np.float64)
    np.savez(os.path.join(OUT, "g7_stag_pairs.npz"), **out)
    print("wrote g7_stag_pairs.npz", {k: v.shape for k, v in out.items()})

    # process_dataset on a tiny dataset: the .npy is written before the crash (quirk 18)
    tmp = os.path.join(OUT, "_tmp_stag")
    os.makedirs(tmp, exist_ok=True)
    try:
        data = rs.randn(12, 6, 4)
        np.savez(os.path.join(tmp, "TINY.npz"), data=data)
        err = ""
        try:
            process_dataset(os.path.join(tmp, "TINY.npz"), "TINY", sparsity=0.34)
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
        sta = np.load(os.path.join(tmp, "stag_034_TINY.npy"), allow_pickle=False)
        np.savez(os.path.join(OUT, "g7b_stag_dataset.npz"), data=data, sta=sta, error=np.array(err))
        print("wrote g7b_stag_dataset.npz; reference error:", err)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)

    N = 40
    coords = np.arange(N, dtype=np.int64)[:, None]           # np.where(mask) on a 1-D mask
    feats = rs.randn(N, 12)
    feats[7] = feats[3]                                      # exact ties
    feats[20] = 2.5 * feats[11]
    feats[30] = 0.0                                          # zero norm -> 1e-12 guard
    sta = calculate_distances(coords, feats)
    np.savez(os.path.join(OUT, "g8_fast_stag.npz"), coords=coords, feats=feats, sta_upper=sta)
    print("wrote g8_fast_stag.npz", sta.shape, int((sta != 0).sum()))
    return 0


if __name__ == "__main__":
    sys.exit(main())
