"""CPU: the graph-builder oracle (oracle/stag_ref.py) against the reference's golden vectors."""
import os

import numpy as np

from oracle import stag_ref as ref


def load(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name), allow_pickle=False))


def test_stag_pairs_golden(golden_dir):
    g = load(golden_dir, "g7_stag_pairs.npz")
    for T in (12, 48):
        data, pairs, emd = g[f"data_T{T}"], g[f"pairs_T{T}"], g[f"emd_T{T}"]
        got = np.array([ref.process_node_pair(int(i), int(j), data) for i, j in pairs])
        np.testing.assert_allclose(got, emd, rtol=0, atol=1e-9)


def test_stag_dataset_golden(golden_dir):
    g = load(golden_dir, "g7b_stag_dataset.npz")
    np.testing.assert_allclose(ref.sta_matrix(g["data"]), g["sta"], rtol=0, atol=1e-9)
    assert "pickle" in str(g["error"])  # quirk 18: the reference crashes before the CSVs


def test_fast_stag_golden(golden_dir):
    g = load(golden_dir, "g8_fast_stag.npz")
    sta = ref.calculate_distances(g["coords"], g["feats"])
    np.testing.assert_allclose(sta, g["sta_upper"], rtol=0, atol=1e-14)
