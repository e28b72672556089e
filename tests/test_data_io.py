"""Data / graph I/O against files the reference itself produced
(tests/golden/gen_golden_data.py runs prepareData.py and the lib/ loaders)."""
import os

import numpy as np
import pytest
import torch

from dstagnn_drought_amd import data as D


def _g(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name), allow_pickle=False))


@pytest.mark.parametrize("name", ["g10_prepare_a.npz", "g10_prepare_b.npz", "g10_prepare_c.npz"])
def test_read_and_generate_dataset_matches_reference(golden_dir, tmp_path, name):
    g = _g(golden_dir, name)
    T, N, F, h, d, w, pph, nfp = (int(v) for v in g["meta"])
    npz = tmp_path / "SYN.npz"
    np.savez(npz, data=g["data"])
    all_data = D.read_and_generate_dataset(str(npz), w, d, h, nfp, points_per_hour=pph, save=True)
    saved = dict(np.load(str(tmp_path / f"SYN_r{h}_d{d}_w{w}_dstagnn.npz")))
    assert sorted(saved) == sorted(k[4:] for k in g if k.startswith("out_"))
    for k, v in saved.items():
        ref = g["out_" + k]
        assert v.dtype == ref.dtype and v.shape == ref.shape, k
        np.testing.assert_array_equal(v, ref, err_msg=k)  # bit-identical
    np.testing.assert_array_equal(all_data["train"]["x"], g["out_train_x"])
    np.testing.assert_array_equal(all_data["stats"]["_std"], g["out_std"])


def test_sample_indices_agree_with_vectorised_windows(golden_dir):
    g = _g(golden_dir, "g10_prepare_b.npz")
    T, N, F, h, d, w, pph, nfp = (int(v) for v in g["meta"])
    data = g["data"]
    idx = int(g["out_train_timestamp"][3, 0])
    ws, ds, hs, tgt = D.get_sample_indices(data, w, d, h, idx, nfp, pph)
    assert ws is None and ds.shape == (d * nfp, N, F) and hs.shape == (h * nfp, N, F)
    x = np.concatenate([ds, hs], 0).transpose(1, 2, 0)  # (N, F, Tin) before normalisation
    mean, std = g["out_mean"][0], g["out_std"][0]
    np.testing.assert_allclose((x - mean) / std, g["out_train_x"][3], rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(tgt[..., -1].T, g["out_train_target"][3])
    assert D.search_data(T, 1, T - nfp + 1, nfp, 1, pph) is None      # target runs past the end
    assert D.search_data(T, 2, 12, nfp, 1, 12) is None                 # window before t = 0
    with pytest.raises(ValueError):
        D.search_data(T, 1, 100, nfp, 1, -1)


def test_too_short_series_raises(tmp_path):
    np.savez(tmp_path / "S.npz", data=np.zeros((20, 3, 1)))
    with pytest.raises(ValueError):
        D.read_and_generate_dataset(str(tmp_path / "S.npz"), 0, 0, 1, 12, points_per_hour=12)


def test_graph_loaders_match_reference(golden_dir, tmp_path):
    g = _g(golden_dir, "g11_graph_io.npz")
    N = int(g["N"])
    files = {}
    for k in ("dense_txt", "edge_txt", "id_txt", "edge_id_txt"):
        p = tmp_path / k
        p.write_text(str(g[k]))
        files[k] = str(p)
    for fn, key in ((lambda: D.load_weighted_adjacency_matrix(files["dense_txt"], N), "wam"),
                    (lambda: D.load_weighted_adjacency_matrix2(files["dense_txt"], N), "wam2"),
                    (lambda: D.load_PA(files["dense_txt"]), "pa"),
                    (lambda: D.get_adjacency_matrix2(files["edge_txt"], N), "adj2"),
                    (lambda: D.get_adjacency_matrix2(files["edge_id_txt"], N, id_filename=files["id_txt"]),
                     "adj2_id")):
        got = fn()
        assert got.dtype == g[key].dtype, key
        np.testing.assert_array_equal(got, g[key], err_msg=key)
    assert int(g["adj2_distance_raises"]) == 1
    with pytest.raises(ValueError):
        D.get_adjacency_matrix2(files["edge_txt"], N, type_="distance")


def test_masked_mape_matches_reference(golden_dir):
    g = _g(golden_dir, "g11_graph_io.npz")
    assert D.masked_mape_np(g["mape_true"], g["mape_pred"], 0) == pytest.approx(float(g["mape_0"]), rel=0, abs=0)
    with np.errstate(all="ignore"):
        assert D.masked_mape_np(np.nan_to_num(g["mape_true"]), g["mape_pred"]) == pytest.approx(
            float(g["mape_nan"]), rel=1e-12, nan_ok=True)


def test_load_graphdata_channel1(golden_dir, tmp_path):
    g = _g(golden_dir, "g10_prepare_a.npz")
    stem = tmp_path / "SYN"
    np.savez(str(stem) + "_r1_d0_w0_dstagnn.npz", **{k[4:]: v for k, v in g.items() if k.startswith("out_")})
    (tx, tl, tt, vx, vl, vt, sx, sl, st, mean, std) = D.load_graphdata_channel1(str(stem) + ".npz", 1, 0, 0, "cpu", 16)
    assert tx.dtype == torch.float32 and tuple(tx.shape) == g["out_train_x"].shape
    np.testing.assert_array_equal(vx.numpy(), g["out_val_x"].astype(np.float32))
    assert len(tl) == -(-tx.shape[0] // 16) and len(vl) == -(-vx.shape[0] // 16)
    xb, yb = next(iter(sl))  # test loader: not shuffled
    np.testing.assert_array_equal(xb.numpy(), g["out_test_x"][:16].astype(np.float32))
    np.testing.assert_array_equal(mean, g["out_mean"])
    # DistributedSampler-style sharding: each rank sees a disjoint part of the training set
    from torch.utils.data.distributed import DistributedSampler
    seen = []
    for rank in range(2):
        out = D.load_graphdata_channel1(str(stem) + ".npz", 1, 0, 0, "cpu", 8,
                                        sampler=lambda ds, r=rank: DistributedSampler(ds, 2, r, shuffle=False))
        seen.append(torch.cat([b[0] for b in out[1]]))
    assert seen[0].shape[0] + seen[1].shape[0] == tx.shape[0]


def test_prepare_cli(golden_dir, tmp_path):
    g = _g(golden_dir, "g10_prepare_b.npz")
    T, N, F, h, d, w, pph, nfp = (int(v) for v in g["meta"])
    np.savez(tmp_path / "SYN.npz", data=g["data"])
    conf = tmp_path / "c.conf"
    conf.write_text(f"[Data]\ngraph_signal_matrix_filename = {tmp_path}/SYN.npz\npoints_per_hour = {pph}\n"
                    f"num_for_predict = {nfp}\n[Training]\nnum_of_weeks = {w}\nnum_of_days = {d}\n"
                    f"num_of_hours = {h}\n")
    D.main(["--config", str(conf)])
    out = dict(np.load(tmp_path / f"SYN_r{h}_d{d}_w{w}_dstagnn.npz"))
    np.testing.assert_array_equal(out["test_x"], g["out_test_x"])
