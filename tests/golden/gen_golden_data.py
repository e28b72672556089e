#!/usr/bin/env python
"""Golden fixtures for the data / graph I/O row, made by RUNNING the
reference (test infrastructure, build container only; skips when /root/reference is absent).

  g10_prepare_{a,b}.npz  prepareData.py run as a subprocess on a synthetic series with a
                         temporary config (its CLI runs at import): the input series and
                         the ``*_dstagnn.npz`` the reference wrote (prepareData.py:63-147).
  g11_graph_io.npz       lib/dataloader.py loaders and lib/utils1.get_adjacency_matrix2 on
                         small synthetic CSVs (stored as text in the fixture) + masked_mape_np.

Only inputs and the reference's outputs are stored, never its source.
Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_data.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

CONF = """[Data]
adj_filename = unused.csv
graph_signal_matrix_filename = {npz}
stag_filename = unused.csv
strg_filename = unused.csv
num_of_vertices = {N}
points_per_hour = {pph}
num_for_predict = {nfp}
len_input = {lin}
dataset_name = SYN

[Training]
num_of_weeks = {w}
num_of_days = {d}
num_of_hours = {h}
"""


def prepare_case(name, T, N, F, dtype, h, d, w, pph, nfp, seed):
    rs = np.random.RandomState(seed)
    data = (rs.randn(T, N, F) * 3 + 1).astype(dtype)
    with tempfile.TemporaryDirectory() as td:
        npz = os.path.join(td, "SYN.npz")
        np.savez(npz, data=data)
        conf = os.path.join(td, "syn.conf")
        with open(conf, "w") as f:
            f.write(CONF.format(npz=npz, N=N, pph=pph, nfp=nfp, lin=(h + d + w) * nfp, w=w, d=d, h=h))
        env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
        subprocess.run([sys.executable, os.path.join(REF, "prepareData.py"), "--config", conf], check=True, env=env,
                       cwd=td, stdout=subprocess.DEVNULL)
        got = dict(np.load(os.path.join(td, f"SYN_r{h}_d{d}_w{w}_dstagnn.npz")))
    meta = np.array([T, N, F, h, d, w, pph, nfp])
    np.savez_compressed(os.path.join(OUT, name), data=data, meta=meta, **{"out_" + k: v for k, v in got.items()})
    print(name, {k: v.shape for k, v in got.items()})


def graph_io_case():
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    from lib.dataloader import load_weighted_adjacency_matrix, load_weighted_adjacency_matrix2, load_PA
    from lib.utils1 import get_adjacency_matrix2
    from lib.metrics import masked_mape_np
    rs = np.random.RandomState(3)
    N = 12
    dense = np.where(rs.rand(N, N) < 0.25, rs.rand(N, N) * 5, 0.0)
    dense[rs.rand(N, N) < 0.05] = -1.0  # negative entries count as absent
    np.fill_diagonal(dense, 1.0)
    dense_txt = "\n".join(",".join(repr(float(v)) for v in row) for row in dense) + "\n"
    edges = [(int(i), int(j), float(rs.rand() * 100)) for i, j in zip(rs.randint(0, N, 30), rs.randint(0, N, 30))]
    edge_txt = "from,to,cost\n" + "".join(f"{i},{j},{c}\n" for i, j, c in edges) + "7,8\n"  # a short row is skipped
    ids = rs.permutation(np.arange(100, 100 + N))
    id_txt = "\n".join(str(int(i)) for i in ids) + "\n"
    edge_id_txt = "from,to,cost\n" + "".join(f"{ids[i]},{ids[j]},{c}\n" for i, j, c in edges)
    out = {"dense_txt": np.array(dense_txt), "edge_txt": np.array(edge_txt), "id_txt": np.array(id_txt),
           "edge_id_txt": np.array(edge_id_txt), "N": np.array(N)}
    with tempfile.TemporaryDirectory() as td:
        def w(name, txt):
            p = os.path.join(td, name)
            with open(p, "w") as f:
                f.write(txt)
            return p
        pd_ = w("dense.csv", dense_txt)
        pe = w("edges.csv", edge_txt)
        pi = w("ids.txt", id_txt)
        pei = w("edges_id.csv", edge_id_txt)
        out["wam"] = load_weighted_adjacency_matrix(pd_, N)
        out["wam2"] = load_weighted_adjacency_matrix2(pd_, N)
        out["pa"] = load_PA(pd_)
        out["adj2"] = get_adjacency_matrix2(pe, N)
        out["adj2_id"] = get_adjacency_matrix2(pei, N, id_filename=pi)
        try:
            get_adjacency_matrix2(pe, N, type_="distance")
            out["adj2_distance_raises"] = np.array(0)
        except ValueError:
            out["adj2_distance_raises"] = np.array(1)
    yt = rs.rand(6, 7).astype(np.float32) * 10
    yt[0, :3] = 0.0
    yt[2, 4] = np.nan
    yp = yt + rs.randn(6, 7).astype(np.float32)
    out["mape_true"], out["mape_pred"] = yt, yp
    out["mape_0"] = np.array(masked_mape_np(yt, yp, 0))
    out["mape_nan"] = np.array(masked_mape_np(np.nan_to_num(yt), yp))
    np.savez_compressed(os.path.join(OUT, "g11_graph_io.npz"), **out)
    print("g11_graph_io.npz", sorted(out))


def main():
    if not os.path.isdir(REF):
        print("reference absent: nothing to do")
        return
    prepare_case("g10_prepare_a.npz", 120, 7, 3, np.float64, 1, 0, 0, 12, 12, 0)   # PEMS-style (r1_d0_w0)
    prepare_case("g10_prepare_b.npz", 330, 5, 2, np.float32, 2, 1, 0, 12, 12, 1)  # hours + days windows
    prepare_case("g10_prepare_c.npz", 60, 4, 4, np.float64, 3, 0, 0, 2, 4, 2)     # pph*units < nfp (overlap)
    graph_io_case()


if __name__ == "__main__":
    main()
