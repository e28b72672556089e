"""CPU: the C-ABI library loads and exports every symbol include/dstagnn.h declares; the
PyTorch-ROCm operator library registers every dstagnn:: op; the Python surface mirrors the
reference (state_dict keys, make_model init RNG order, error behaviour)."""
import ctypes
import json
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    with open(os.path.join(ROOT, "include", "dstagnn.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(dstagnn_\w+)\s*\(", src, re.M)))


class BlockDims(ctypes.Structure):  # struct dstagnn_block_dims (include/dstagnn.h)
    _fields_ = [(n, ctypes.c_int) for n in ("B", "N", "F", "T", "n_heads", "d_k", "d_v", "d_model", "K", "C",
                                            "res_mode", "train")] + \
        [("drop_p", ctypes.c_float), ("seed", ctypes.c_uint64), ("cheb_sparse", ctypes.c_int),
         ("cheb_flash", ctypes.c_int), ("cheb_nnz", ctypes.c_int), ("cheb_apa_nnz", ctypes.c_int),
         ("sample_base", ctypes.c_int64)]


def c_abi():
    from dstagnn_drought_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.dstagnn_last_error.restype = ctypes.c_char_p
    return lib


def test_library_exports_header_symbols():
    lib = c_abi()
    names = header_functions()
    assert len(names) >= 9, names
    for n in names:
        assert hasattr(lib, n), f"libdstagnn.so does not export {n}"
    assert lib.dstagnn_version() >= 1


OPS = ["block", "block_fwd", "block_bwd", "block_time_stage", "dropout_masks", "cheb_sat_fwd", "cheb_sat_bwd",
       "gemm_f32", "head_fwd", "head_bwd", "stag_prep", "stag_emd_pairs", "stag_emd_lds_bytes", "emd_dense",
       "fast_stag_distances", "graph_topk", "version", "block_cheb_out", "block_relu_out", "prof_start", "prof_stop",
       "set_splitk_target", "set_gemm_bf16"]


def test_torch_ops_registered():
    from dstagnn_drought_amd import _lib
    ops = _lib.load()
    for n in OPS:
        assert hasattr(ops, n), f"torch.ops.dstagnn.{n} missing"
    assert ops.version() >= 1
    assert ops.stag_emd_lds_bytes(287, 4) > 0
    # the autograd op refuses CPU tensors loudly (no CPU path)
    with pytest.raises(RuntimeError):
        ops.block(torch.zeros(1, 4, 1, 12), None, [], [], [torch.zeros(3, 4, 4), torch.zeros(4, 4)],
                  [3, 8, 8, 16, 3, 8], 0.05, 0, 0)


def test_block_sizes_and_shape_errors():
    lib = c_abi()
    d = BlockDims(32, 170, 32, 12, 3, 32, 32, 512, 3, 32, 1, 1, 0.05, 0)
    sv, sc = ctypes.c_size_t(0), ctypes.c_size_t(0)
    assert lib.dstagnn_block_sizes(ctypes.byref(d), ctypes.byref(sv), ctypes.byref(sc)) == 0
    assert sv.value > 32 * 3 * 170 * 170 * 4 * 2  # P and W
    bad = BlockDims(1, 16, 4, 12, 2, 8, 8, 16, 2, 8, 0, 0, 0.05, 0)  # GAMBIA in_channels=4 (quirk 8)
    rc = lib.dstagnn_block_sizes(ctypes.byref(bad), ctypes.byref(sv), ctypes.byref(sc))
    assert rc == 10001
    assert b"must match" in lib.dstagnn_last_error()
    neg = BlockDims(32, 170, 32, 12, 3, 32, 32, 512, 3, 32, 1, 1, 0.05, 0)
    neg.sample_base = -1
    assert lib.dstagnn_block_sizes(ctypes.byref(neg), ctypes.byref(sv), ctypes.byref(sc)) == 10002


def test_block_pickles_without_host_caches():
    """the module's host-side caches (a torch.classes BlockPlan, which has no
    pickler, and Parameter identities) stay out of pickled / deep-copied state; a copy rebuilds
    them on its first call."""
    import copy
    import io
    import dstagnn_drought_amd as D
    N, T, K = 10, 12, 3
    adj = np.eye(N) + np.roll(np.eye(N), 1, 1)
    cheb = [torch.from_numpy(c).float() for c in D.cheb_polynomial(D.scaled_Laplacian(adj), K)]
    blk = D.DSTAGNN_block("cpu", 1, 1, K, 8, 8, 1, cheb, adj, adj, N, T, 16, 8, 8, 2)
    blk.__dict__["_pcache"] = {"plan": [None, lambda: None]}  # unpicklable, like a BlockPlan
    blk._param_list()
    buf = io.BytesIO()
    torch.save(blk, buf)
    buf.seek(0)
    back = torch.load(buf, weights_only=False)  # our own freshly written object
    assert "_pcache" not in back.__dict__ and "_plist" not in back.__dict__
    assert back.sample_base is None
    dup = copy.deepcopy(blk)
    assert "_pcache" not in dup.__dict__
    assert sorted(dup.state_dict()) == sorted(blk.state_dict())
    assert "_pcache" in blk.__dict__  # the original keeps its caches


def _golden_model(golden_dir):
    import dstagnn_drought_amd as D
    g = np.load(os.path.join(golden_dir, "g4_model.npz"))
    m = json.loads(str(g["meta"]))
    torch.manual_seed(m["seed"])
    model = D.make_model("cpu", 1, m["nb_block"], 1, m["K"], m["C"], m["C"], 1, torch.FloatTensor(g["adj_tmd"]),
                         torch.FloatTensor(g["adj_pa"]), torch.FloatTensor(g["adj_tmd"]), m["num_for_predict"],
                         m["T"], m["N"], m["D"], m["d_k"], m["d_k"], m["n_heads"])
    return g, m, model


def test_state_dict_and_init_match_reference(golden_dir):
    g, m, model = _golden_model(golden_dir)
    sd = model.state_dict()
    ref_keys = [k[6:] for k in g.files if k.startswith("param/")]
    assert list(sd.keys()) == ref_keys  # same names, same registration order
    for k in ref_keys:  # identical RNG-driven init (quirk 9)
        np.testing.assert_array_equal(sd[k].numpy(), g["param/" + k])
    cheb = model.BlockList[0].cheb_conv_SAt.cheb_polynomials
    for k in range(m["K"]):
        np.testing.assert_allclose(cheb[k].numpy(), g[f"cheb_{k}"], rtol=1e-6, atol=1e-6)


def test_cpu_forward_fails_loudly(golden_dir):
    g, m, model = _golden_model(golden_dir)
    with pytest.raises(RuntimeError, match="HIP"):
        model(torch.from_numpy(g["x"]))


def test_gambia_in_channels_4_raises(golden_dir):
    import dstagnn_drought_amd as D
    g = np.load(os.path.join(golden_dir, "g4_model.npz"))
    with open(os.path.join(golden_dir, "g9_gambia_error.json")) as f:
        ref_err = json.load(f)
    torch.manual_seed(1)
    m4 = D.make_model("cpu", 4, 2, 4, 2, 8, 8, 1, torch.FloatTensor(g["adj_tmd"]), torch.FloatTensor(g["adj_pa"]),
                      torch.FloatTensor(g["adj_tmd"]), 12, 12, 16, 16, 8, 8, 2)
    with pytest.raises(RuntimeError) as ei:
        m4(torch.randn(1, 16, 4, 12))
    assert ref_err["type"] == "RuntimeError"
    assert str(ei.value) == ref_err["message"]


def test_graph_helpers_match_reference(golden_dir):
    import dstagnn_drought_amd as D
    g = np.load(os.path.join(golden_dir, "g6_laplacian_pems04.npz"))
    Lt = D.scaled_Laplacian(torch.from_numpy(g["adj_tmd"]))
    assert Lt.dtype == torch.float32
    np.testing.assert_allclose(Lt.numpy(), g["L_tilde"], rtol=1e-4, atol=1e-5)  # ARPACK random v0: ~1e-5 run-to-run
    polys = D.cheb_polynomial(Lt.numpy(), 3)
    for k in range(3):
        np.testing.assert_allclose(polys[k].astype(np.float32), g[f"cheb_{k}"], rtol=1e-4, atol=1e-5)
