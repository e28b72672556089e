"""ctypes binding of libdstagnn.so (the C-ABI declared in include/dstagnn.h).

torch is imported first on purpose: PyTorch-ROCm ships its own libamdhip64.so.7,
and loading it before libdstagnn.so makes the dynamic loader resolve our NEEDED
libamdhip64.so.7 to that same runtime (one HIP runtime per process), so torch
device pointers and streams are valid in our kernels.

There is no fallback: if the library is missing or fails to load, every entry
point raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the library load, see module docstring)

MAX_K = 8
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DSTAGNN_LIB", os.path.join(_HERE, "libdstagnn.so"))

RES_NONE, RES_BCAST, RES_FULL = 0, 1, 2

_fp = ctypes.POINTER(ctypes.c_float)
_vp = ctypes.c_void_p


class BlockDims(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int), ("N", ctypes.c_int), ("F", ctypes.c_int), ("T", ctypes.c_int),
                ("n_heads", ctypes.c_int), ("d_k", ctypes.c_int), ("d_v", ctypes.c_int),
                ("d_model", ctypes.c_int), ("K", ctypes.c_int), ("C", ctypes.c_int),
                ("res_mode", ctypes.c_int), ("train", ctypes.c_int), ("drop_p", ctypes.c_float),
                ("seed", ctypes.c_uint64), ("cheb_sparse", ctypes.c_int)]


# field order == struct dstagnn_block_params / dstagnn_block_grads
PARAM_FIELDS = ["pre_conv_w", "pre_conv_b", "embT_pos", "embT_g", "embT_b", "embS_pos", "embS_g", "embS_b",
                "tat_wq", "tat_wk", "tat_wv", "tat_fc", "tat_ln_g", "tat_ln_b", "sat_wq", "sat_wk",
                ("theta", MAX_K), ("mask", MAX_K), ("gtu_w", 3), ("gtu_b", 3), "res_w", "res_b",
                "fcmy_w", "fcmy_b", "ln_g", "ln_b"]


def _mk_struct(name):
    fields = []
    for f in PARAM_FIELDS:
        if isinstance(f, tuple):
            fields.append((f[0], _vp * f[1]))
        else:
            fields.append((f, _vp))
    return type(name, (ctypes.Structure,), {"_fields_": fields})


BlockParams = _mk_struct("BlockParams")
BlockGrads = _mk_struct("BlockGrads")


class Graph(ctypes.Structure):
    _fields_ = [("cheb", _vp), ("adj_pa", _vp), ("nnz", ctypes.c_int), ("csc_ptr", _vp), ("csc_row", _vp),
                ("csr_ptr", _vp), ("csr_col", _vp)]


class Idx(ctypes.Structure):
    _fields_ = [("div", ctypes.c_int64), ("s0", ctypes.c_int64), ("s1", ctypes.c_int64)]


class GemmDesc(ctypes.Structure):
    _fields_ = [("M", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int), ("batch", ctypes.c_int),
                ("A", _vp), ("a_m", Idx), ("a_k", Idx), ("a_z", Idx), ("a_off", ctypes.c_int64),
                ("B", _vp), ("b_k", Idx), ("b_n", Idx), ("b_z", Idx), ("b_off", ctypes.c_int64),
                ("C", _vp), ("c_m", Idx), ("c_n", Idx), ("c_z", Idx), ("c_off", ctypes.c_int64),
                ("alpha", ctypes.c_float), ("beta", ctypes.c_float),
                ("bias", _vp), ("bias_stride", ctypes.c_int64), ("relu", ctypes.c_int)]


_lib = None
_load_error = None


def load():
    """Load (once) and return the ctypes handle; raise loudly if it is unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"dstagnn_drought_amd: HIP library not built ({LIB_PATH} missing); "
                           "run `make` or __graft_entry__.build(). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    sig = {
        "dstagnn_block_sizes": [P(BlockDims), P(ctypes.c_size_t), P(ctypes.c_size_t)],
        "dstagnn_block_forward": [P(BlockDims), P(BlockParams), P(Graph), _vp, _vp, _vp, _vp,
                                  _vp, ctypes.c_size_t, _vp, ctypes.c_size_t, _vp],
        "dstagnn_block_backward": [P(BlockDims), P(BlockParams), P(Graph), _vp, _vp, _vp, _vp, _vp, _vp,
                                   P(BlockGrads), _vp, ctypes.c_size_t, _vp, ctypes.c_size_t, _vp],
        "dstagnn_cheb_sat_forward": [ctypes.c_int] * 7 + [_vp] * 4 + [P(Graph)] + [_vp] * 5
                                    + [ctypes.c_size_t, _vp],
        "dstagnn_cheb_sat_backward": [ctypes.c_int] * 7 + [_vp] * 2 + [P(Graph)] + [_vp] * 10
                                     + [ctypes.c_size_t, _vp],
        "dstagnn_gemm_f32": [P(GemmDesc), _vp, ctypes.c_size_t, _vp],
        "dstagnn_block_time_stage": [P(BlockDims), P(BlockParams), P(Graph), _vp, _vp, _vp, _vp,
                                     _vp, ctypes.c_size_t, _vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                     P(ctypes.c_float), _vp],
        "dstagnn_dropout_mask": [P(BlockDims), ctypes.c_int, _vp, _vp],
        "dstagnn_stag_prep": [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, _vp],
        "dstagnn_stag_emd_pairs": [_vp, _vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, ctypes.c_int64,
                                   _vp, _vp, _vp, _vp],
        "dstagnn_emd_dense": [_vp, _vp, _vp, ctypes.c_int, ctypes.c_int64, _vp, _vp, _vp],
        "dstagnn_fast_stag_distances": [_vp, ctypes.c_int, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_double, _vp, _vp],
        "dstagnn_graph_topk": [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, _vp],
        "dstagnn_stag_emd_lds_bytes": [ctypes.c_int, ctypes.c_int],
        "dstagnn_head_scratch_bytes": [],
        "dstagnn_head_forward": [ctypes.c_int] * 7 + [_vp] * 8 + [ctypes.c_size_t, _vp],
        "dstagnn_head_backward": [ctypes.c_int] * 7 + [_vp] * 12 + [ctypes.c_size_t, _vp],
        "dstagnn_last_error": [],
        "dstagnn_version": [],
    }
    for name, args in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    lib.dstagnn_last_error.restype = ctypes.c_char_p
    lib.dstagnn_stag_emd_lds_bytes.restype = ctypes.c_int64
    lib.dstagnn_head_scratch_bytes.restype = ctypes.c_int64
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load().dstagnn_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def idx(div=0, s0=0, s1=0):
    return Idx(int(div), int(s0), int(s1))
