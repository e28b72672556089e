"""Loader of the PyTorch-ROCm operator library (_C.so: TORCH_LIBRARY(dstagnn, ...),
csrc/torch_ops.cpp) over the C-ABI library libdstagnn.so (include/dstagnn.h).

torch is imported first: PyTorch-ROCm ships its own libamdhip64.so, and loading it before
our libraries makes the dynamic loader resolve their NEEDED libamdhip64 to that same
runtime (one HIP runtime per process), so torch device pointers and streams are valid in
our kernels.  After load(), every operator is ``torch.ops.dstagnn.<name>``.

There is no fallback: if the library is missing or fails to load, load() raises.
"""
import os

import torch

MAX_K = 8
_HERE = os.path.dirname(os.path.abspath(__file__))
EXT_PATH = os.environ.get("DSTAGNN_EXT", os.path.join(_HERE, "_C.so"))
LIB_PATH = os.path.join(_HERE, "libdstagnn.so")

RES_NONE, RES_BCAST, RES_FULL = 0, 1, 2
# dstagnn::block flags
F_TRAIN, F_SPARSE, F_DIRECT, F_POISON, F_FLASH = 1, 2, 4, 8, 16

_ops = None


def load():
    """Load (once) the operator library and return the ``torch.ops.dstagnn`` namespace."""
    global _ops
    if _ops is not None:
        return _ops
    if not os.path.exists(EXT_PATH) or not os.path.exists(LIB_PATH):
        raise RuntimeError(f"dstagnn_drought_amd: HIP libraries not built ({EXT_PATH} / {LIB_PATH}); "
                           "run `make` or __graft_entry__.build(). There is no CPU fallback.")
    torch.ops.load_library(EXT_PATH)
    _ops = torch.ops.dstagnn
    return _ops


def build_stamp():
    """Identity of the native build in this tree: sha256 (first 16 hex digits) of
    libdstagnn.so and of _C.so.  Profiles under profiles/ record the stamp of the build they
    measured; bench.py marks a profile whose stamp differs from its own library as stale."""
    import hashlib

    def sha(path):
        h = hashlib.sha256()
        with open(path, "rb") as f:
            for chunk in iter(lambda: f.read(1 << 20), b""):
                h.update(chunk)
        return h.hexdigest()[:16]
    return {"lib_sha256": sha(LIB_PATH), "ext_sha256": sha(EXT_PATH)}


def gemm_maps(*maps):
    """Flatten 9 (div, s0, s1) index maps (a_m a_k a_z b_k b_n b_z c_m c_n c_z) for
    dstagnn::gemm_f32; a missing map is (0, 0, 0)."""
    out = []
    for m in maps:
        m = tuple(m) + (0,) * (3 - len(m))
        out.extend(int(v) for v in m)
    return out
