"""The C-ABI alone on the GPU (the launchers callable "so C++
unit tests can call it without torch"): tests/native/block_abi_test, a hipcc-built host program
linked only against libdstagnn.so (no torch, no Python in its process), fills
dstagnn_block_dims / params / graph from a reference-written golden, sizes its buffers with
dstagnn_block_sizes, runs dstagnn_block_forward + dstagnn_block_backward on a hipStream_t it
creates, and compares out, re_At, grad_x, grad_res_att and every parameter gradient with the
golden at 1e-4 * max(1, max|ref|).

This test only writes the bundle the program reads (raw arrays from the golden file and the
graph index data the package builds at init, model.support_index / flash_support) and runs the
program as a child process; the comparison happens inside the program."""
import json
import os
import subprocess

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "block_abi_test")


def _write_bundle(golden_dir, name, out_dir):
    import dstagnn_drought_amd as D
    from dstagnn_drought_amd import block_fn as bf
    g = dict(np.load(os.path.join(golden_dir, name), allow_pickle=False))
    m = json.loads(str(g["meta"]))
    cheb = [torch.from_numpy(g[f"cheb_{k}"]) for k in range(m["K"])]
    blk = D.DSTAGNN_block("cpu", m["num_of_d"], m["num_of_d"], m["K"], m["C"], m["C"], 1, cheb, g["adj_pa"],
                          g["adj_tmd"], m["N"], m["T"], m["D"], m["d_k"], m["d_v"], m["n_heads"])
    blk.load_state_dict({k[6:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("param/")})
    blk = blk.cuda().eval()
    B, N, F, T = g["x"].shape
    graph = blk._graph()
    sparse = bf.use_sparse(graph, blk.meta, T)
    flash = bf.use_flash(graph, blk.meta, T, None, B)
    if flash:
        graph = blk._flash_graph(graph)
    man = []

    def put(key, arr):
        a = arr.detach().cpu().numpy() if torch.is_tensor(arr) else np.asarray(arr)
        if a.dtype in (np.float64, np.float32):
            a, dt = np.ascontiguousarray(a, np.float32), "f32"
        else:
            a, dt = np.ascontiguousarray(a, np.int32), "i32"
        a.tofile(os.path.join(out_dir, key + ".bin"))
        man.append(f"{key} {dt} {a.size}")

    names, ps, slots = blk._param_list()
    for n, p, s in zip(names, ps, slots):
        put(f"p{s}", p)
        if "grad/" + n in g:
            put(f"exp_grad_p{s}", g["grad/" + n])
    for k in ["cheb", "adj_pa"] + (["csc_ptr", "csc_row", "csr_ptr", "csr_col"] if sparse else []) + \
             (list(bf.FLASH_KEYS) if flash else []):
        put(k, graph[k])
    put("x", g["x"])
    res_mode = 0
    if "res_att" in g:
        put("res_att", g["res_att"])
        res_mode = 2 if g["res_att"].shape[1] == F else 1
        if "grad_res_att" in g:
            put("exp_grad_res", g["grad_res_att"])
    put("d_out", g["g_out"])
    put("d_re_at", g["g_re"])
    put("exp_out", g["out"])
    put("exp_re_at", g["re_at"])
    put("exp_grad_x", g["grad_x"])
    with open(os.path.join(out_dir, "manifest.txt"), "w") as f:
        f.write("\n".join(man) + "\n")
    with open(os.path.join(out_dir, "dims.txt"), "w") as f:
        f.write(" ".join(str(v) for v in (B, N, F, T, m["n_heads"], m["d_k"], m["d_v"], m["D"], m["K"], m["C"],
                                          res_mode, int(sparse), int(flash))) + "\n")
    return bf.block_paths(blk, torch.from_numpy(g["x"]).cuda(),
                          torch.from_numpy(g["res_att"]).cuda() if "res_att" in g else 0)


@pytest.mark.parametrize("name", ["g13_block_inner_prod.npz", "g14_block_first_prod.npz", "g3_block_inner.npz"])
def test_native_c_abi_block_vs_golden(golden_dir, name, tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    assert os.path.exists(EXE), f"{EXE} not built (make)"
    paths = _write_bundle(golden_dir, name, str(tmp_path))
    r = subprocess.run([EXE, str(tmp_path)], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0 and "ABI_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
    from dstagnn_drought_amd.block_fn import PATH_BITS
    bits = int(r.stdout.split("paths 0x")[1].split()[0], 16)
    assert bits == sum(b for n_, b in PATH_BITS.items() if n_ in paths), (hex(bits), sorted(paths))
    if "_prod" in name:  # the production kernels ran in the C++ process (the path is a function of the dims)
        assert {"flash_small", "cheb_agg", "tat_fused_fwd", "tat_fused_bwd", "gtu_fused_fwd", "gtu_fused_bwd"} <= paths
