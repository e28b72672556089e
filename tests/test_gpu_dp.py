"""The data-parallel overlap on real HIP blocks (dp.py's post-hook path had only
been exercised with CPU tensors built in Python).  Two ranks share the one GPU over gloo
(RCCL refuses two ranks on one device; the driver's 8-GPU scaling bench runs RCCL itself):
each runs a DSTAGNN_block forward + backward in direct-gradient mode with
GradAllReducer.attach, so the all-reduce of the block's flat gradient buffer is issued from
the post-hook on the dstagnn autograd node; then the same step without attach.

Checked: the hook fired with the block's flat buffer (one in-flight reduction after the
backward, none without attach), the reduced gradients equal the non-overlapped path's, and
every rank holds the same mean."""
import json
from pathlib import Path
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(worker, tmp_path, nproc=2):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2", DSTAGNN_DP_OUT=str(tmp_path))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}", "--master-addr",
           "127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "tests", worker)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.gpu
def test_dp_overlap_on_hip_blocks(tmp_path):
    _launch("dp_gpu_worker.py", tmp_path)
    recs = [json.loads((tmp_path / f"rank{r_}.json").read_text()) for r_ in (0, 1)]
    assert sorted(x["rank"] for x in recs) == [0, 1], recs
    for x in recs:
        assert x["flat"], x                         # the backward packed one flat gradient buffer
        assert x["inflight_with_attach"] == 1, x    # ... whose all-reduce the node's post-hook issued
        assert x["inflight_without"] == 0, x
        assert x["same_keys"] and x["ranks_agree"], x
        assert x["max_err"] <= 1e-6, x              # same sums, same order: equal to fp32 rounding


@pytest.mark.gpu
def test_dp_step_equals_one_gpu_step(tmp_path):
    """a world-2 data-parallel step (each rank B/2 samples, HIP blocks, the
    attach() all-reduce, Adam) equals the 1-GPU step on the concatenated batch — eval AND train
    mode: the dropout masks are keyed by the global sample index (rank * B + b), so each rank's
    forward is BIT-identical to its slice of the full-batch forward (split-K off); the mean
    all-reduced gradients equal the full-batch gradients to 1e-5 * max(1, scale) (two fp32
    summation orders of the same sum), the parameters after one Adam step (lr 1e-4) likewise
    wherever |grad| > 1e-3 * max|grad| of the tensor (Adam's normalised first step turns a
    rounding-level gradient's undetermined sign into an O(lr) move; fcmy.0.bias, whose gradient
    cancels exactly to rounding level everywhere, see test_gpu_train.py, is held by the
    gradient check only)."""
    _launch("dp_equiv_worker.py", tmp_path)
    recs = [json.loads((tmp_path / f"equiv_rank{r_}.json").read_text()) for r_ in (0, 1)]
    for rec in recs:
        for mode in ("eval", "train"):
            x = rec[mode]
            assert x["fwd_exact"], (rec["rank"], mode, x)
            assert x["same_grad_keys"], (rec["rank"], mode, x)
            assert abs(x["loss_dp"] - x["loss_ref"]) <= 1e-6 * max(1.0, abs(x["loss_ref"])), (rec["rank"], mode, x)
            assert x["grad_err"] <= 1e-5, (rec["rank"], mode, x)
            assert x["param_err"] <= 1e-5, (rec["rank"], mode, x)
            assert x["param_err2"] <= 1e-5, (rec["rank"], mode, x)  # HipAdam's cached second step
            assert x["optimizer"] == {"dp": "HipAdam", "ref": "HipAdam"}, x


@pytest.mark.gpu
def test_rccl_world1_reducer(tmp_path):
    """RCCL itself (backend "nccl", device_id as bench.py's init_ranks) on the
    one GPU of a lease, world size 1, through bench.py's DP step: the post-hook all-reduce of the
    block's flat gradient buffer on RCCL's stream beside the library's side stream completes,
    the gradients are unchanged bit for bit, and the reducer's per-step cost is recorded
    (tests/rccl_worker.py; the 8-GPU scaling curve is the driver's)."""
    _launch("rccl_worker.py", tmp_path, nproc=1)
    rec = json.loads((tmp_path / "rccl_world1.json").read_text())
    print("rccl world 1:", rec)
    keep = os.environ.get("DSTAGNN_PROFILE_OUT")  # (tools/gpu_check.sh: kept as profiles/<round>_rccl_world1.json)
    if keep:
        os.makedirs(keep, exist_ok=True)
        (Path(keep) / "rccl_world1.json").write_text(json.dumps(rec))
    assert rec["backend"] == "nccl" and rec["world"] == 1, rec
    assert rec["hook_inflight"] == 1, rec   # the node's post-hook issued the async all-reduce
    assert rec["exact"] and rec["collective_ok"], rec
