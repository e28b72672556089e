"""bench.py --gpus N self-launch: run without a launcher it starts N
ranks through torch.distributed.run; every rank joins one process group and rank 0 prints
one JSON line with n_gpus = N.  Exercised here over gloo on CPU (--launch-probe does only
the launcher + one collective, no GPU work)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = dict(os.environ, DSTAGNN_DIST_BACKEND="gloo", **env)
    e.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=240)


def test_self_launch_two_ranks():
    r = _run(["--gpus", "2", "--launch-probe"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["ranks_seen"] == 2 and rec["rank_sum"] == 1


def test_world_size_mismatch_fails_loudly():
    e = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--launch-probe"], cwd=ROOT,
                       env=e, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
