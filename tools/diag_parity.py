"""Diagnostic: every tensor's error against the fp64 oracle (err / max(1, max|ref|)) for a few
block configurations, without asserting — for reading how an error scales with the batch and
which path (fused / unfused Chebyshev attention) carries it.
usage: python tools/diag_parity.py name:B:flash[:first[:res_kind[:train]]] [...]
       e.g. pems07:2:1 pems07:66:0 t16h3:2:auto:1:0:0"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import test_gpu_parity as T  # noqa: E402


def main():
    for spec in sys.argv[1:]:
        f = spec.split(":")
        name, B, fl = f[:3]
        first = len(f) > 3 and f[3] == "1"
        res_kind = int(f[4]) if len(f) > 4 else None
        train = len(f) > 5 and f[5] == "1"
        flash = None if fl == "auto" else bool(int(fl))
        errs, owns = {}, {}
        T._run_config_vs_oracle(name, first, int(B), flash=flash, tol=1e30, errs=errs, owns=owns, res_kind=res_kind,
                                train=train)
        worst = sorted(errs.items(), key=lambda kv: -kv[1])[:8]
        print(f"{spec}: " + " ".join(f"{k}={v:.2e}(own {owns.get(k, 0):.1e})" for k, v in worst), flush=True)


if __name__ == "__main__":
    main()
