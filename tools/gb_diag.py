"""Per-output relative errors of one block config against the fp64 oracle, every key (no stop at
the first failure: run under `python -O`).  usage: python -O tools/gb_diag.py [config] [B] [first]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_parity as T  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "pems08"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
first = len(sys.argv) > 3 and sys.argv[3] == "1"
errs, owns = {}, {}
T._run_config_vs_oracle(cfg, first, B, errs=errs, owns=owns)
for k in errs:
    print(f"{k:40s} err/scale {errs[k]:.3e}  fp32-ref own {owns.get(k, 0):.3e}")
