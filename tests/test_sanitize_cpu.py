"""CPU: the host-compilable native code under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY §5).  The network-simplex EMD solver (csrc/emd_simplex.hpp, the code
the stag.hip kernel runs) is built for the host with -fsanitize=address,undefined and driven
over random cosine / dense problems (tests/native/emd_sanitize_main.cpp); any sanitizer report
or a wrong / non-terminating solve fails the test.  The GPU code itself cannot be sanitized on
this pool (no GPU ASan / XNACK)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_emd_solver_asan_ubsan(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "emd_sanitize"
    src = [os.path.join(ROOT, "tests", "native", "emd_host.cpp"), os.path.join(ROOT, "tests", "native",
                                                                              "emd_sanitize_main.cpp")]
    cmd = [gxx, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=all", "-o", str(exe)] + src
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "0 bad" in r.stdout, r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
