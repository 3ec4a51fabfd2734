"""The closed-loop model's integer square root (``isqrt64`` in csrc/sim/queue_sim.h) is exact:
its single-precision estimate below 2^48 and double-precision one above are corrected to
floor(sqrt(x)). Compiles ``csrc/tests/isqrt_check.cc`` with the host compiler and runs it."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_isqrt64_is_exact(tmp_path):
    exe = tmp_path / "isqrt_check"
    subprocess.run(["g++", "-O2", "-std=c++17", str(ROOT / "csrc" / "tests" / "isqrt_check.cc"), "-o", str(exe)],
                   check=True, capture_output=True, text=True)
    r = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("0 failures")
