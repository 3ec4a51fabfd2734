"""Host C++ unit tests of the native runtime: plain, ASan+UBSan and TSan builds (csrc/tests)."""
import os
import subprocess

import pytest

from kube_sqs_autoscaler_amd.ops import build


@pytest.mark.parametrize("sanitizer", [None, "asan", "tsan"])
def test_native_unit_tests(sanitizer):
    exe = build.build_native_tests(sanitizer, jobs=8)
    env = dict(os.environ)
    env["TSAN_OPTIONS"] = "halt_on_error=1 second_deadlock_stack=1"
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "0 failed" in r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
    assert "runtime error:" not in r.stderr  # UBSan
