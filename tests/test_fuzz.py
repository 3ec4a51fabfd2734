"""Wire-parser fuzzing (csrc/tests/fuzz_wire.cc): libFuzzer + ASan/UBSan over the JSON, XML,
URL/Atoi/RFC3339 parsers, HTTP responses into the SQS and kube clients, and HTTP requests into
the server. The CI budget is a fixed number of runs from the checked-in seed corpus; longer
campaigns: ``build/fuzz_wire -max_total_time=600 <dir> csrc/tests/fuzz_corpus``."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

from kube_sqs_autoscaler_amd.ops import build

CORPUS = Path(build.CSRC) / "tests" / "fuzz_corpus"


@pytest.fixture(scope="module")
def fuzzer():
    if not Path(build.CLANGXX).exists() and shutil.which(build.CLANGXX) is None:
        pytest.skip("no libFuzzer-capable clang")
    return build.build_fuzzer(jobs=8)


def test_seed_corpus_covers_every_target():
    firsts = {p.read_bytes()[0] % 7 for p in CORPUS.iterdir()}
    assert firsts == set(range(7))


def test_fuzz_wire_parsers(fuzzer, tmp_path):
    work = tmp_path / "corpus"
    work.mkdir()
    env = dict(os.environ, UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(fuzzer), "-runs=15000", "-seed=1", "-timeout=10", "-rss_limit_mb=2048",
                        f"-artifact_prefix={tmp_path}/", str(work), str(CORPUS)],
                       capture_output=True, text=True, timeout=600, env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "Done 15000 runs" in r.stderr
    assert "runtime error:" not in r.stderr


@pytest.mark.parametrize("text", ["1012-12-29T12:00:02.5+02:00", "0001-01-01T00:00:00Z"])
def test_rfc3339_before_1677_saturates(nat, text):
    """Found by the fuzzer: years outside int64 nanoseconds overflowed (UB)."""
    assert nat.parse_rfc3339(text) == -(2**63)


def test_rfc3339_after_2262_saturates(nat):
    assert nat.parse_rfc3339("3000-01-01T00:00:00Z") == 2**63 - 1


def test_http_server_reaps_connection_threads(nat):
    """Found by the fuzzer: the server kept one dead thread per closed connection."""
    import socket

    import time

    srv = nat.FakeSqsServer()
    srv.start()
    try:
        def live_threads():
            return len(os.listdir("/proc/self/task"))

        base = live_threads()
        for _ in range(200):
            with socket.create_connection(("127.0.0.1", srv.port)) as s:
                s.sendall(b"GET / HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
                while s.recv(4096):
                    pass
        # An exited but unjoined thread is gone from /proc/self/task yet keeps its stack mapping,
        # so the leak is counted where it lives: the server's list of unjoined connection threads
        # (finished ones are joined on the next accept; the last connection's may still be there).
        # Address-space size (VmSize) is no signal: glibc's per-thread malloc arenas reserve 64 MiB
        # each under contention and never give the reservation back.
        assert srv.connection_threads() <= 2
        deadline = time.monotonic() + 5
        while live_threads() > base + 1 and time.monotonic() < deadline:  # the last one exiting
            time.sleep(0.01)
        assert live_threads() <= base + 1
    finally:
        srv.stop()
