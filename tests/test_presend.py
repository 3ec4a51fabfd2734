"""Pre-send (HttpClient::stage, LoopConfig.presend): the pre-poll warm-up hands all but the last
bytes of the poll's SQS request to the kernel corked. Nothing may reach the wire before the poll
sends the rest, the request must arrive byte for byte, and a request that turns out different
drops the staged connection instead of corrupting the next one."""
import socket
import threading
import time

import pytest

from kube_sqs_autoscaler_amd.bench.latency import BenchEnv

BODY = b"Action=GetQueueAttributes&AttributeName.1=ApproximateNumberOfMessages&" + b"x" * 300


class RecordingServer:
    """Plain HTTP/1.1 keep-alive server recording when each request's first byte arrived and the
    bytes of every request; answers 200 to each complete request."""

    def __init__(self):
        self.sock = socket.socket()
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(8)
        self.sock.settimeout(0.05)
        self.port = self.sock.getsockname()[1]
        self.first_byte_at, self.requests, self.partial = [], [], []
        self._stop = False
        self.thread = threading.Thread(target=self._serve, daemon=True)
        self.thread.start()

    def _serve(self):
        while not self._stop:
            try:
                c, _ = self.sock.accept()
            except OSError:
                continue
            threading.Thread(target=self._conn, args=(c,), daemon=True).start()

    def _conn(self, c):
        buf = b""
        while True:
            try:
                d = c.recv(65536)
            except OSError:
                d = b""
            if not d:
                if buf:
                    self.partial.append(buf)
                c.close()
                return
            if not buf:
                self.first_byte_at.append(time.monotonic())
            buf += d
            head, sep, rest = buf.partition(b"\r\n\r\n")
            if not sep:
                continue
            n = int([l.split(b":")[1] for l in head.split(b"\r\n") if l.lower().startswith(b"content-length")][0])
            if len(rest) < n:
                continue
            self.requests.append(head + sep + rest[:n])
            buf = rest[n:]
            c.sendall(b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\nok")

    def close(self):
        self._stop = True
        self.thread.join()
        self.sock.close()


@pytest.fixture
def server():
    s = RecordingServer()
    yield s
    s.close()


def test_staged_request_reaches_the_wire_only_with_the_poll(nat, server):
    c = nat.HttpClient(f"http://127.0.0.1:{server.port}", nat.TlsOptions(), 5 * nat.SECOND)
    assert c.request("POST", "/", None, b"warm")[0] == 200  # a live keep-alive connection
    hdrs = [("Content-Type", "application/x-www-form-urlencoded")]
    assert c.stage("POST", "/", hdrs, BODY) is True
    time.sleep(0.05)  # far longer than the warm-up window (the kernel holds corked data <= 200 ms)
    assert len(server.first_byte_at) == 1
    t0 = time.monotonic()
    status, _, body = c.request("POST", "/", hdrs, BODY)
    assert status == 200 and body == b"ok"
    assert len(server.first_byte_at) == 2 and server.first_byte_at[1] >= t0
    assert server.requests[1].endswith(BODY) and b"POST / HTTP/1.1" in server.requests[1]
    st = c.stats()
    assert st["presends"] == 1 and st["presend_discards"] == 0 and st["connects"] == 1


def test_a_different_request_drops_the_staged_connection(nat, server):
    c = nat.HttpClient(f"http://127.0.0.1:{server.port}", nat.TlsOptions(), 5 * nat.SECOND)
    assert c.request("POST", "/", None, b"warm")[0] == 200
    assert c.stage("POST", "/", None, BODY) is True
    other = BODY.replace(b"x", b"y")  # e.g. a signature for the next second
    status, _, _ = c.request("POST", "/", None, other)
    assert status == 200
    assert server.requests[-1].endswith(other)
    st = c.stats()
    assert st["presend_discards"] == 1 and st["presends"] == 0 and st["connects"] == 2
    deadline = time.monotonic() + 5
    while not server.partial and time.monotonic() < deadline:  # the old connection closed
        time.sleep(0.01)
    assert server.partial and BODY.startswith(server.partial[0].split(b"\r\n\r\n", 1)[1][:10])


def test_stage_needs_a_live_connection(nat, server):
    c = nat.HttpClient(f"http://127.0.0.1:{server.port}", nat.TlsOptions(), 5 * nat.SECOND)
    assert c.stage("POST", "/", None, BODY) is False  # nothing dialled yet
    assert c.request("POST", "/", None, BODY)[0] == 200


def test_staged_request_over_tls(nat):
    kube = nat.FakeKubeServer()
    kube.start("127.0.0.1", 0, True)
    kube.add_deployment("ns", "d", 3)
    try:
        tls = nat.TlsOptions()
        tls.ca_pem = kube.cert_pem
        c = nat.HttpClient(kube.url, tls, 5 * nat.SECOND)
        path = "/apis/apps/v1/namespaces/ns/deployments/d"
        assert c.request("GET", path)[0] == 200
        padding = [("X-Padding", "p" * 200)]
        assert c.stage("GET", path, padding) is True
        status, _, body = c.request("GET", path, padding)
        assert status == 200 and b'"replicas":3' in body.replace(b" ", b"")
        assert c.stats()["presends"] == 1
    finally:
        kube.stop()


@pytest.mark.parametrize("presend", [True, False])
def test_cadenced_polls_presend_their_sqs_request(nat, presend):
    """At a cadence with --poll-prewarm, each poll's SQS request is staged before its due time
    and completed by the poll -- signatures still verify, decisions unchanged."""
    env = BenchEnv(1, busy_poll_ns=25_000, poll_period_ns=20_000_000, prewarm_ns=1_000_000, presend=presend)
    try:
        env.run(12)
        res = env.collect(12, 1.0)
        st = env.sqs_apis[0].stats()["http"]
        assert res.signature_failures == 0 and len(res.samples) >= 10
        if presend:
            assert st["presends"] >= 8 and st["presend_discards"] <= 2
        else:
            assert st["presends"] == 0
    finally:
        env.close()


def test_poll_presend_flag_off_by_default_and_wired():
    """--poll-presend (default off) is LoopConfig.presend; the CLI's loop config follows it."""
    from kube_sqs_autoscaler_amd.autoscaler import loop_config
    from kube_sqs_autoscaler_amd.config import parse_args

    off = parse_args(["--sqs-queue-url=u"])
    on = parse_args(["--sqs-queue-url=u", "--poll-presend"])
    assert off.poll_presend is False and on.poll_presend is True
    for cfg in (off, on):
        lc = loop_config(cfg.targets[0], cfg.pipeline_reads, cfg.poll_prewarm_ns, 1, cfg.poll_presend)
        assert lc.presend is cfg.poll_presend


@pytest.mark.parametrize("prewarm_ms,staged", [(1, True), (60, False)])
def test_presend_only_with_a_lead_far_inside_the_cork_limit(nat, prewarm_ms, staged):
    """Linux releases TCP_CORK after 200 ms: a warm-up lead of kMaxPresendLead (50 ms) or more
    never stages, so no partial request can reach the peer before the poll."""
    env = BenchEnv(1, busy_poll_ns=25_000, poll_period_ns=3 * prewarm_ms * 1_000_000, prewarm_ns=prewarm_ms * 1_000_000,
                   presend=True)
    try:
        env.run(5)
        st = env.sqs_apis[0].stats()["http"]
        assert (st["presends"] >= 2) if staged else (st["presends"] == 0 and st["presend_discards"] == 0)
    finally:
        env.close()
