"""--poll-prewarm against an endpoint that does not answer: the warm-up dial runs under a short
budget (HttpClient::kWarmDialBudget, 100 ms, or twice the last successful dial) instead of
--api-timeout, and is not repeated while the endpoint stays down, so the SQS depth read -- which
comes after the warm-up -- keeps the reference's cadence (sleep-then-poll,
/root/reference/main.go:41-43)."""
import json
import socket
import threading
import time

import pytest
import yaml

AKID, SECRET, REGION, TOKEN = "AKIDWARM", "warm/secret", "us-east-1", "warm-token"
MS = 1_000_000


class SilentEndpoint:
    """Accepts TCP connections and never sends a byte: a TLS client's handshake waits for a
    ServerHello that never comes, as with an apiserver behind a black-holing network."""

    def __init__(self):
        self.sock = socket.socket()
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(64)
        self.port = self.sock.getsockname()[1]
        self.conns = []
        self._stop = False
        self.thread = threading.Thread(target=self._accept, daemon=True)
        self.thread.start()

    def _accept(self):
        self.sock.settimeout(0.05)
        while not self._stop:
            try:
                c, _ = self.sock.accept()
                self.conns.append(c)
            except OSError:
                continue

    def close(self):
        self._stop = True
        self.thread.join()
        for c in self.conns:
            c.close()
        self.sock.close()


@pytest.fixture
def silent():
    s = SilentEndpoint()
    yield s
    s.close()


def test_warm_dial_is_bounded_and_not_repeated_while_down(nat, silent):
    tls = nat.TlsOptions()
    tls.insecure_skip_verify = True
    c = nat.HttpClient(f"https://127.0.0.1:{silent.port}", tls, 5 * nat.SECOND)
    t0 = time.monotonic()
    assert c.warm() is False
    first = time.monotonic() - t0
    assert 0.08 <= first < 1.0, first  # ~100 ms, not the client's 5 s timeout
    t0 = time.monotonic()
    assert c.warm() is False
    assert time.monotonic() - t0 < 0.02  # no second dial while the endpoint is down
    t0 = time.monotonic()
    with pytest.raises(nat.NativeError):  # the request dials under its own timeout
        c.request("GET", "/", timeout_ns=300 * MS)
    assert 0.25 <= time.monotonic() - t0 < 2.0


def test_warm_dials_again_once_a_request_connected(nat):
    """The skip lasts until the endpoint is reachable: a request that connects re-enables the
    warm-up's dial (here: after the server dropped the connection, warm() redials)."""
    silent = SilentEndpoint()
    port = silent.port
    tls = nat.TlsOptions()
    tls.insecure_skip_verify = True
    c = nat.HttpClient(f"https://127.0.0.1:{port}", tls, 5 * nat.SECOND)
    assert c.warm(20 * MS) is False
    silent.close()
    kube = nat.FakeKubeServer()
    kube.start("127.0.0.1", port, True)
    try:
        assert c.warm() is False  # still skipping: nothing has connected since the failure
        status, _, _ = c.request("GET", "/healthz")
        assert status in (200, 404)
        kube.drop_connections()
        deadline = time.monotonic() + 5
        while c.stats()["connects"] < 2 and time.monotonic() < deadline:
            c.warm()  # the peer closed the connection: the warm-up dials a new one
            time.sleep(0.01)
        assert c.stats()["connects"] == 2
    finally:
        kube.stop()


def test_poll_cadence_holds_while_the_apiserver_drops_packets(nat, silent, tmp_path):
    """A queue likely to scale (depth over the threshold) warms its apiserver connection before
    every poll. With the apiserver black-holed, each poll's own GET fails at --api-timeout
    (300 ms), as the reference's would, but the warm-up no longer adds another --api-timeout in
    front of the SQS read: polls start a poll period after the previous one ended, except the
    first, which carries the one bounded (100 ms) warm-up dial."""
    from kube_sqs_autoscaler_amd.cli import main

    sqs = nat.FakeSqsServer()
    sqs.require_signature(AKID, SECRET, REGION)
    sqs.start()
    url = sqs.url + "/123/jobs"
    sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500", "ApproximateNumberOfMessagesDelayed": "0",
                             "ApproximateNumberOfMessagesNotVisible": "0"})
    kc = tmp_path / "kubeconfig"
    kc.write_text(yaml.safe_dump({
        "current-context": "t",
        "clusters": [{"name": "c", "cluster": {"server": f"https://127.0.0.1:{silent.port}",
                                               "insecure-skip-tls-verify": True}}],
        "users": [{"name": "u", "user": {"token": TOKEN}}],
        "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
    trace = tmp_path / "spans.jsonl"
    env = {"AWS_ACCESS_KEY_ID": AKID, "AWS_SECRET_ACCESS_KEY": SECRET, "KUBE_CONFIG_PATH": str(kc)}
    try:
        rc = main([f"--sqs-queue-url={url}", "--kubernetes-deployment=w", f"--aws-region={REGION}",
                   f"--sqs-endpoint={sqs.url}", "--poll-period=50ms", "--scale-up-cool-down=0s", "--api-timeout=300ms",
                   "--log-level=fatal", f"--trace-file={trace}"], environ=env, max_iterations=6)
    finally:
        sqs.stop()
    assert rc == 0
    spans = [json.loads(line) for line in trace.read_text().splitlines()]
    assert len(spans) == 6 and all(s["depth"] == 500 and s["up"] == "failed" for s in spans)
    # poll i starts at ts_i - total_ns_i; the previous poll ended at ts_{i-1}
    gaps = [(b["ts"] - b["total_ns"] - a["ts"]) / MS for a, b in zip(spans, spans[1:])]
    assert all(g < 50 + 150 for g in gaps), gaps  # never a 300 ms warm-up dial in front of a poll
    assert sorted(gaps)[len(gaps) // 2] < 50 + 30, gaps


class SlowTlsEndpoint:
    """A healthy TLS endpoint whose handshake starts `delay` s after the TCP accept (a distant
    apiserver or a proxy): answers every request with 200 and closes the connection."""

    def __init__(self, nat, tmp_path, delay):
        import ssl

        cert, key = nat.generate_self_signed("127.0.0.1")
        (tmp_path / "c.pem").write_text(cert)
        (tmp_path / "k.pem").write_text(key)
        self.ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        self.ctx.load_cert_chain(str(tmp_path / "c.pem"), str(tmp_path / "k.pem"))
        self.delay = delay
        self.sock = socket.socket()
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(16)
        self.sock.settimeout(0.05)
        self.port = self.sock.getsockname()[1]
        self._stop = False
        self.thread = threading.Thread(target=self._serve, daemon=True)
        self.thread.start()

    def _serve(self):
        while not self._stop:
            try:
                c, _ = self.sock.accept()
            except OSError:
                continue
            threading.Thread(target=self._one, args=(c,), daemon=True).start()

    def _one(self, c):
        try:
            time.sleep(self.delay)
            c.settimeout(5)
            s = self.ctx.wrap_socket(c, server_side=True)
            buf = b""
            while b"\r\n\r\n" not in buf:
                d = s.recv(4096)
                if not d:
                    return
                buf += d
            s.sendall(b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\nConnection: close\r\n\r\nok")
            s.close()
        except OSError:
            c.close()

    def close(self):
        self._stop = True
        self.thread.join()
        self.sock.close()


def test_warm_dial_budget_follows_a_slow_healthy_endpoint(nat, tmp_path):
    """A healthy endpoint whose dial takes longer than the 100 ms budget: the first warm-up gives
    up (and the request dials itself); after that the warm-up budget is twice the last dial time,
    so the endpoint is warmed again instead of failing every other poll."""
    ep = SlowTlsEndpoint(nat, tmp_path, 0.15)
    try:
        tls = nat.TlsOptions()
        tls.insecure_skip_verify = True
        c = nat.HttpClient(f"https://127.0.0.1:{ep.port}", tls, 5 * nat.SECOND)
        assert c.warm() is False  # 100 ms < the 150 ms handshake delay
        status, _, body = c.request("GET", "/")
        assert status == 200 and body == b"ok"  # the request's own dial (~150 ms) succeeds
        # the server closed the connection ("Connection: close"): the next warm-up redials, now
        # under 2 x ~150 ms
        t0 = time.monotonic()
        assert c.warm() is True
        assert 0.14 <= time.monotonic() - t0 < 1.0
        assert c.stats()["connects"] == 2
    finally:
        ep.close()
