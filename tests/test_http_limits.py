"""Hostile or broken peers: the native HTTP client bounds what it buffers (csrc/core/http.cc
kMaxBody = 128 MiB, 1 MiB header / line caps) instead of growing until the 200 MiB pod dies."""
import socket
import threading

import pytest


def one_shot_server(payload: bytes, trickle: bytes = b""):
    """Accepts one connection, reads the request head, sends `payload`, then `trickle` forever
    (until the client goes away)."""
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)

    def run():
        c, _ = srv.accept()
        with c:
            buf = b""
            while b"\r\n\r\n" not in buf:
                d = c.recv(4096)
                if not d:
                    return
                buf += d
            try:
                c.sendall(payload)
                while trickle:
                    c.sendall(trickle)
            except OSError:
                pass

    t = threading.Thread(target=run, daemon=True)
    t.start()
    return srv, t


@pytest.mark.parametrize("payload,trickle,msg", [
    (b"HTTP/1.1 200 OK\r\nContent-Length: 1000000000000\r\n\r\n", b"", "bad Content-Length"),
    (b"HTTP/1.1 200 OK\r\nContent-Length: 99999999999999999999999\r\n\r\n", b"", "bad Content-Length"),
    (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nfffffffffff\r\n", b"", "message body too large"),
    (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nfffffffffffffffffffffffff\r\n", b"", "malformed chunk size"),
    (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n", b"x" * 65536, "line too long"),
    (b"HTTP/1.1 200 OK\r\nConnection: close\r\n\r\n", b"y" * (1 << 20), "message body too large"),
    (b"HTTP/1.1 200 OK\r\nX-Junk: ", b"z" * 65536, "header too large"),
])
def test_client_bounds_hostile_responses(nat, payload, trickle, msg):
    srv, t = one_shot_server(payload, trickle)
    try:
        c = nat.HttpClient(f"http://127.0.0.1:{srv.getsockname()[1]}", nat.TlsOptions(), 60 * nat.SECOND)
        with pytest.raises(nat.NativeError, match=msg):
            c.request("GET", "/", [], b"")
        c.close()
    finally:
        srv.close()


def test_hostname_resolution_works_and_is_bounded(nat):
    """Names resolve on a helper thread bounded by the call deadline (getaddrinfo has none)."""
    import time

    kube = nat.FakeKubeServer()
    kube.start()
    try:
        kube.add_deployment("ml", "w", 2)
        c = nat.HttpClient(f"http://localhost:{kube.port}", nat.TlsOptions(), 5 * nat.SECOND)
        status, _, body = c.request("GET", "/apis/apps/v1/namespaces/ml/deployments/w/scale", [], b"")
        assert status == 200 and b'"replicas":2' in body
    finally:
        kube.stop()
    c = nat.HttpClient("http://ksa-no-such-host.invalid:80", nat.TlsOptions(), 500_000_000)
    t0 = time.perf_counter()
    with pytest.raises(nat.NativeError, match="lookup ksa-no-such-host.invalid"):
        c.request("GET", "/", [], b"")
    assert time.perf_counter() - t0 < 2.0
