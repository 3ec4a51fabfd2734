"""Forward-proxy support: Go's proxy selection rules and the native client through a real proxy.

The reference inherits ``http.ProxyFromEnvironment`` from aws-sdk-go's and client-go's default
transports (``/root/reference/sqs/sqs.go:36``, ``/root/reference/scale/scale.go:31-52``), and
client-go v0.19 adds the kubeconfig ``proxy-url``. The rule table below follows
golang.org/x/net/http/httpproxy as documented. No Go toolchain is available here to replay its
test table, so the cases are written from those rules ("parity unpinned" against a live Go
binary).
"""
import base64
import select
import socket
import socketserver
import threading

import pytest

from kube_sqs_autoscaler_amd.autoscaler import kube_proxy, new_deployment_api, new_http_client
from kube_sqs_autoscaler_amd.kube.config import RestConfig, build_config_from_flags
from kube_sqs_autoscaler_amd.sqs.credentials import static_provider
from kube_sqs_autoscaler_amd.utils import proxy
from kube_sqs_autoscaler_amd.utils.log import capture_logger

AKID, SECRET, REGION, TOKEN = "AKIDTEST", "secret/KEY", "eu-west-1", "tok-123"
NAMES = ["ApproximateNumberOfMessages"]

# ---------------------------------------------------------------------------------------------
# selection rules


def cfg(**kw):
    return proxy.ProxyConfig(**kw)


@pytest.mark.parametrize("env,url,want", [
    # scheme picks the variable
    ({"HTTPS_PROXY": "http://p:3128"}, "https://sqs.eu-west-1.amazonaws.com", "http://p:3128"),
    ({"HTTPS_PROXY": "http://p:3128"}, "http://example.com", ""),
    ({"HTTP_PROXY": "http://p:3128"}, "http://example.com/x", "http://p:3128"),
    ({"HTTP_PROXY": "http://p:3128"}, "https://example.com", ""),
    # upper case wins; lower case is the fallback; empty upper falls through
    ({"HTTPS_PROXY": "http://up:1", "https_proxy": "http://low:2"}, "https://a.com", "http://up:1"),
    ({"https_proxy": "http://low:2"}, "https://a.com", "http://low:2"),
    ({"HTTPS_PROXY": "", "https_proxy": "http://low:2"}, "https://a.com", "http://low:2"),
    # no scheme -> http:// prepended; credentials kept
    ({"HTTPS_PROXY": "proxy.corp:3128"}, "https://a.com", "http://proxy.corp:3128"),
    ({"HTTPS_PROXY": "http://u:p@proxy:8080"}, "https://a.com", "http://u:p@proxy:8080"),
    # localhost and loopback never go through the proxy
    ({"HTTPS_PROXY": "http://p:1"}, "https://localhost:6443", ""),
    ({"HTTPS_PROXY": "http://p:1"}, "https://127.0.0.1:6443", ""),
    ({"HTTPS_PROXY": "http://p:1"}, "https://127.9.9.9", ""),
    ({"HTTPS_PROXY": "http://p:1"}, "https://[::1]:443", ""),
])
def test_proxy_for(env, url, want):
    assert proxy.ProxyConfig.from_environment(env).proxy_for(url) == want


P = "http://p:3128"


@pytest.mark.parametrize("no_proxy,url,proxied", [
    ("*", "https://a.com", False),
    ("", "https://a.com", True),
    # domains: a bare name matches itself and subdomains; a leading dot or *. only subdomains
    ("a.com", "https://a.com", False),
    ("a.com", "https://x.a.com", False),
    ("a.com", "https://xa.com", True),
    (".a.com", "https://a.com", True),
    (".a.com", "https://x.a.com", False),
    ("*.a.com", "https://a.com", True),
    ("*.a.com", "https://x.y.a.com", False),
    ("A.COM ", "https://x.a.com", False),  # case and whitespace
    # ports: an entry with a port matches only that port (default ports filled in)
    ("a.com:443", "https://a.com", False),
    ("a.com:8443", "https://a.com", True),
    ("a.com:8443", "https://a.com:8443", False),
    # IPs and CIDRs (the in-cluster apiserver address is usually excluded this way)
    ("10.96.0.1", "https://10.96.0.1:443", False),
    ("10.96.0.1:443", "https://10.96.0.1", False),
    ("10.96.0.1:6443", "https://10.96.0.1", True),
    ("10.0.0.0/8", "https://10.96.0.1", False),
    ("10.0.0.0/8", "https://11.0.0.1", True),
    ("fd00::/8", "https://[fd00::1]:443", False),
    ("::2", "https://[::2]", False),
    ("[::2]:443", "https://[::2]", False),
    # CIDR entries never match names; junk entries are ignored
    ("10.0.0.0/8", "https://a.com", True),
    ("bad/cidr,a.com", "https://a.com", False),
    (",,", "https://a.com", True),
    # several entries
    ("169.254.169.254,.svc,.cluster.local,10.0.0.0/8", "https://kubernetes.default.svc", False),
    ("169.254.169.254,.svc,.cluster.local,10.0.0.0/8", "https://sqs.us-east-1.amazonaws.com", True),
])
def test_no_proxy(no_proxy, url, proxied):
    got = cfg(https_proxy=P, no_proxy=no_proxy).proxy_for(url)
    assert got == (P if proxied else "")


def test_cgi_environment_refuses_http_proxy():
    c = proxy.ProxyConfig.from_environment({"HTTP_PROXY": P, "REQUEST_METHOD": "GET"})
    with pytest.raises(proxy.ProxyError, match="CGI"):
        c.proxy_for("http://a.com")
    assert c.proxy_for("https://a.com") == ""  # HTTPS_PROXY is unaffected (and unset)


def test_proxy_schemes():
    # Go's transport speaks http, https and socks5 proxies; other schemes get http:// prepended
    assert proxy.select("https://a.com", {"HTTPS_PROXY": "socks5://p:1080"}) == "socks5://p:1080"
    assert proxy.select("https://a.com", {}, override="https://u:pw@p:3129") == "https://u:pw@p:3129"
    assert proxy.select("http://a.com", {"HTTP_PROXY": "socks5h://p"}) == "socks5h://p"
    with pytest.raises(proxy.ProxyError, match="only http://, https:// and socks5://"):
        proxy.check_supported("ftp://p:21")
    assert proxy.redact("http://u:secret@p:1") == "http://u:xxxxx@p:1"
    assert proxy.redact("http://p:1") == "http://p:1"


def test_kubeconfig_proxy_url_overrides_environment(tmp_path):
    kc = tmp_path / "config"
    kc.write_text(
        "apiVersion: v1\nkind: Config\ncurrent-context: c\n"
        "clusters: [{name: k, cluster: {server: 'https://10.0.0.1:6443', proxy-url: 'http://kp:3128'}}]\n"
        "contexts: [{name: c, context: {cluster: k, user: u}}]\nusers: [{name: u, user: {token: t}}]\n")
    rc = build_config_from_flags(str(kc), {})
    assert rc.proxy_url == "http://kp:3128"
    assert kube_proxy(rc, {"HTTPS_PROXY": "http://env:1", "NO_PROXY": "*"}) == "http://kp:3128"
    rc.proxy_url = ""
    assert kube_proxy(rc, {"HTTPS_PROXY": "http://env:1"}) == "http://env:1"
    assert kube_proxy(rc, {"HTTPS_PROXY": "http://env:1", "NO_PROXY": "10.0.0.0/8"}) == ""


# ---------------------------------------------------------------------------------------------
# the native client through a real proxy


class _Proxy(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True

    handler = None  # _Handler (set below)

    def __init__(self, reject_with=None):
        super().__init__(("127.0.0.1", 0), type(self).handler)
        self.reject_with = reject_with
        self.connects, self.forwards, self.auth = [], [], []
        self.lock = threading.Lock()
        self.thread = threading.Thread(target=self.serve_forever, daemon=True)
        self.thread.start()

    @property
    def url(self):
        return f"http://127.0.0.1:{self.server_address[1]}"

    def close(self):
        self.shutdown()
        self.server_close()


class _Handler(socketserver.BaseRequestHandler):
    def _read_head(self):
        buf = b""
        while b"\r\n\r\n" not in buf:
            chunk = self.request.recv(4096)
            if not chunk:
                return None, b""
            buf += chunk
        head, _, rest = buf.partition(b"\r\n\r\n")
        return head.decode("latin-1"), rest

    def handle(self):
        srv = self.server
        head, rest = self._read_head()
        if head is None:
            return
        lines = head.split("\r\n")
        method, target, _ = lines[0].split(" ", 2)
        hdrs = {k.strip().lower(): v.strip() for k, v in (l.split(":", 1) for l in lines[1:] if ":" in l)}
        with srv.lock:
            srv.auth.append(hdrs.get("proxy-authorization", ""))
        if srv.reject_with:
            self.request.sendall(f"HTTP/1.1 {srv.reject_with}\r\nContent-Length: 0\r\n\r\n".encode())
            return
        if method == "CONNECT":
            host, port = target.rsplit(":", 1)
            with srv.lock:
                srv.connects.append(target)
            up = socket.create_connection((host.strip("[]"), int(port)))
            self.request.sendall(b"HTTP/1.1 200 Connection established\r\n\r\n")
            self._relay(up, b"")
        else:
            assert target.startswith("http://"), target  # absolute-form
            with srv.lock:
                srv.forwards.append(f"{method} {target}")
            authority = target[len("http://"):].split("/", 1)[0]
            host, port = authority.rsplit(":", 1)
            up = socket.create_connection((host, int(port)))
            # relay the request as received (servers accept absolute-form) and everything after it
            self._relay(up, head.encode("latin-1") + b"\r\n\r\n" + rest)

    def _relay(self, up, first):
        if first:
            up.sendall(first)
        socks = [self.request, up]
        try:
            while True:
                r, _, _ = select.select(socks, [], [], 5)
                if not r:
                    return
                for s in r:
                    data = s.recv(65536)
                    if not data:
                        return
                    (up if s is self.request else self.request).sendall(data)
        finally:
            up.close()


_Proxy.handler = _Handler


@pytest.fixture
def http_proxy():
    p = _Proxy()
    yield p
    p.close()


def test_https_through_connect_tunnel_with_auth(nat, http_proxy):
    k = nat.FakeKubeServer()
    k.require_token(TOKEN)
    k.start("127.0.0.1", 0, True)
    try:
        k.add_deployment("ml", "worker", 1)
        # explicit proxy-url (applies even to loopback, like client-go's rest.Config.Proxy)
        user_proxy = http_proxy.url.replace("http://", "http://svc%2Dacct:p%40ss@")
        rc = RestConfig(host=k.url, bearer_token=TOKEN, ca_pem=k.cert_pem, proxy_url=user_proxy)
        api = new_deployment_api(rc, "ml", "scale")
        p = nat.PodAutoScaler(api, "worker", "ml", 5, 1, 1, 1, capture_logger([]), nat.RealClock())
        for _ in range(3):
            p.scale_up()
        assert k.replicas("ml", "worker") == 4
        port = k.url.rsplit(":", 1)[1]
        assert http_proxy.connects == [f"127.0.0.1:{port}"]  # one tunnel, kept alive for 6 requests
        assert http_proxy.auth == ["Basic " + base64.b64encode(b"svc-acct:p@ss").decode()]
        assert api.stats()["http"]["connects"] == 1
    finally:
        k.stop()


def test_tls_verification_is_end_to_end(nat, http_proxy):
    k = nat.FakeKubeServer()
    k.start("127.0.0.1", 0, True)
    try:
        k.add_deployment("ml", "worker", 1)
        rc = RestConfig(host=k.url, proxy_url=http_proxy.url)  # no CA: the tunnel must not hide that
        api = new_deployment_api(rc, "ml", "scale")
        p = nat.PodAutoScaler(api, "worker", "ml", 5, 1, 1, 1, capture_logger([]), nat.RealClock())
        with pytest.raises(nat.NativeError, match="x509"):
            p.scale_up()
    finally:
        k.stop()


def test_plain_http_uses_absolute_form(nat, http_proxy):
    s = nat.FakeSqsServer()
    s.require_signature(AKID, SECRET, REGION)
    s.start()
    try:
        o = nat.SqsHttpOptions()
        o.region, o.endpoint = REGION, s.url
        o.proxy = http_proxy.url.replace("http://", "http://u:pw@")
        api = nat.HttpSqsApi(o, static_provider(AKID, SECRET), nat.RealClock())
        url = f"{s.url}/123456789012/jobs"
        s.set_attributes(url, {"ApproximateNumberOfMessages": "7"})
        c = nat.SqsClient(api, url, NAMES)
        assert c.num_messages() == 7
        assert c.num_messages() == 7
        assert s.signature_failures() == 0  # SigV4 signs Host, not the request line
        assert http_proxy.forwards == [f"POST {s.url}/"]
        assert http_proxy.auth == ["Basic " + base64.b64encode(b"u:pw").decode()]
    finally:
        s.stop()


def test_https_sqs_through_tunnel(nat, http_proxy):
    s = nat.FakeSqsServer()
    s.require_signature(AKID, SECRET, REGION)
    s.start("127.0.0.1", 0, True)
    try:
        o = nat.SqsHttpOptions()
        o.region, o.endpoint, o.proxy = REGION, s.url, http_proxy.url
        t = nat.TlsOptions()
        t.ca_pem = s.cert_pem
        o.tls = t
        api = nat.HttpSqsApi(o, static_provider(AKID, SECRET), nat.RealClock())
        url = f"{s.url}/123456789012/jobs"
        s.set_attributes(url, {"ApproximateNumberOfMessages": "5"})
        assert nat.SqsClient(api, url, NAMES).num_messages() == 5
        assert len(http_proxy.connects) == 1 and http_proxy.auth == [""]
    finally:
        s.stop()


def test_proxy_rejection_and_unreachable_proxy(nat):
    p = _Proxy(reject_with="407 Proxy Authentication Required")
    k = nat.FakeKubeServer()
    k.start("127.0.0.1", 0, True)
    try:
        c = nat.HttpClient(k.url, nat.TlsOptions(), 2_000_000_000)
        c.set_proxy(p.url)
        assert c.proxied
        with pytest.raises(nat.NativeError, match="proxy CONNECT 127.0.0.1:[0-9]+: 407 Proxy Authentication Required"):
            c.request("GET", "/version")
        dead = socket.socket()
        dead.bind(("127.0.0.1", 0))
        port = dead.getsockname()[1]
        dead.close()
        c.set_proxy(f"http://127.0.0.1:{port}")
        with pytest.raises(nat.NativeError, match="^proxyconnect tcp: dial tcp"):
            c.request("GET", "/version")
        with pytest.raises(nat.NativeError, match="unknown scheme"):
            c.set_proxy("ftp://127.0.0.1:1")
        c.set_proxy("")
        assert not c.proxied
    finally:
        k.stop()
        p.close()


def test_apiserver_helper_clients_use_the_proxy(nat, http_proxy):
    k = nat.FakeKubeServer()
    k.start("127.0.0.1", 0, True)
    try:
        rc = RestConfig(host=k.url, ca_pem=k.cert_pem, proxy_url=http_proxy.url)
        c = new_http_client(rc, 2_000_000_000)
        assert c.proxied
        status, _, _ = c.request("GET", "/api/v1/nodes")
        assert status == 200 and len(http_proxy.connects) == 1
    finally:
        k.stop()


def test_server_accepts_absolute_form(nat):
    k = nat.FakeKubeServer()
    k.start()
    try:
        k.add_deployment("ml", "worker", 2)
        with socket.create_connection(("127.0.0.1", int(k.url.rsplit(":", 1)[1]))) as s:
            s.sendall(f"GET {k.url}/apis/apps/v1/namespaces/ml/deployments/worker/scale HTTP/1.1\r\n"
                      f"Host: x\r\nConnection: close\r\n\r\n".encode())
            data = b""
            while chunk := s.recv(65536):
                data += chunk
        assert data.startswith(b"HTTP/1.1 200") and b'"replicas":2' in data.replace(b" ", b"")
    finally:
        k.stop()


# ---------------------------------------------------------------------------------------------
# https:// proxies (TLS to the proxy; TLS inside TLS for https origins) and socks5:// proxies


class _TlsProxy(_Proxy):
    """The CONNECT / absolute-form proxy above, reached over TLS."""

    def __init__(self, cert_pem, key_pem, tmp_path, reject_with=None):
        import ssl

        (tmp_path / "proxy.crt").write_text(cert_pem)
        (tmp_path / "proxy.key").write_text(key_pem)
        self.ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        self.ctx.load_cert_chain(str(tmp_path / "proxy.crt"), str(tmp_path / "proxy.key"))
        super().__init__(reject_with)

    def get_request(self):
        sock, addr = self.socket.accept()
        return self.ctx.wrap_socket(sock, server_side=True, do_handshake_on_connect=False), addr

    @property
    def url(self):
        return f"https://127.0.0.1:{self.server_address[1]}"


class _TlsHandler(_Handler):
    def setup(self):
        try:
            self.request.do_handshake()
            self.ok = True
        except OSError:  # the client rejected our certificate
            self.ok = False

    def handle(self):
        if self.ok:
            super().handle()

    def _relay(self, up, first):
        # like _Handler._relay, but decrypted bytes buffered in the TLS object are not visible
        # to select(): drain them after every read
        if first:
            up.sendall(first)
        try:
            while True:
                r, _, _ = select.select([self.request, up], [], [], 5)
                if not r:
                    return
                for s in r:
                    if s is self.request:
                        data = self.request.recv(65536)
                        while data and self.request.pending():
                            data += self.request.recv(self.request.pending())
                        if not data:
                            return
                        up.sendall(data)
                    else:
                        data = up.recv(65536)
                        if not data:
                            return
                        self.request.sendall(data)
        finally:
            up.close()


_TlsProxy.handler = _TlsHandler


class _Socks5(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True

    def __init__(self, user=None, password=None, reply=0):
        super().__init__(("127.0.0.1", 0), _Socks5Handler)
        self.user, self.password, self.reply = user, password, reply
        self.targets, self.methods, self.auth = [], [], []
        self.thread = threading.Thread(target=self.serve_forever, daemon=True)
        self.thread.start()

    @property
    def url(self):
        return f"socks5://127.0.0.1:{self.server_address[1]}"

    def close(self):
        self.shutdown()
        self.server_close()


class _Socks5Handler(_Handler):
    def _recv(self, n):
        buf = b""
        while len(buf) < n:
            chunk = self.request.recv(n - len(buf))
            if not chunk:
                raise ConnectionError("eof")
            buf += chunk
        return buf

    def handle(self):
        srv = self.server
        ver, n = self._recv(2)
        methods = list(self._recv(n))
        srv.methods.append(methods)
        if srv.user is not None:
            if 2 not in methods:
                self.request.sendall(b"\x05\xff")
                return
            self.request.sendall(b"\x05\x02")
            _, ulen = self._recv(2)
            user = self._recv(ulen).decode()
            (plen,) = self._recv(1)
            password = self._recv(plen).decode()
            srv.auth.append((user, password))
            ok = (user, password) == (srv.user, srv.password)
            self.request.sendall(b"\x01\x00" if ok else b"\x01\x01")
            if not ok:
                return
        else:
            self.request.sendall(b"\x05\x00")
        ver, cmd, _, atyp = self._recv(4)
        if atyp == 1:
            host = socket.inet_ntop(socket.AF_INET, self._recv(4))
        elif atyp == 4:
            host = socket.inet_ntop(socket.AF_INET6, self._recv(16))
        else:
            (ln,) = self._recv(1)
            host = self._recv(ln).decode()
        port = int.from_bytes(self._recv(2), "big")
        srv.targets.append((atyp, host, port))
        if srv.reply:
            self.request.sendall(bytes([5, srv.reply, 0, 1, 0, 0, 0, 0, 0, 0]))
            return
        up = socket.create_connection(("127.0.0.1" if host == "localhost" else host, port))
        self.request.sendall(b"\x05\x00\x00\x01\x7f\x00\x00\x01\x00\x00")
        self._relay(up, b"")


def test_https_proxy_tls_inside_tls(nat, tmp_path):
    """An https origin behind an https proxy: TLS to the proxy (verified with the client's trust
    settings against the proxy's name, as Go's transport does), CONNECT, then the origin's TLS
    inside it -- verified end to end, keep-alive across requests."""
    cert, key = nat.generate_self_signed("127.0.0.1")
    p = _TlsProxy(cert, key, tmp_path)
    k = nat.FakeKubeServer()
    k.require_token(TOKEN)
    k.start("127.0.0.1", 0, True)
    try:
        k.add_deployment("ml", "worker", 1)
        user_proxy = p.url.replace("https://", "https://ops:pw@")
        rc = RestConfig(host=k.url, bearer_token=TOKEN, ca_pem=k.cert_pem + cert, proxy_url=user_proxy)
        api = new_deployment_api(rc, "ml", "scale")
        pa = nat.PodAutoScaler(api, "worker", "ml", 5, 1, 1, 1, capture_logger([]), nat.RealClock())
        for _ in range(3):
            pa.scale_up()
        assert k.replicas("ml", "worker") == 4
        assert p.connects == [f"127.0.0.1:{k.url.rsplit(':', 1)[1]}"]
        assert p.auth == ["Basic " + base64.b64encode(b"ops:pw").decode()]
        assert api.stats()["http"]["connects"] == 1
    finally:
        k.stop()
        p.close()


def test_https_proxy_certificate_is_verified(nat, tmp_path):
    cert, key = nat.generate_self_signed("127.0.0.1")
    p = _TlsProxy(cert, key, tmp_path)
    k = nat.FakeKubeServer()
    k.start("127.0.0.1", 0, True)
    try:
        k.add_deployment("ml", "worker", 1)
        rc = RestConfig(host=k.url, ca_pem=k.cert_pem, proxy_url=p.url)  # the proxy's cert is not trusted
        api = new_deployment_api(rc, "ml", "scale")
        pa = nat.PodAutoScaler(api, "worker", "ml", 5, 1, 1, 1, capture_logger([]), nat.RealClock())
        with pytest.raises(nat.NativeError, match="proxyconnect tcp: x509"):
            pa.scale_up()
        assert p.connects == []
    finally:
        k.stop()
        p.close()


def test_https_proxy_plain_http_origin(nat, tmp_path):
    """An http origin (a local SQS endpoint) behind an https proxy: absolute-form requests over
    the TLS connection to the proxy; SigV4 still verifies."""
    cert, key = nat.generate_self_signed("127.0.0.1")
    p = _TlsProxy(cert, key, tmp_path)
    s = nat.FakeSqsServer()
    s.require_signature(AKID, SECRET, REGION)
    s.start()
    try:
        url = s.url + "/1/q"
        s.set_attributes(url, {"ApproximateNumberOfMessages": "7"})
        o = nat.SqsHttpOptions()
        o.region, o.endpoint, o.proxy = REGION, s.url, p.url
        tls = nat.TlsOptions()
        tls.ca_pem = cert  # trust for the proxy's certificate
        o.tls = tls
        api = nat.HttpSqsApi(o, static_provider(AKID, SECRET), nat.RealClock())
        client = nat.SqsClient(api, url, NAMES)
        assert [client.num_messages() for _ in range(3)] == [7, 7, 7]
        assert p.forwards[0].startswith("POST http://127.0.0.1:") and p.connects == []
        assert s.signature_failures() == 0
    finally:
        s.stop()
        p.close()


def test_socks5_proxy_with_auth_to_tls_origin(nat):
    sp = _Socks5(user="ops", password="p@ss")
    k = nat.FakeKubeServer()
    k.require_token(TOKEN)
    k.start("127.0.0.1", 0, True)
    try:
        k.add_deployment("ml", "worker", 1)
        rc = RestConfig(host=k.url, bearer_token=TOKEN, ca_pem=k.cert_pem,
                        proxy_url=sp.url.replace("socks5://", "socks5://ops:p%40ss@"))
        api = new_deployment_api(rc, "ml", "scale")
        pa = nat.PodAutoScaler(api, "worker", "ml", 5, 1, 1, 1, capture_logger([]), nat.RealClock())
        pa.scale_up()
        pa.scale_up()
        assert k.replicas("ml", "worker") == 3
        port = int(k.url.rsplit(":", 1)[1])
        assert sp.targets == [(1, "127.0.0.1", port)]  # one tunnel; an IP literal goes as IPv4
        assert sp.methods == [[0, 2]] and sp.auth == [("ops", "p@ss")]
    finally:
        k.stop()
        sp.close()


def test_socks5_proxy_sends_host_names_unresolved(nat):
    """A host name goes to the proxy as a domain (ATYP 3), and an http origin gets origin-form
    requests (a SOCKS tunnel is not an HTTP proxy)."""
    sp = _Socks5()
    s = nat.FakeSqsServer()
    s.start()
    try:
        port = int(s.url.rsplit(":", 1)[1])
        c = nat.HttpClient(f"http://localhost:{port}", nat.TlsOptions(), 2_000_000_000)
        c.set_proxy(sp.url)
        status, _, _ = c.request("GET", "/")
        assert status in (400, 404, 405)  # the fake answered over the tunnel
        assert sp.targets == [(3, "localhost", port)] and sp.methods == [[0]]
    finally:
        s.stop()
        sp.close()


def test_socks5_errors(nat):
    k = nat.FakeKubeServer()
    k.start("127.0.0.1", 0, True)
    refused, needs_auth = _Socks5(reply=5), _Socks5(user="u", password="p")
    try:
        c = nat.HttpClient(k.url, nat.TlsOptions(), 2_000_000_000)
        c.set_proxy(refused.url)
        with pytest.raises(nat.NativeError, match=r"^socks connect tcp 127\.0\.0\.1:[0-9]+->127\.0\.0\.1:[0-9]+: connection refused"):
            c.request("GET", "/version")
        c.set_proxy(needs_auth.url)  # no credentials in the URL
        with pytest.raises(nat.NativeError, match="no acceptable authentication methods"):
            c.request("GET", "/version")
        c.set_proxy(needs_auth.url.replace("socks5://", "socks5://u:wrong@"))
        with pytest.raises(nat.NativeError, match="authentication failed"):
            c.request("GET", "/version")
        c.set_proxy("socks5://127.0.0.1")  # default port 1080
        with pytest.raises(nat.NativeError, match="proxyconnect tcp: dial tcp 127.0.0.1:1080"):
            c.request("GET", "/version")
    finally:
        k.stop()
        refused.close()
        needs_auth.close()
