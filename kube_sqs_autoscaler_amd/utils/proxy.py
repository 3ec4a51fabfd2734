"""Forward-proxy selection with Go's ``net/http`` rules.

The reference reaches SQS through aws-sdk-go's default HTTP client and the apiserver through
client-go. Both use ``http.ProxyFromEnvironment`` (golang.org/x/net/http/httpproxy), so a pod
behind an egress proxy works when ``HTTPS_PROXY`` / ``NO_PROXY`` are set. client-go v0.19
(``/root/reference/go.mod:15``) also honours a kubeconfig cluster's ``proxy-url``. This module
picks the proxy the same way. The native ``HttpClient::set_proxy`` (``csrc/core/http.cc``)
speaks the three proxy kinds Go's transport does: ``http://`` and ``https://`` proxies (CONNECT
tunnels for https origins, absolute-form requests for http ones; an https proxy is itself
reached over verified TLS) and ``socks5://`` (a SOCKS5 CONNECT, host names resolved by the
proxy).

Rules (httpproxy ``Config.ProxyFunc``):

* ``HTTPS_PROXY`` applies to https URLs and ``HTTP_PROXY`` to http URLs. The upper-case name
  wins; the lower-case name is the fallback.
* A value without a usable scheme gets ``http://`` prepended (``proxy:3128`` works).
* ``localhost`` and loopback IPs are never proxied.
* ``NO_PROXY`` is a comma list. Each entry may be:
  * ``*`` — proxy nothing;
  * a CIDR (``10.0.0.0/8``);
  * an IP, optionally with a port;
  * a domain, optionally with a port. ``foo.com`` matches ``foo.com`` and its subdomains;
    ``.foo.com`` and ``*.foo.com`` match subdomains only.
* With ``REQUEST_METHOD`` set (a CGI environment), ``HTTP_PROXY`` is refused.
"""
from __future__ import annotations

import ipaddress
import os
import urllib.parse
from dataclasses import dataclass, field
from typing import List, Mapping, Optional, Tuple

SUPPORTED_SCHEMES = ("http", "https", "socks5", "socks5h")  # what the native client speaks to a proxy


class ProxyError(ValueError):
    pass


def _env_any(env: Mapping[str, str], *names: str) -> str:
    for n in names:
        v = env.get(n)
        if v:  # Go's getEnvAny: first non-empty
            return v
    return ""


def parse_proxy(value: str) -> str:
    """httpproxy ``parseProxy``: returns a normalised ``scheme://[userinfo@]host:port`` or ``""``."""
    value = value.strip()
    if not value:
        return ""
    u = urllib.parse.urlsplit(value)
    if u.scheme not in SUPPORTED_SCHEMES or not u.hostname:
        u = urllib.parse.urlsplit("http://" + value)
        if not u.hostname:
            raise ProxyError(f"invalid proxy address {value!r}")
    return urllib.parse.urlunsplit((u.scheme, u.netloc, "", "", ""))


def _split_host_port(addr: str) -> Tuple[str, str]:
    if addr.startswith("["):
        end = addr.find("]")
        if end < 0:
            raise ValueError(addr)
        rest = addr[end + 1:]
        if rest and not rest.startswith(":"):
            raise ValueError(addr)
        return addr[1:end], rest[1:]
    if addr.count(":") == 1:
        h, p = addr.split(":")
        return h, p
    if ":" in addr:
        raise ValueError(addr)  # bare IPv6 without brackets and port: not host:port
    return addr, ""


def _ip(s: str):
    try:
        return ipaddress.ip_address(s)
    except ValueError:
        return None


@dataclass
class ProxyConfig:
    http_proxy: str = ""
    https_proxy: str = ""
    no_proxy: str = ""
    cgi: bool = False
    _ips: List[Tuple[object, str]] = field(default_factory=list, init=False, repr=False)
    _nets: List[object] = field(default_factory=list, init=False, repr=False)
    _domains: List[Tuple[str, str, bool]] = field(default_factory=list, init=False, repr=False)
    _all: bool = field(default=False, init=False, repr=False)

    def __post_init__(self):
        for raw in self.no_proxy.split(","):
            p = raw.strip().lower()
            if not p:
                continue
            if p == "*":
                self._all = True
                return
            if "/" in p:
                try:
                    self._nets.append(ipaddress.ip_network(p, strict=False))
                except ValueError:
                    pass
                continue
            try:
                host, port = _split_host_port(p)
            except ValueError:
                host, port = p, ""
            if not host:
                continue
            ip = _ip(host)
            if ip is not None:
                self._ips.append((ip, port))
                continue
            if host.startswith("*."):
                host = host[1:]
            match_host = not host.startswith(".")
            if match_host:
                host = "." + host
            self._domains.append((host, port, match_host))

    @classmethod
    def from_environment(cls, environ: Optional[Mapping[str, str]] = None) -> "ProxyConfig":
        env = os.environ if environ is None else environ
        return cls(http_proxy=_env_any(env, "HTTP_PROXY", "http_proxy"),
                   https_proxy=_env_any(env, "HTTPS_PROXY", "https_proxy"),
                   no_proxy=_env_any(env, "NO_PROXY", "no_proxy"),
                   cgi=bool(env.get("REQUEST_METHOD")))

    def use_proxy(self, host: str, port: str) -> bool:
        """httpproxy ``useProxy`` on a canonical ``host``/``port``."""
        if host == "localhost":
            return False
        host = host.strip().lower()
        ip = _ip(host)
        if ip is not None and ip.is_loopback:
            return False
        if self._all:
            return False
        if ip is not None:
            if any(ip in n for n in self._nets):
                return False
            if any(ip == m and (not mp or mp == port) for m, mp in self._ips):
                return False
        for dom, dport, match_host in self._domains:
            if host.endswith(dom) or (match_host and host == dom[1:]):
                if not dport or dport == port:
                    return False
        return True

    def proxy_for(self, url: str) -> str:
        """The proxy URL to use for ``url`` or ``""`` to connect directly."""
        u = urllib.parse.urlsplit(url)
        scheme = u.scheme.lower()
        if scheme == "https":
            proxy = parse_proxy(self.https_proxy)
        elif scheme == "http":
            proxy = parse_proxy(self.http_proxy)
            if proxy and self.cgi:
                raise ProxyError("refusing to use HTTP_PROXY value in CGI environment; see golang.org/s/cgihttpproxy")
        else:
            return ""
        if not proxy:
            return ""
        host = (u.hostname or "").lower()
        port = str(u.port) if u.port else ("443" if scheme == "https" else "80")
        return proxy if self.use_proxy(host, port) else ""


def check_supported(proxy: str) -> str:
    """Rejects a proxy scheme the native client does not speak (fail loudly rather than
    connect directly)."""
    if proxy and urllib.parse.urlsplit(proxy).scheme not in SUPPORTED_SCHEMES:
        raise ProxyError(f"proxy {redact(proxy)}: only http://, https:// and socks5:// proxies are supported")
    return proxy


def redact(proxy: str) -> str:
    """``http://user:pass@host:3128`` → ``http://user:xxxxx@host:3128`` (for logs)."""
    u = urllib.parse.urlsplit(proxy)
    if u.password is None:
        return proxy
    netloc = u.netloc.replace(":" + u.password + "@", ":xxxxx@", 1)
    return urllib.parse.urlunsplit((u.scheme, netloc, u.path, u.query, u.fragment))


def select(url: str, environ: Optional[Mapping[str, str]] = None, override: str = "") -> str:
    """Proxy for ``url``: a kubeconfig ``proxy-url`` override wins over the environment
    (client-go ``rest.Config.Proxy``); ``""`` = direct."""
    if override:
        return check_supported(parse_proxy(override))
    return check_supported(ProxyConfig.from_environment(environ).proxy_for(url))
