"""Prometheus metrics + health endpoints (extension; the reference has none).

Pull model: nothing runs per poll on the Python side. On each scrape the collector reads the
native per-worker counters (``Runner.stats()``), so the control loop never takes the GIL for
observability. The text exposition format (0.0.4) is written here with the standard library
only: the slim image ships Python, PyYAML and nothing else (Dockerfile).

Endpoints on ``--metrics-addr``: ``/metrics`` (Prometheus text format), ``/healthz`` and
``/readyz`` (see :class:`Health`).
"""
from __future__ import annotations

import math
import socket
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from .ops import native
from .parallel.fleet import Fleet

_COUNTERS = [
    ("polls", "Control-loop iterations (SQS polls)"),
    ("depth_errors", "Polls whose queue depth could not be read"),
    ("scale_ups", "Successful scale-up writes"),
    ("scale_downs", "Successful scale-down writes"),
    ("noop_ups", "Scale-ups that were no-ops at max-pods"),
    ("noop_downs", "Scale-downs that were no-ops at min-pods"),
    ("cooldown_skips_up", "Scale-ups skipped by the cool-down"),
    ("cooldown_skips_down", "Scale-downs skipped by the cool-down"),
    ("failed_ups", "Scale-ups that failed"),
    ("failed_downs", "Scale-downs that failed"),
    ("speculative_reads", "Deployment GETs sent with the SQS poll (--pipeline-reads)"),
    ("speculative_reads_used", "Speculative GETs consumed by a scale decision"),
    ("speculative_reads_gated", "Polls that sent no speculative GET because no scale call was likely"),
    ("apiserver_reads", "Deployment GETs of the control loop (speculative + synchronous)"),
]

# Per-worker API client counters: (metric, help, client attribute, stats key)
_API_COUNTERS = [
    ("apiserver_gets", "Deployment/scale GETs sent to the kube-apiserver", "kube_api", "gets"),
    ("apiserver_writes", "Deployment/scale PUT/PATCH requests sent to the kube-apiserver", "kube_api", "updates"),
    ("apiserver_conflicts", "Writes rejected with 409 Conflict", "kube_api", "conflicts"),
    ("apiserver_errors", "kube-apiserver requests that failed", "kube_api", "errors"),
    ("sqs_calls", "GetQueueAttributes calls (including SDK-style retries)", "sqs_api", "calls"),
    ("sqs_retries", "GetQueueAttributes retries", "sqs_api", "retries"),
    ("sqs_errors", "GetQueueAttributes calls that failed", "sqs_api", "errors"),
    ("sqs_throttle_retries", "Retries with the throttle back-off (429/502/503/504 or a throttling code)", "sqs_api",
     "throttle_retries"),
    ("apiserver_throttled", "Requests that waited for the client-side --kube-api-qps throttle", "kube_api", "throttled"),
    ("apiserver_throttle_seconds", "Time spent waiting for the client-side throttle", "kube_api", "throttle_ns"),
    ("speculative_reads_skipped", "Pipelined GETs not sent because no throttle token was free", "kube_api",
     "speculative_skipped"),
    ("apiserver_retries", "kube-apiserver requests retried after Retry-After (429/5xx) or a reset GET", "kube_api",
     "retry_after"),
    ("apiserver_scale_fallbacks", "Switches from the /scale subresource to whole-Deployment GET+PUT (RBAC refused /scale)",
     "kube_api", "scale_fallbacks"),
]
_NS_COUNTERS = {"throttle_ns"}  # exported in seconds

# Per-worker transport counters of each client's keep-alive connection (HttpClientStats, the
# "http" sub-dict of the client stats), labelled client="sqs" | "apiserver": (metric, help, key)
_HTTP_COUNTERS = [
    ("http_requests", "HTTP requests written (retries included)", "requests"),
    ("http_connects", "Connections dialled (TCP, plus the TLS handshake over HTTPS)", "connects"),
    ("http_tls_resumptions", "TLS handshakes that resumed a session instead of a full handshake", "tls_resumptions"),
    ("http_reconnect_retries", "Requests re-sent on a fresh connection after a reused one failed before any "
                               "response byte", "reconnect_retries"),
    ("http_idle_closed", "Keep-alive connections found closed by the peer before a request", "idle_closed"),
    ("http_presends", "Polls whose SQS request was staged during the warm-up and released at the due time",
     "presends"),
    ("http_presend_discards", "Staged requests dropped (the poll's request differed, or the connection was "
                              "replaced) together with their connection", "presend_discards"),
]
_CLIENT_LABEL = {"sqs_api": "sqs", "kube_api": "apiserver"}


def _client_stats(client) -> dict:
    try:
        return dict(client.stats())
    except (AttributeError, TypeError):  # in-process fakes without transport counters
        return {}


def _num(v: float) -> str:
    """Sample values and ``le`` bounds as the Prometheus client libraries write them."""
    v = float(v)
    if math.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    if math.isnan(v):
        return "NaN"
    return repr(v)


def _label(v: str) -> str:
    return str(v).replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


class _Family:
    """One metric family of the text exposition: HELP, TYPE, then its samples."""

    def __init__(self, name: str, kind: str, help_text: str) -> None:
        self.name, self.kind, self.help = name, kind, help_text
        self.samples: List[Tuple[str, List[Tuple[str, str]], float]] = []

    def add(self, suffix: str, labels: List[Tuple[str, str]], value: float) -> None:
        self.samples.append((suffix, labels, value))

    def render(self, out: List[str]) -> None:
        out.append(f"# HELP {self.name} {self.help.replace(chr(92), chr(92) * 2).replace(chr(10), chr(92) + 'n')}")
        out.append(f"# TYPE {self.name} {self.kind}")
        for suffix, labels, value in self.samples:
            lv = ",".join(f'{k}="{_label(v)}"' for k, v in sorted(labels))
            out.append(f"{self.name}{suffix}{{{lv}}} {_num(value)}" if lv else f"{self.name}{suffix} {_num(value)}")


class FleetCollector:
    def __init__(self, fleet: Fleet, health: Optional["Health"] = None,
                 credential_fetches: Optional[Callable[[], Dict[str, int]]] = None,
                 credential_stale_signs: Optional[Callable[[], Dict[str, int]]] = None) -> None:
        """``credential_fetches``: the process's AWS credential fetches so far, per region (the
        thread fleet's shared providers, or the process fleet's broker). ``credential_stale_signs``:
        per region, the SQS requests signed with a set kept after its refresh failed (the broker)."""
        self.fleet = fleet
        self.health = health
        self.credential_fetches = credential_fetches
        self.credential_stale_signs = credential_stale_signs

    def families(self) -> List[_Family]:
        stats = self.fleet.stats()
        fams = {k: _Family(f"ksa_{k}_total", "counter", h) for k, h in _COUNTERS}
        api = {k: _Family(f"ksa_{k}_total", "counter", h) for k, h, _, _ in _API_COUNTERS}
        http = {k: _Family(f"ksa_{k}_total", "counter", h) for k, h, _ in _HTTP_COUNTERS}
        depth = _Family("ksa_queue_depth", "gauge", "Last observed queue depth (sum of attributes)")
        reps = _Family("ksa_replicas", "gauge", "Last observed Deployment replicas")
        failing = _Family("ksa_consecutive_failed_polls", "gauge",
                          "Polls in a row that failed to read the queue depth or to write the Deployment")
        failing_s = _Family("ksa_failing_seconds", "gauge",
                            "How long every poll has been failing (0 after a successful poll)")
        cpu = _Family("ksa_poll_cpu_seconds_total", "counter",
                      "CPU time of the worker thread in its polls (warm-up and busy-poll spinning included)")
        lat = _Family("ksa_poll_to_patch_seconds", "summary", "Poll start -> replica write acknowledged")
        hist = _Family("ksa_poll_to_patch_latency_seconds", "histogram",
                       "Poll start -> replica write acknowledged, per scaling poll")
        bounds = [b / 1e9 for b in native().latency_bucket_le_ns] + [math.inf]
        for w, s in zip(self.fleet.workers, stats):
            lv = [("deployment", s["deployment"]), ("queue", s["queue"])]
            for k, _ in _COUNTERS:
                fams[k].add("", lv, s[k])
            clients = {a: _client_stats(getattr(w, a, None)) for a in ("kube_api", "sqs_api")}
            for k, _, attr, key in _API_COUNTERS:
                if key in clients[attr]:
                    v = clients[attr][key]
                    api[k].add("", lv, v / 1e9 if key in _NS_COUNTERS else v)
            for attr, name in _CLIENT_LABEL.items():
                transport = clients[attr].get("http") or {}
                for k, _, key in _HTTP_COUNTERS:
                    if key in transport:
                        http[k].add("", lv + [("client", name)], transport[key])
            depth.add("", lv, s["last_depth"])
            reps.add("", lv, s["last_replicas"])
            failing.add("", lv, s.get("consecutive_failed_polls", 0))
            failing_s.add("", lv, w.runner.failing_ns() / 1e9)
            cpu.add("", lv, s.get("poll_cpu_ns", 0) / 1e9)
            # every sample since start (the latency ring only keeps the latest)
            lat.add("_count", lv, s["latency_samples"])
            lat.add("_sum", lv, s["latency_sum_ns"] / 1e9)
            cum = 0
            for le, n in zip(bounds, s["latency_buckets"]):
                cum += n
                hist.add("_bucket", lv + [("le", _num(le))], cum)
            hist.add("_count", lv, cum)
            hist.add("_sum", lv, s["latency_sum_ns"] / 1e9)
        out = [*fams.values(), *(f for f in (*api.values(), *http.values()) if f.samples), depth, reps, failing,
               failing_s, cpu, lat, hist]
        if self.credential_fetches is not None:
            creds = _Family("ksa_aws_credential_fetches_total", "counter",
                            "AWS credential fetches of the process (one source per region, shared by its queues)")
            for region, n in sorted(self.credential_fetches().items()):
                creds.add("", [("region", region)], n)
            out.append(creds)
        if self.credential_stale_signs is not None:
            stale = _Family("ksa_aws_credential_stale_signs_total", "counter",
                            "SQS requests signed with an AWS credential set inside its 5-minute refresh window because "
                            "its refresh failed (the set valid for more than a minute yet)")
            for region, n in sorted(self.credential_stale_signs().items()):
                stale.add("", [("region", region)], n)
            out.append(stale)
        return out

    def exposition(self) -> bytes:
        out: List[str] = []
        for f in self.families():
            f.render(out)
        return ("\n".join(out) + "\n").encode()


class Health:
    """Liveness and readiness of the process.

    * ``/healthz`` fails when the fleet is stopping, or when a running worker has made no
      progress for longer than its budget: ``poll period + 8 x api timeout + 60 s``. The
      budget covers an SQS call with 3 SDK retries, the GET, the write, and a 409 re-read, each
      bounded by ``--api-timeout``. Deliberate waits are not: SQS back-off, a server's
      ``Retry-After`` (up to an hour) and the client-side throttle count as progress up to
      their end (``Runner.idle_ns``), so a worker correctly backing off is not restarted. A
      worker stuck past all of them is wedged, and a restart (Kubernetes' liveness probe) is the
      recovery. The reference has no probes and hangs on a stalled call.
    * ``/readyz`` is OK for a standby replica under ``--leader-elect``, since waiting for the
      lease is its healthy state. Otherwise it is OK once every worker has completed a poll,
      and fails again while a worker's every poll has failed -- to read the queue depth or to
      write the Deployment -- for ``failure_window_ns`` (``--readiness-failure-window``, 5 min;
      0 disables). A pod that can never read its queue or write its Deployment (a wrong IAM
      role, a Role without ``update``) then shows NotReady instead of healthy forever; one
      good poll makes it ready again. Liveness stays as it is: like the reference, the loop
      retries such a poll forever (main.go:44-47,57-60,71-74), and a restart would not fix a
      permission. A standby that never became ready would stall every rolling update of a
      2-replica Deployment.
    """

    def __init__(self, fleet: Fleet, stale_after_ns: Optional[Sequence[int]] = None, leader_elect: bool = False,
                 failure_window_ns: int = 300 * 10**9) -> None:
        self.fleet = fleet
        self.stale_after_ns = list(stale_after_ns) if stale_after_ns is not None else None
        self.role = "standby" if leader_elect else "active"
        self.failure_window_ns = failure_window_ns

    @staticmethod
    def budget_ns(poll_period_ns: int, api_timeout_ns: int) -> int:
        return poll_period_ns + 8 * api_timeout_ns + 60 * 10**9

    def set_role(self, role: str) -> None:
        self.role = role

    def live(self) -> Tuple[bool, str]:
        if self.fleet.stopped:
            return False, "stopping"
        if self.role == "standby" or not self.fleet.started or self.stale_after_ns is None:
            return True, "ok"
        for w, limit in zip(self.fleet.workers, self.stale_after_ns):
            idle = w.runner.idle_ns()
            if idle > limit:
                return False, f"worker {w.target.name} made no progress for {idle / 1e9:.0f}s (budget {limit / 1e9:.0f}s)"
        return True, "ok"

    def ready(self) -> Tuple[bool, str]:
        if self.role == "standby" and not self.fleet.stopped:
            return True, "standby"
        ok, why = self.live()
        if not ok:
            return False, why
        if not all(s["polls"] > 0 for s in self.fleet.stats()):
            return False, "waiting for first poll"
        if self.failure_window_ns > 0:
            for w in self.fleet.workers:
                failing = w.runner.failing_ns()
                if failing >= self.failure_window_ns:
                    n = w.runner.stats().get("consecutive_failed_polls", 0)
                    err = w.runner.last_error()
                    return False, (f"worker {w.target.name}: every poll failed for {failing / 1e9:.0f}s ({n} polls)"
                                   + (f"; last error: {err}" if err else ""))
        return True, "ok"


def parse_addr(addr: str) -> Tuple[str, int]:
    """Go's ``host:port`` listen address: ``:9090`` (every interface), ``0.0.0.0:9090``,
    ``[::]:9090`` (an IPv6 literal in brackets). Returns ("", port) for every interface."""
    host, sep, port = addr.rpartition(":")
    if not sep:
        raise ValueError(f"address {addr}: missing port in address")
    if host.startswith("[") and host.endswith("]"):
        host = host[1:-1]
    return host, int(port)


class _Server(ThreadingHTTPServer):
    daemon_threads = True
    dual_stack = False

    def server_bind(self) -> None:
        if self.dual_stack:  # "[::]" taking IPv4 too, as Go's ":port" listener does
            self.socket.setsockopt(socket.IPPROTO_IPV6, socket.IPV6_V6ONLY, 0)
        super().server_bind()


def _listen(host: str, port: int, handler) -> ThreadingHTTPServer:
    if host:
        cls = type("_Server6" if ":" in host else "_Server4", (_Server,),
                   {"address_family": socket.AF_INET6 if ":" in host else socket.AF_INET})
        return cls((host, port), handler)
    # every interface: dual-stack IPv6 where the host has it (an IPv6-only cluster reaches the
    # pod on its IPv6 address), plain IPv4 otherwise
    if socket.has_ipv6:
        try:
            cls = type("_ServerDual", (_Server,), {"address_family": socket.AF_INET6, "dual_stack": True})
            return cls(("::", port), handler)
        except OSError:
            pass
    return type("_Server4", (_Server,), {"address_family": socket.AF_INET})(("0.0.0.0", port), handler)


class MetricsServer:
    def __init__(self, fleet: Fleet, addr: str, health: Optional[Health] = None,
                 credential_fetches: Optional[Callable[[], Dict[str, int]]] = None,
                 credential_stale_signs: Optional[Callable[[], Dict[str, int]]] = None) -> None:
        self.fleet = fleet
        self.health = health or Health(fleet)
        hl = self.health
        self.collector = FleetCollector(fleet, credential_fetches=credential_fetches,
                                        credential_stale_signs=credential_stale_signs)
        coll = self.collector

        class Handler(BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802
                if self.path == "/metrics":
                    body, code, ctype = coll.exposition(), 200, "text/plain; version=0.0.4; charset=utf-8"
                elif self.path in ("/healthz", "/readyz"):
                    ok, why = hl.live() if self.path == "/healthz" else hl.ready()
                    body, code, ctype = why.encode(), (200 if ok else 503), "text/plain"
                else:
                    body, code, ctype = b"not found", 404, "text/plain"
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):  # silence http.server access logs
                pass

        host, port = parse_addr(addr)
        self.httpd = _listen(host, port, Handler)
        self.port = self.httpd.server_address[1]
        self._thread: Optional[threading.Thread] = None

    def start(self) -> None:
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="ksa-metrics", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
