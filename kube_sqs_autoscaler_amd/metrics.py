"""Prometheus metrics + health endpoints (extension; the reference has none).

Pull model: nothing runs per poll on the Python side. On each scrape the collector reads the
native per-worker counters (``Runner.stats()``) and the latency ring (``Runner.latencies()``),
so the control loop never takes the GIL for observability.

Endpoints on ``--metrics-addr``: ``/metrics`` (Prometheus text format), ``/healthz`` and
``/readyz`` (see :class:`Health`).
"""
from __future__ import annotations

import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Optional, Sequence, Tuple

from prometheus_client import CollectorRegistry, generate_latest
from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily, HistogramMetricFamily, SummaryMetricFamily

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


def _client_stats(client) -> dict:
    try:
        return dict(client.stats())
    except (AttributeError, TypeError):  # in-process fakes without transport counters
        return {}


class FleetCollector:
    def __init__(self, fleet: Fleet) -> None:
        self.fleet = fleet

    def collect(self):
        labels = ["deployment", "queue"]
        stats = self.fleet.stats()
        fams = {k: CounterMetricFamily(f"ksa_{k}", h, labels=labels) for k, h in _COUNTERS}
        depth = GaugeMetricFamily("ksa_queue_depth", "Last observed queue depth (sum of attributes)", labels=labels)
        reps = GaugeMetricFamily("ksa_replicas", "Last observed Deployment replicas", labels=labels)
        lat = SummaryMetricFamily("ksa_poll_to_patch_seconds", "Poll start -> replica write acknowledged", labels=labels)
        hist = HistogramMetricFamily("ksa_poll_to_patch_latency_seconds",
                                     "Poll start -> replica write acknowledged, per scaling poll", labels=labels)
        bounds = [b / 1e9 for b in native().latency_bucket_le_ns]
        api = {k: CounterMetricFamily(f"ksa_{k}", h, labels=labels) for k, h, _, _ in _API_COUNTERS}
        for w, s in zip(self.fleet.workers, stats):
            lv = [s["deployment"], s["queue"]]
            for k, _ in _COUNTERS:
                fams[k].add_metric(lv, s[k])
            clients = {a: _client_stats(getattr(w, a, None)) for a in ("kube_api", "sqs_api")}
            for k, _, attr, key in _API_COUNTERS:
                if key in clients[attr]:
                    v = clients[attr][key]
                    api[k].add_metric(lv, v / 1e9 if key in _NS_COUNTERS else v)
            depth.add_metric(lv, s["last_depth"])
            reps.add_metric(lv, s["last_replicas"])
            # every sample since start (the latency ring only keeps the latest)
            lat.add_metric(lv, count_value=s["latency_samples"], sum_value=s["latency_sum_ns"] / 1e9)
            cum, buckets = 0, []
            for le, n in zip(bounds + [float("inf")], s["latency_buckets"]):
                cum += n
                buckets.append(("+Inf" if le == float("inf") else repr(le), cum))
            hist.add_metric(lv, buckets, sum_value=s["latency_sum_ns"] / 1e9)
        yield from fams.values()
        yield from (f for f in api.values() if f.samples)
        yield depth
        yield reps
        yield lat
        yield hist


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
      lease is its healthy state. Otherwise it is OK once every worker has completed a poll.
      A standby that never became ready would stall every rolling update of a 2-replica
      Deployment.
    """

    def __init__(self, fleet: Fleet, stale_after_ns: Optional[Sequence[int]] = None, leader_elect: bool = False) -> None:
        self.fleet = fleet
        self.stale_after_ns = list(stale_after_ns) if stale_after_ns is not None else None
        self.role = "standby" if leader_elect else "active"

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
        return True, "ok"


def parse_addr(addr: str) -> Tuple[str, int]:
    host, _, port = addr.rpartition(":")
    return (host or "0.0.0.0"), int(port)


class MetricsServer:
    def __init__(self, fleet: Fleet, addr: str, health: Optional[Health] = None) -> None:
        self.fleet = fleet
        self.health = health or Health(fleet)
        hl = self.health
        self.registry = CollectorRegistry()
        self.registry.register(FleetCollector(fleet))
        reg = self.registry

        class Handler(BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802
                if self.path == "/metrics":
                    body, code, ctype = generate_latest(reg), 200, "text/plain; version=0.0.4; charset=utf-8"
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
        self.httpd = ThreadingHTTPServer((host, port), Handler)
        self.port = self.httpd.server_address[1]
        self._thread: Optional[threading.Thread] = None

    def start(self) -> None:
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="ksa-metrics", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
