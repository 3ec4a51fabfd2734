"""Prometheus metrics + health endpoints (extension; the reference has none).

Pull model: nothing runs per poll on the Python side. On each scrape the collector reads the
native per-worker counters (``Runner.stats()``) and the latency ring (``Runner.latencies()``),
so the control loop never takes the GIL for observability.

Endpoints on ``--metrics-addr``: ``/metrics`` (Prometheus text format), ``/healthz`` (process
alive and workers not stopped), ``/readyz`` (every worker completed at least one poll).
"""
from __future__ import annotations

import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Optional, Tuple

from prometheus_client import CollectorRegistry, generate_latest
from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily, SummaryMetricFamily

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
]


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
        lat = SummaryMetricFamily("ksa_poll_to_patch_seconds", "Poll end -> replica write latency", labels=labels)
        api = {k: CounterMetricFamily(f"ksa_{k}", h, labels=labels) for k, h, _, _ in _API_COUNTERS}
        for w, s in zip(self.fleet.workers, stats):
            lv = [s["deployment"], s["queue"]]
            for k, _ in _COUNTERS:
                fams[k].add_metric(lv, s[k])
            clients = {a: _client_stats(getattr(w, a, None)) for a in ("kube_api", "sqs_api")}
            for k, _, attr, key in _API_COUNTERS:
                if key in clients[attr]:
                    api[k].add_metric(lv, clients[attr][key])
            depth.add_metric(lv, s["last_depth"])
            reps.add_metric(lv, s["last_replicas"])
            samples = w.runner.latencies()
            lat.add_metric(lv, count_value=s["latency_samples"], sum_value=sum(samples) / 1e9)
        yield from fams.values()
        yield from (f for f in api.values() if f.samples)
        yield depth
        yield reps
        yield lat


def parse_addr(addr: str) -> Tuple[str, int]:
    host, _, port = addr.rpartition(":")
    return (host or "0.0.0.0"), int(port)


class MetricsServer:
    def __init__(self, fleet: Fleet, addr: str) -> None:
        self.fleet = fleet
        self.registry = CollectorRegistry()
        self.registry.register(FleetCollector(fleet))
        reg = self.registry
        fl = fleet

        class Handler(BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802
                if self.path == "/metrics":
                    body, code, ctype = generate_latest(reg), 200, "text/plain; version=0.0.4; charset=utf-8"
                elif self.path == "/healthz":
                    ok = not fl.stopped
                    body, code, ctype = (b"ok" if ok else b"stopping"), (200 if ok else 503), "text/plain"
                elif self.path == "/readyz":
                    ok = all(s["polls"] > 0 for s in fl.stats())
                    body, code, ctype = (b"ok" if ok else b"waiting for first poll"), (200 if ok else 503), "text/plain"
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
