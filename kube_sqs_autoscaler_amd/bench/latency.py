"""Poll -> scale-patch latency benchmark against localhost fake SQS / kube-apiserver servers.

BASELINE.json's metric is the p50 of the time from the end of the poll sleep to the end of the
replica write (``Runner`` records it per iteration, csrc/core/runner.cc), at 1/2/4/8
concurrently tracked queues. Every tracked queue gets its own native worker thread, its own
persistent connections and its own Deployment; all of them share one fake SQS endpoint and one
fake apiserver (as production shares AWS and the apiserver).

The wire path is the production one: SigV4-signed ``GetQueueAttributes`` (verified by the
fake), bearer-token kube REST calls with resourceVersion preconditions, real attribute summing
and clamp arithmetic, info-level logrus lines written to a file descriptor.

Two paths are measured: the optimised default (``/scale`` subresource + pipelined read: the
Deployment GET overlaps the SQS call) and the reference-equivalent one (full-object GET+PUT,
strictly sequential -- what /root/reference/scale/scale.go:54-107 does after sqs.go:51).

Trace: the fake serves the BASELINE.json "step trace" 200 -> 0 -> 200 ... one value per poll,
with scale-up-messages=100 / scale-down-messages=10, min 1 / max 8 and zero poll period and
cool-downs, so *every* iteration performs SQS + GET + write (the 3-round-trip scaling path of
SURVEY.md §3.2) -- the path whose latency the metric names.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..autoscaler import new_deployment_api, new_pod_autoscaler, new_sqs_api, new_sqs_client
from ..config import TargetConfig
from ..kube.config import RestConfig
from ..ops import native
from ..sqs.credentials import static_provider

AKID = "AKIDBENCHEXAMPLE"
SECRET = "bench/secret/key/EXAMPLEKEY"
TOKEN = "bench-bearer-token"
REGION = "us-east-1"


@dataclass
class LatencyResult:
    queues: int
    mode: str
    steps: int
    pipeline: bool = True
    samples: List[int] = field(default_factory=list)  # ns
    wall_s: float = 0.0
    sqs_requests: int = 0
    kube_requests: int = 0
    sqs_connections: int = 0
    kube_connections: int = 0
    signature_failures: int = 0
    final_replicas: List[int] = field(default_factory=list)

    def pct(self, p: float) -> float:
        """Nearest-rank percentile in milliseconds."""
        if not self.samples:
            return float("nan")
        v = sorted(self.samples)
        import math

        k = max(1, math.ceil(p / 100.0 * len(v)))
        return v[min(k, len(v)) - 1] / 1e6

    def summary(self) -> Dict[str, float]:
        return {
            "queues": self.queues,
            "mode": self.mode,
            "pipeline_reads": self.pipeline,
            "p50_ms": round(self.pct(50), 4),
            "p90_ms": round(self.pct(90), 4),
            "p99_ms": round(self.pct(99), 4),
            "samples": len(self.samples),
            "iterations_per_s": round(self.queues * self.steps / self.wall_s, 1) if self.wall_s else 0.0,
        }


class BenchEnv:
    """Fake servers + one worker per queue."""

    def __init__(self, queues: int, mode: str = "scale", tls: bool = False, sqs_latency_ns: int = 0,
                 kube_latency_ns: int = 0, log_fd: Optional[int] = None, pipeline: bool = True,
                 busy_poll_ns: int = 0, servers: str = "shared", loggers: str = "shared"):
        nat = native()
        self.nat = nat
        self.mode = mode
        self.pipeline = pipeline
        # servers="per-queue": every queue gets its own fake SQS endpoint and fake apiserver, as
        # separate processes (one rank per GPU) have; "shared": one of each serves every queue.
        n_servers = queues if servers == "per-queue" else 1
        self.sqs_servers, self.kube_servers = [], []
        for _ in range(n_servers):
            sqs = nat.FakeSqsServer()
            sqs.require_signature(AKID, SECRET, REGION)
            sqs.start("127.0.0.1", 0, tls)
            sqs.set_latency(sqs_latency_ns)
            kube = nat.FakeKubeServer()
            kube.require_token(TOKEN)
            kube.start("127.0.0.1", 0, tls)
            kube.set_latency(kube_latency_ns)
            self.sqs_servers.append(sqs)
            self.kube_servers.append(kube)
        self.sqs, self.kube = self.sqs_servers[0], self.kube_servers[0]
        self.clock = nat.RealClock()
        self._devnull = None
        if log_fd is None:
            self._devnull = os.open(os.devnull, os.O_WRONLY)
            log_fd = self._devnull
        self.loggers = []
        for _ in range(queues if loggers == "per-queue" else 1):
            lg = nat.Logger()
            lg.set_sink_fd(log_fd)
            self.loggers.append(lg)
        self.log = self.loggers[0]
        high = {"ApproximateNumberOfMessages": "150", "ApproximateNumberOfMessagesDelayed": "20",
                "ApproximateNumberOfMessagesNotVisible": "30"}
        low = {"ApproximateNumberOfMessages": "0", "ApproximateNumberOfMessagesDelayed": "0",
               "ApproximateNumberOfMessagesNotVisible": "0"}
        creds = static_provider(AKID, SECRET)
        self.runners = []
        self.kube_apis, self.sqs_apis = [], []
        self.targets = []
        self.server_of = []  # queue -> index of the server pair that serves it
        for q in range(queues):
            si = q % n_servers
            sqs, kube, log = self.sqs_servers[si], self.kube_servers[si], self.loggers[q % len(self.loggers)]
            rest = RestConfig(host=kube.url, bearer_token=TOKEN, insecure=tls)
            sqs_tls = None
            if tls:
                sqs_tls = nat.TlsOptions()
                sqs_tls.ca_pem = sqs.cert_pem
                rest.insecure = False
                rest.ca_pem = kube.cert_pem
            url = f"{sqs.url}/000000000000/bench-queue-{q}"
            name = f"gpu-worker-{q}"
            sqs.set_attribute_cycle(url, [high, low])
            kube.add_deployment("bench", name, 1)
            self.server_of.append(si)
            t = TargetConfig(queue_url=url, deployment=name, namespace="bench", poll_period_ns=0,
                             scale_up_cool_down_ns=0, scale_down_cool_down_ns=0, scale_up_messages=100,
                             scale_down_messages=10, max_pods=8, min_pods=1)
            kube_api = new_deployment_api(rest, "bench", mode, 30 * nat.SECOND, self.clock, busy_poll_ns=busy_poll_ns)
            scaler = new_pod_autoscaler(t, kube_api, log, self.clock)
            sqs_api = new_sqs_api(REGION, self.clock, endpoint=sqs.url, credentials=creds, tls=sqs_tls,
                                  busy_poll_ns=busy_poll_ns)
            client = new_sqs_client(t, sqs_api)
            self.kube_apis.append(kube_api)
            self.sqs_apis.append(sqs_api)
            cfg = nat.LoopConfig()
            cfg.poll_period_ns = 0
            cfg.scale_up_cool_down_ns = 0
            cfg.scale_down_cool_down_ns = 0
            cfg.scale_up_messages = 100
            cfg.scale_down_messages = 10
            cfg.prefetch = pipeline
            self.runners.append(nat.Runner(cfg, client, scaler, self.clock, log))
            self.targets.append(t)

    def run(self, iterations: int) -> float:
        """All workers run ``iterations`` polls concurrently; returns wall seconds."""
        sup = self.nat.Supervisor()
        for r in self.runners:
            sup.add(r)
        t0 = time.perf_counter()
        sup.start(iterations)
        sup.join()
        return time.perf_counter() - t0

    def collect(self, steps: int, wall: float) -> LatencyResult:
        res = LatencyResult(queues=len(self.runners), mode=self.mode, steps=steps, pipeline=self.pipeline, wall_s=wall)
        for r in self.runners:
            res.samples.extend(r.latencies())
        res.sqs_requests = sum(s.requests() for s in self.sqs_servers)
        res.kube_requests = sum(k.requests() for k in self.kube_servers)
        res.sqs_connections = sum(s.connections() for s in self.sqs_servers)
        res.kube_connections = sum(k.connections() for k in self.kube_servers)
        res.signature_failures = sum(s.signature_failures() for s in self.sqs_servers)
        res.final_replicas = [self.kube_servers[si].replicas("bench", t.deployment)
                              for si, t in zip(self.server_of, self.targets)]
        return res

    def clear(self) -> None:
        for r in self.runners:
            r.clear_latencies()

    def close(self) -> None:
        for s in self.sqs_servers:
            s.stop()
        for k in self.kube_servers:
            k.stop()
        if self._devnull is not None:
            os.close(self._devnull)
            self._devnull = None


def phase_breakdown(steps: int = 2000, warmup: int = 200, **kw) -> Dict[str, float]:
    """Median per-phase times (us) of the scaling iteration, from the native span trace.

    ``depth_us`` is the SQS call (the pipelined GET is in flight during it), ``get_wait_us`` the
    extra wait for the GET response afterwards (0 when it arrived during the SQS call),
    ``write_us`` the replica write, ``patch_us`` the poll->patch span the metric reports.
    """
    import json
    import statistics
    import tempfile

    env = BenchEnv(1, **kw)
    try:
        env.run(warmup)
        with tempfile.TemporaryFile() as f:
            env.runners[0].set_trace_fd(f.fileno())
            env.run(steps)
            env.runners[0].set_trace_fd(-1)
            f.seek(0)
            spans = [json.loads(l) for l in f.read().decode().splitlines()]
    finally:
        env.close()
    med = lambda k: round(statistics.median(s[k] for s in spans) / 1e3, 2)
    return {"depth_us": med("depth_ns"), "get_wait_us": med("get_ns"), "write_us": med("update_ns"),
            "patch_us": med("patch_latency_ns")}


def measure(queues: int, steps: int, warmup: int, mode: str = "scale", **kw) -> LatencyResult:
    env = BenchEnv(queues, mode, **kw)
    try:
        if warmup:
            env.run(warmup)
        env.clear()
        wall = env.run(steps)
        return env.collect(steps, wall)
    finally:
        env.close()
