"""Poll -> scale-patch latency benchmark against localhost fake SQS / kube-apiserver servers.

BASELINE.json's metric is the p50 of the time from the end of the poll sleep to the end of the
replica write (``Runner`` records it per iteration, csrc/core/runner.cc), at 1/2/4/8
concurrently tracked queues. Every tracked queue gets its own native worker thread, its own
persistent connections and its own Deployment (``BenchEnv`` documents where the fake endpoints
run).

The wire path is the production one: SigV4-signed ``GetQueueAttributes`` (verified by the
fake), bearer-token kube REST calls with resourceVersion preconditions, real attribute summing
and clamp arithmetic, info-level logrus lines written to a file descriptor.

Two paths are measured: the optimised default (``/scale`` subresource + pipelined read: the
Deployment GET overlaps the SQS call) and the reference-equivalent one (full-object GET+PUT,
strictly sequential -- what /root/reference/scale/scale.go:54-107 does after sqs.go:51).

Trace: the fake serves the BASELINE.json "step trace" 200 -> 0 -> 200 ... one value per poll,
with scale-up-messages=100 / scale-down-messages=10, min 1 / max 8 and zero cool-downs, so
*every* iteration performs SQS + GET + write (the 3-round-trip scaling path of SURVEY.md §3.2)
-- the path whose latency the metric names. ``measure`` polls back to back (the hot loop);
``measure_cadenced`` polls at a production ``--poll-period``.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..autoscaler import DEFAULT_SPIN_BUDGET_PPM, new_deployment_api, new_pod_autoscaler, new_sqs_api, new_sqs_client
from ..config import TargetConfig
from ..kube.config import RestConfig
from ..ops import fakes, native
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


HIGH = {"ApproximateNumberOfMessages": "150", "ApproximateNumberOfMessagesDelayed": "20",
        "ApproximateNumberOfMessagesNotVisible": "30"}
LOW = {"ApproximateNumberOfMessages": "0", "ApproximateNumberOfMessagesDelayed": "0",
       "ApproximateNumberOfMessagesNotVisible": "0"}


def start_fake_endpoints(queues: int, n_servers: int, tls: bool = False, sqs_latency_ns: int = 0,
                         kube_latency_ns: int = 0, cpus: Optional[List[List[int]]] = None, offset: int = 0,
                         hot: bool = False, timing: bool = False, only: str = "both"):
    """``n_servers`` fake SQS + apiserver pairs serving ``queues`` bench queues numbered from
    ``offset`` (queue offset+q on pair q % n_servers): the 200 <-> 0 attribute cycle per queue
    and one Deployment per queue. ``cpus[i]``: the CPUs pair i's threads run on (None: unpinned).
    ``hot``: each server is one busy-polling thread that never sleeps (HttpServer::set_hot).
    ``timing``: the servers record each request's wake-up delay and service time
    (HttpServer::set_timing; off by default, it adds two syscalls per request). ``only``:
    ``sqs`` or ``kube`` starts that kind alone (the other list comes back empty)."""
    if only not in ("both", "sqs", "kube"):
        raise ValueError(f"only must be both, sqs or kube, not {only!r}")
    fk = fakes()
    sqs_servers, kube_servers = [], []
    for i in range(n_servers):
        servers = []
        if only in ("both", "sqs"):
            sqs = fk.FakeSqsServer()
            sqs.require_signature(AKID, SECRET, REGION)
            servers.append((sqs, sqs_latency_ns))
            sqs_servers.append(sqs)
        if only in ("both", "kube"):
            kube = fk.FakeKubeServer()
            kube.require_token(TOKEN)
            servers.append((kube, kube_latency_ns))
            kube_servers.append(kube)
        for srv, latency in servers:
            if cpus is not None:
                srv.set_cpus(cpus[i])
            srv.set_hot(hot)
            srv.set_timing(timing)
            srv.start("127.0.0.1", 0, tls)
            srv.set_latency(latency)
    for q in range(queues):
        si = q % n_servers
        if sqs_servers:
            sqs_servers[si].set_attribute_cycle(queue_url(sqs_servers[si].url, offset + q), [HIGH, LOW])
        if kube_servers:
            kube_servers[si].add_deployment("bench", deployment_name(offset + q), 1)
    return sqs_servers, kube_servers


def thread_count(pid: str = "self") -> int:
    """Threads of a process (/proc/<pid>/status), 0 when unknown."""
    try:
        with open(f"/proc/{pid}/status") as f:
            for line in f:
                if line.startswith("Threads:"):
                    return int(line.split()[1])
    except OSError:
        pass
    return 0


def queue_url(sqs_url: str, q: int) -> str:
    return f"{sqs_url}/000000000000/bench-queue-{q}"


def deployment_name(q: int) -> str:
    return f"gpu-worker-{q}"


class _Endpoint:
    """Parent-side view of one fake server living in the endpoint process."""

    def __init__(self, url: str, cert_pem: str):
        self.url, self.cert_pem = url, cert_pem


class RemoteEndpoints:
    """The fake endpoints in a child process (``python -m kube_sqs_autoscaler_amd.bench.fakeserve``):
    what an autoscaler sees in production, where SQS and the apiserver are other machines'
    processes -- their threads do not share the autoscaler's process, allocator or CPU share."""

    def __init__(self, queues: int, n_servers: int, tls: bool, sqs_latency_ns: int, kube_latency_ns: int,
                 cpus: Optional[List[List[int]]] = None, offset: int = 0, hot: bool = False,
                 timing: bool = False, only: str = "both"):
        import json
        import subprocess
        import sys

        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        extra = ((["--cpus", json.dumps(cpus)] if cpus is not None else []) + (["--hot"] if hot else [])
                 + (["--timing"] if timing else []))
        self.proc = subprocess.Popen(
            [sys.executable, "-m", "kube_sqs_autoscaler_amd.bench.fakeserve", "--queues", str(queues), "--pairs",
             str(n_servers), "--tls", str(int(tls)), "--sqs-latency-ns", str(sqs_latency_ns), "--kube-latency-ns",
             str(kube_latency_ns), "--queue-offset", str(offset), "--only", only, *extra], cwd=root, stdin=subprocess.PIPE,
            stdout=subprocess.PIPE, text=True)
        line = self.proc.stdout.readline()
        if not line:
            raise RuntimeError("fake endpoint process failed to start")
        info = json.loads(line)
        self.sqs = [_Endpoint(e["url"], e["cert_pem"]) for e in info["sqs"]]
        self.kube = [_Endpoint(e["url"], e["cert_pem"]) for e in info["kube"]]
        self.pid = info["pid"]

    def stats(self) -> dict:
        import json

        self.proc.stdin.write("stats\n")
        self.proc.stdin.flush()
        return json.loads(self.proc.stdout.readline())

    def timings(self) -> dict:
        """{"sqs": [(wake_ns, service_ns), ...], "kube": [...]}, then cleared (fakeserve)."""
        import json

        self.proc.stdin.write("timings\n")
        self.proc.stdin.flush()
        return json.loads(self.proc.stdout.readline())

    def close(self) -> None:
        if self.proc.poll() is None:
            try:
                self.proc.stdin.write("quit\n")
                self.proc.stdin.flush()
                self.proc.wait(timeout=10)
            except Exception:
                self.proc.kill()
                self.proc.wait()


class BenchEnv:
    """Fake servers + one worker per queue.

    ``servers``: ``shared`` -- one fake SQS + apiserver pair in this process for every queue;
    ``per-queue`` -- one pair per queue, in this process; ``process`` -- one pair serving every
    queue, in an endpoint process of its own; ``split`` -- production's shape: one fake SQS
    serving every queue in an endpoint process of its own and one apiserver in another (SQS and
    the apiserver are different machines' processes, so the pipelined GET and the SQS request of
    a poll are not served by one process's threads); ``processes`` -- one endpoint process per
    queue (as separate ranks see it: no two queues' endpoint threads share a process).

    ``poll_period_ns``: every queue's ``--poll-period`` (0: back to back, the hot loop);
    ``stagger``: queue i of N starts i/N of a poll period late (Supervisor.stagger), so N
    queues at one cadence do not poll in one burst. ``hot_endpoints``: every fake server is one
    busy-polling thread (HttpServer::set_hot), awake whenever a request arrives, as a loaded
    production endpoint is (supported with ``shared``, ``process`` and ``split``). ``prewarm_ns``: the
    loop's pre-poll warm-up (``--poll-prewarm``); ``spin_budget_ppm``: the share of the poll
    period a worker may spin beyond the --busy-poll window (LoopConfig; None: the CLI's default,
    ``--busy-poll-budget=0``);
    ``presend``: stage each poll's SQS request during the warm-up (LoopConfig.presend; the CLI's
    --poll-presend, off by default); ``prewarm_spin``: spin to the due time after the warm-up for
    a near endpoint (LoopConfig.prewarm_spin);
    these, ``busy_poll_ns``, ``mode`` and ``pipeline`` may be lists, one value per queue, cycled
    (paired comparisons within one run: :func:`measure_cadenced_arms`). ``timing``: the clients time every request's
    phases (HttpTiming), traced polls carry the breakdown (``detail``), and the fakes record each
    request's wake-up delay and service time (HttpServer::set_timing)."""

    def __init__(self, queues: int, mode: str = "scale", tls: bool = False, sqs_latency_ns: int = 0,
                 kube_latency_ns: int = 0, log_fd: Optional[int] = None, pipeline: bool = True,
                 busy_poll_ns: int = 0, servers: str = "shared", log_level: str = "info", sqs_protocol: str = "query",
                 poll_period_ns: int = 0, stagger: bool = False, hot_endpoints: bool = False, prewarm_ns: int = 0,
                 timing: bool = False, spin_budget_ppm=None, presend=False, prewarm_spin=True):
        nat = native()
        self.nat = nat
        self.mode = mode
        self.pipeline = pipeline
        self.stagger = stagger
        n_servers = queues if servers in ("per-queue", "processes") else 1
        self.remote = None
        self.remotes = []
        if servers == "process":
            self.remote = RemoteEndpoints(queues, 1, tls, sqs_latency_ns, kube_latency_ns, hot=hot_endpoints,
                                          timing=timing)
            self.remotes = [self.remote]
            self.sqs_servers, self.kube_servers = self.remote.sqs, self.remote.kube
        elif servers == "split":
            self.remotes = [RemoteEndpoints(queues, 1, tls, sqs_latency_ns, kube_latency_ns, hot=hot_endpoints,
                                            timing=timing, only=kind) for kind in ("sqs", "kube")]
            self.remote = self.remotes[0]
            self.sqs_servers, self.kube_servers = self.remotes[0].sqs, self.remotes[1].kube
        elif servers == "processes":
            self.remotes = [RemoteEndpoints(1, 1, tls, sqs_latency_ns, kube_latency_ns, offset=q, timing=timing)
                            for q in range(queues)]
            self.remote = self.remotes[0]
            self.sqs_servers = [r.sqs[0] for r in self.remotes]
            self.kube_servers = [r.kube[0] for r in self.remotes]
        elif servers in ("shared", "per-queue"):
            self.sqs_servers, self.kube_servers = start_fake_endpoints(queues, n_servers, tls, sqs_latency_ns,
                                                                       kube_latency_ns, hot=hot_endpoints,
                                                                       timing=timing)
        else:
            raise ValueError(f"servers must be shared, per-queue, process, split or processes, not {servers!r}")
        self.sqs, self.kube = self.sqs_servers[0], self.kube_servers[0]
        self.clock = nat.RealClock()
        # one logger writing to one file, like the reference's global logrus logger
        self._devnulls = []
        fd = log_fd
        if fd is None:
            fd = os.open(os.devnull, os.O_WRONLY)
            self._devnulls.append(fd)
        self.log = nat.Logger()
        self.log.set_sink_fd(fd)
        self.log.set_level(log_level)
        creds = static_provider(AKID, SECRET)
        self.runners = []
        self.kube_apis, self.sqs_apis = [], []
        self.targets = []
        self.server_of = []  # queue -> index of the server pair that serves it
        per_queue = lambda v, q: v[q % len(v)] if isinstance(v, (list, tuple)) else v  # noqa: E731
        for q in range(queues):
            si = q % n_servers
            sqs, kube = self.sqs_servers[si], self.kube_servers[si]
            bp_q, pw_q = per_queue(busy_poll_ns, q), per_queue(prewarm_ns, q)
            mode_q, pipeline_q = per_queue(mode, q), per_queue(pipeline, q)
            rest = RestConfig(host=kube.url, bearer_token=TOKEN, insecure=tls)
            sqs_tls = None
            if tls:
                sqs_tls = nat.TlsOptions()
                sqs_tls.ca_pem = sqs.cert_pem
                rest.insecure = False
                rest.ca_pem = kube.cert_pem
            t = TargetConfig(queue_url=queue_url(sqs.url, q), deployment=deployment_name(q), namespace="bench",
                             poll_period_ns=poll_period_ns, scale_up_cool_down_ns=0, scale_down_cool_down_ns=0,
                             scale_up_messages=100, scale_down_messages=10, max_pods=8, min_pods=1)
            kube_api = new_deployment_api(rest, "bench", mode_q, 30 * nat.SECOND, self.clock, busy_poll_ns=bp_q)
            scaler = new_pod_autoscaler(t, kube_api, self.log, self.clock)
            sqs_api = new_sqs_api(REGION, self.clock, endpoint=sqs.url, protocol=sqs_protocol, credentials=creds,
                                  tls=sqs_tls, busy_poll_ns=bp_q)
            if timing:
                sqs_api.set_timing(True)
                kube_api.set_timing(True)
            cfg = nat.LoopConfig()
            cfg.poll_period_ns = poll_period_ns
            cfg.scale_up_cool_down_ns = 0
            cfg.scale_down_cool_down_ns = 0
            cfg.scale_up_messages = 100
            cfg.scale_down_messages = 10
            cfg.prefetch = pipeline_q
            cfg.prewarm_ns = pw_q
            cfg.presend = per_queue(presend, q)
            cfg.prewarm_spin = per_queue(prewarm_spin, q)
            # the CLI's share (autoscaler.loop_config) unless given
            cfg.spin_budget_ppm = (DEFAULT_SPIN_BUDGET_PPM // queues if spin_budget_ppm is None
                                   else per_queue(spin_budget_ppm, q))
            # connect both clients when the worker starts, on its own thread (as --poll-prewarm
            # does before a poll): the on-wire GET never dials, and a dial from this thread would
            # put every worker's connection state in this thread's allocator arena, side by side
            cfg.connect_at_start = True
            self.server_of.append(si)
            self.kube_apis.append(kube_api)
            self.sqs_apis.append(sqs_api)
            self.runners.append(nat.Runner(cfg, new_sqs_client(t, sqs_api), scaler, self.clock, self.log))
            self.targets.append(t)

    def run(self, iterations: int) -> float:
        """All workers run ``iterations`` polls concurrently; returns wall seconds."""
        sup = self.nat.Supervisor()
        sup.stagger = self.stagger
        for r in self.runners:
            sup.add(r)
        t0 = time.perf_counter()
        sup.start(iterations)
        sup.join()
        wall = time.perf_counter() - t0
        self.last_thread_sched = dict(sup.thread_sched())  # the worker threads, as they exited
        return wall

    def collect(self, steps: int, wall: float) -> LatencyResult:
        res = LatencyResult(queues=len(self.runners), mode=self.mode, steps=steps, pipeline=self.pipeline, wall_s=wall)
        for r in self.runners:
            res.samples.extend(r.latencies())
        if self.remotes:
            for rem in self.remotes:
                st = rem.stats()
                res.sqs_requests += st["sqs_requests"]
                res.kube_requests += st["kube_requests"]
                res.sqs_connections += st["sqs_connections"]
                res.kube_connections += st["kube_connections"]
                res.signature_failures += st["signature_failures"]
                res.final_replicas += st["replicas"]
            return res
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

    def server_timings(self) -> dict:
        """Every fake endpoint's per-request (wake-up delay, service time), then cleared."""
        if self.remotes:
            out = {"sqs": [], "kube": []}
            for rem in self.remotes:
                t = rem.timings()
                out["sqs"] += t["sqs"]
                out["kube"] += t["kube"]
            return out
        out = {"sqs": [t for x in self.sqs_servers for t in x.timings()],
               "kube": [t for x in self.kube_servers for t in x.timings()]}
        for x in (*self.sqs_servers, *self.kube_servers):
            x.clear_timings()
        return out

    def close(self) -> None:
        if self.remotes:
            for rem in self.remotes:
                rem.close()
        else:
            for s in self.sqs_servers:
                s.stop()
            for k in self.kube_servers:
                k.stop()
        for fd in self._devnulls:
            os.close(fd)
        self._devnulls = []


def phase_breakdown(steps: int = 2000, warmup: int = 200, timing: bool = False, **kw) -> Dict[str, float]:
    """Median per-phase times (us) of the scaling iteration, from the native span trace.

    ``depth_us`` is the SQS call (the pipelined GET is in flight during it), ``get_wait_us`` the
    extra wait for the GET response afterwards (0 when it arrived during the SQS call),
    ``write_us`` the replica write, ``patch_us`` the poll->patch span the metric reports.
    ``timing``: also every call's phases (HttpTiming), under ``calls``.
    """
    import json
    import statistics
    import tempfile

    env = BenchEnv(1, timing=timing, **kw)
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
    out = {"depth_us": med("depth_ns"), "get_wait_us": med("get_ns"), "write_us": med("update_ns"),
           "patch_us": med("patch_latency_ns")}
    if timing:
        out["calls"] = _detail_medians([s for s in spans if s["patch_latency_ns"] >= 0])
    return out


def measure_processes(queues: int, steps: int, warmup: int, mode: str = "scale", tls: bool = False,
                      pipeline: bool = True, busy_poll_ns: int = 0, sqs_latency_ns: int = 0, kube_latency_ns: int = 0,
                      log_level: str = "info", **_ignored) -> LatencyResult:
    """``measure`` with every queue in a worker process of its own (``--worker-processes``,
    parallel/procfleet.py) against one endpoint process per queue. Each worker runs
    ``warmup + steps`` polls back to back and the last ``steps`` latencies of each are kept."""
    from ..parallel.procfleet import ProcessFleet

    nat = native()
    remotes = [RemoteEndpoints(1, 1, tls, sqs_latency_ns, kube_latency_ns, offset=q) for q in range(queues)]
    creds = static_provider(AKID, SECRET)
    targets = []
    for q in range(queues):
        targets.append(TargetConfig(queue_url=queue_url(remotes[q].sqs[0].url, q), deployment=deployment_name(q),
                                    namespace="bench", poll_period_ns=0, scale_up_cool_down_ns=0,
                                    scale_down_cool_down_ns=0, scale_up_messages=100, scale_down_messages=10,
                                    max_pods=8, min_pods=1))

    def build(q):
        def make():
            clock = nat.RealClock()
            fd = os.open(os.devnull, os.O_WRONLY)
            log = nat.Logger()
            log.set_sink_fd(fd)
            log.set_level(log_level)
            sqs_ep, kube_ep = remotes[q].sqs[0], remotes[q].kube[0]
            rest = RestConfig(host=kube_ep.url, bearer_token=TOKEN, insecure=tls)
            sqs_tls = None
            if tls:
                sqs_tls = nat.TlsOptions()
                sqs_tls.ca_pem = sqs_ep.cert_pem
                rest.insecure = False
                rest.ca_pem = kube_ep.cert_pem
            t = targets[q]
            kube_api = new_deployment_api(rest, "bench", mode, 30 * nat.SECOND, clock, busy_poll_ns=busy_poll_ns)
            scaler = new_pod_autoscaler(t, kube_api, log, clock)
            sqs_api = new_sqs_api(REGION, clock, endpoint=sqs_ep.url, credentials=creds, tls=sqs_tls,
                                  busy_poll_ns=busy_poll_ns)
            cfg = nat.LoopConfig()
            cfg.poll_period_ns = cfg.scale_up_cool_down_ns = cfg.scale_down_cool_down_ns = 0
            cfg.scale_up_messages, cfg.scale_down_messages = 100, 10
            cfg.prefetch = pipeline

            class W:
                runner = nat.Runner(cfg, new_sqs_client(t, sqs_api), scaler, clock, log)
            return W
        return make

    fleet = None
    try:
        fleet = ProcessFleet([build(q) for q in range(queues)], targets)
        fleet.wait_ready()
        t0 = time.perf_counter()
        fleet.start(warmup + steps)
        fleet.join()
        wall = time.perf_counter() - t0
        if any(c != 0 for c in fleet.exit_codes()):
            raise RuntimeError(f"bench worker process failed: exit codes {fleet.exit_codes()}")
        res = LatencyResult(queues=queues, mode=mode, steps=steps, pipeline=pipeline, wall_s=wall)
        for w in fleet.workers:
            res.samples.extend(w.runner.latencies()[-steps:])
        for rem in remotes:
            st = rem.stats()
            res.sqs_requests += st["sqs_requests"]
            res.kube_requests += st["kube_requests"]
            res.sqs_connections += st["sqs_connections"]
            res.kube_connections += st["kube_connections"]
            res.signature_failures += st["signature_failures"]
            res.final_replicas += st["replicas"]
        return res
    finally:
        if fleet is not None:
            fleet.close()
        for rem in remotes:
            rem.close()


def measure(queues: int, steps: int, warmup: int, mode: str = "scale", workers: str = "threads",
            **kw) -> LatencyResult:
    """``workers``: ``threads`` (one process, a thread per queue) or ``processes`` (a worker
    process per queue, ``measure_processes``)."""
    if workers == "processes":
        return measure_processes(queues, steps, warmup, mode, **kw)
    env = BenchEnv(queues, mode, **kw)
    try:
        if warmup:
            env.run(warmup)
        env.clear()
        wall = env.run(steps)
        return env.collect(steps, wall)
    finally:
        env.close()


def _pct_ns(v: List[int], p: float) -> int:
    import math

    v = sorted(v)
    k = max(1, math.ceil(p / 100.0 * len(v)))
    return v[min(k, len(v)) - 1]


def measure_cadenced(poll_period_ns: int, polls: int, queues: int = 16, mode: str = "scale", pipeline: bool = True,
                     busy_poll_ns: int = 0, tls: bool = False, skip: int = 2, servers: str = "split",
                     hot_endpoints: bool = False, prewarm_ns: int = 0, timing: bool = False) -> Dict:
    """Poll -> patch latency at a production poll cadence, not back to back: one path
    (:func:`measure_cadenced_arms` with a single arm; see there)."""
    arm = dict(mode=mode, pipeline=pipeline, busy_poll_ns=busy_poll_ns, prewarm_ns=prewarm_ns)
    return measure_cadenced_arms(poll_period_ns, polls, queues, {"only": arm}, tls, skip, servers, hot_endpoints,
                                 timing)["only"]


def measure_cadenced_arms(poll_period_ns: int, polls: int, queues_per_arm: int, arms: Dict[str, Dict],
                          tls: bool = False, skip: int = 2, servers: str = "split", hot_endpoints: bool = False,
                          timing: bool = False, sqs_latency_ns: int = 0, kube_latency_ns: int = 0,
                          keep_samples: bool = False) -> Dict[str, Dict]:
    """Poll -> patch latency at a production poll cadence for one or more paths side by side.

    The reference sleeps ``--poll-period`` (5 s by default) before every poll
    (/root/reference/main.go:41,83). Between polls the worker thread is asleep, its caches and
    branch predictors are cold, the CPU may sit in a deep idle state, and a keep-alive
    connection unused for longer than ``kFreshConnNs`` gets the idle-close check again. The
    hot-loop rows measure none of that. Here every arm (``name -> dict(mode, pipeline,
    busy_poll_ns, prewarm_ns[, presend, prewarm_spin, spin_budget_ppm])``) gets ``queues_per_arm`` queues; queue q runs arm q % len(arms),
    so the arms' queues interleave in one fleet (a thread each, starts staggered over the
    period) and run ``polls`` polls at ``poll_period_ns`` in the same run, against the same
    ``split`` endpoints (one fake SQS process and one apiserver process serving every queue, as
    production has two services). Comparing paths in one run, not in runs one after the other,
    matters at a cadence: a box's idle-state and frequency behaviour drifts over tens of seconds
    and moved single-path runs of the same path by 2x between consecutive runs
    (profiles/r04c_cadence_probe.jsonl). Every poll scales (the 200/0 trace, zero cool-downs).
    The first ``skip`` polls of each queue (dial, TLS handshake, first allocations) are dropped.
    Phases come from the per-poll spans (``--trace-file`` format), and so does each poll's CPU time
    on the worker thread (``cpu_ns``: warm-up, its spin, busy-polling and the poll itself), reported
    per arm as ``cpu_ms_per_poll``. ``sqs_latency_ns`` / ``kube_latency_ns``: the fakes answer that
    much later (a regional round trip). ``setup`` records what the run had: the CPUs this process
    may use, its threads, and with endpoint processes their threads and CPU per request served.
    ``keep_samples``: each arm also returns its raw ``latencies_ns`` and ``cpu_ns`` (one per kept
    poll), so a caller can pool several runs.
    """
    import json
    import statistics
    import tempfile

    names = list(arms)
    n = len(names)
    col = lambda k, default=None: [arms[a].get(k, default) for a in names]  # noqa: E731 -- cycled per queue
    # each arm's queues get the spin budget the CLI gives a process tracking that many queues
    # (--busy-poll-budget shared by them), not a share diluted by the other arms' queues
    env = BenchEnv(queues_per_arm * n, col("mode"), tls=tls, pipeline=col("pipeline"),
                   busy_poll_ns=col("busy_poll_ns"), servers=servers, poll_period_ns=poll_period_ns, stagger=True,
                   hot_endpoints=hot_endpoints, prewarm_ns=col("prewarm_ns"), timing=timing,
                   spin_budget_ppm=col("spin_budget_ppm", DEFAULT_SPIN_BUDGET_PPM // queues_per_arm),
                   presend=col("presend", False), prewarm_spin=col("prewarm_spin", True),
                   sqs_latency_ns=sqs_latency_ns, kube_latency_ns=kube_latency_ns)
    files = [tempfile.TemporaryFile() for _ in env.runners]
    spans: Dict[str, List[dict]] = {a: [] for a in names}
    quota, quota_period = env.nat.read_cpu_quota()
    # the CPUs this process may run on, and the cgroup's CPU bandwidth (cores' worth; None: no limit)
    setup = {"cpus_available": len(os.sched_getaffinity(0)),
             "cpu_quota_cores": round(quota / quota_period, 2) if quota else None}
    try:
        for r, f in zip(env.runners, files):
            r.set_trace_fd(f.fileno())
        before = [rem.stats() for rem in env.remotes]
        wall = env.run(polls)
        after = [rem.stats() for rem in env.remotes]
        setup["autoscaler_threads"] = thread_count()
        if after:
            setup["endpoint_threads"] = [s.get("threads", 0) for s in after]
            # (hot endpoints busy-poll: their CPU is the whole run's, not per request)
            setup["endpoint_cpu_us_per_request"] = None if hot_endpoints else [
                round((a["cpu_ns"] - b["cpu_ns"]) / 1e3 / max(1, a["sqs_requests"] + a["kube_requests"]
                                                              - b["sqs_requests"] - b["kube_requests"]), 2)
                for a, b in zip(after, before)]
        for q, (r, f) in enumerate(zip(env.runners, files)):
            r.set_trace_fd(-1)
            f.seek(0)
            spans[names[q % n]] += [json.loads(line) for line in f.read().decode().splitlines()][skip:]
        res = env.collect(polls, wall)
        served = env.server_timings()
    finally:
        for f in files:
            f.close()
        env.close()
    out = {}
    for a in names:
        lat = [s["patch_latency_ns"] for s in spans[a] if s["patch_latency_ns"] >= 0]
        scaled = [s for s in spans[a] if s["patch_latency_ns"] >= 0]
        med = (lambda k: round(statistics.median(s[k] for s in scaled) / 1e3, 2)) if scaled else (lambda k: None)
        arm = arms[a]
        out[a] = {
            "poll_period_ms": poll_period_ns / 1e6,
            "queues": queues_per_arm,
            **({"paired_with": [b for b in names if b != a], "queues_in_run": queues_per_arm * n} if n > 1 else {}),
            "mode": arm["mode"],
            "pipeline_reads": arm["pipeline"],
            "tls": tls,
            "hot_endpoints": hot_endpoints,
            "prewarm_us": arm["prewarm_ns"] / 1e3,
            "p50_ms": round(_pct_ns(lat, 50) / 1e6, 4) if lat else None,
            "p90_ms": round(_pct_ns(lat, 90) / 1e6, 4) if lat else None,
            "p99_ms": round(_pct_ns(lat, 99) / 1e6, 4) if lat else None,
            "samples": len(lat),
            "polls": len(spans[a]),
            "errors": sum(1 for s in spans[a] if "error" in s),
            "signature_failures": res.signature_failures,
            "phase_median_us": {"depth_us": med("depth_ns"), "get_wait_us": med("get_ns"), "write_us": med("update_ns"),
                                "patch_us": med("patch_latency_ns")},
            "wall_s": round(wall, 2),
            **_cpu_per_poll(spans[a]),
            "setup": setup,
            **({"latencies_ns": lat, "cpu_ns": [s["cpu_ns"] for s in spans[a] if s.get("cpu_ns", -1) >= 0]}
               if keep_samples else {}),
            # With timing: every client call's phases, and the fake endpoints' side of each
            # request (HttpServer::timings, all arms together) -- how long the endpoint's thread
            # took to wake up for it after the kernel received it, and to answer it.
            **({"endpoint_median_us": {k: {"wake": _median_us([w for w, _ in v]),
                                           "service": _median_us([sv for _, sv in v])} for k, v in served.items()},
                "call_phase_median_us": _detail_medians(scaled)} if timing else {}),
        }
    return out


def _cpu_per_poll(spans: List[dict]) -> Dict:
    """The worker thread's CPU per poll (span ``cpu_ns``): mean and median, milliseconds."""
    import statistics

    cpu = [s["cpu_ns"] for s in spans if s.get("cpu_ns", -1) >= 0]
    if not cpu:
        return {}
    return {"cpu_ms_per_poll": round(sum(cpu) / len(cpu) / 1e6, 4),
            "cpu_ms_per_poll_p50": round(statistics.median(cpu) / 1e6, 4)}


def _detail_medians(spans: List[dict]) -> Dict:
    """Medians (us) of the per-call phases in the spans' ``detail`` (HttpTiming): for the SQS
    call sign / pre (connection check, serialisation) / write / wait (until the kernel received
    the answer) / wake (until this thread read it) / read / parse, and the same HTTP phases for
    the replica write; ``spun``: the share of calls whose answer came while busy-polling."""
    out: Dict[str, Dict] = {}
    for call in ("sqs", "write"):
        rows = [s["detail"][call] for s in spans if s.get("detail") and s["detail"].get(call)]
        if not rows:
            continue
        d = {k: _median_us([r[k] for r in rows if r.get(k, -1) >= 0])
             for k in ("sign", "pre", "write", "wait", "wake", "read", "parse") if k in rows[0]}
        d["spun_share"] = round(sum(1 for r in rows if r.get("spun")) / len(rows), 3)
        out[call] = d
    return out


def _median_us(v: List[int]):
    import statistics

    return round(statistics.median(v) / 1e3, 2) if v else None
