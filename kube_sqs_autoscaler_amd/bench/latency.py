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


HIGH = {"ApproximateNumberOfMessages": "150", "ApproximateNumberOfMessagesDelayed": "20",
        "ApproximateNumberOfMessagesNotVisible": "30"}
LOW = {"ApproximateNumberOfMessages": "0", "ApproximateNumberOfMessagesDelayed": "0",
       "ApproximateNumberOfMessagesNotVisible": "0"}


def start_fake_endpoints(nat, queues: int, n_servers: int, tls: bool = False, sqs_latency_ns: int = 0,
                         kube_latency_ns: int = 0, cpus: Optional[List[List[int]]] = None, offset: int = 0):
    """``n_servers`` fake SQS + apiserver pairs serving ``queues`` bench queues numbered from
    ``offset`` (queue offset+q on pair q % n_servers): the 200 <-> 0 attribute cycle per queue
    and one Deployment per queue. ``cpus[i]``: the CPUs pair i's threads run on (None: unpinned)."""
    sqs_servers, kube_servers = [], []
    for i in range(n_servers):
        sqs = nat.FakeSqsServer()
        sqs.require_signature(AKID, SECRET, REGION)
        kube = nat.FakeKubeServer()
        kube.require_token(TOKEN)
        if cpus is not None:
            sqs.set_cpus(cpus[i])
            kube.set_cpus(cpus[i])
        sqs.start("127.0.0.1", 0, tls)
        sqs.set_latency(sqs_latency_ns)
        kube.start("127.0.0.1", 0, tls)
        kube.set_latency(kube_latency_ns)
        sqs_servers.append(sqs)
        kube_servers.append(kube)
    for q in range(queues):
        si = q % n_servers
        sqs_servers[si].set_attribute_cycle(queue_url(sqs_servers[si].url, offset + q), [HIGH, LOW])
        kube_servers[si].add_deployment("bench", deployment_name(offset + q), 1)
    return sqs_servers, kube_servers


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
                 cpus: Optional[List[List[int]]] = None, offset: int = 0):
        import json
        import subprocess
        import sys

        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        extra = ["--cpus", json.dumps(cpus)] if cpus is not None else []
        self.proc = subprocess.Popen(
            [sys.executable, "-m", "kube_sqs_autoscaler_amd.bench.fakeserve", "--queues", str(queues), "--pairs",
             str(n_servers), "--tls", str(int(tls)), "--sqs-latency-ns", str(sqs_latency_ns), "--kube-latency-ns",
             str(kube_latency_ns), "--queue-offset", str(offset), *extra], cwd=root, stdin=subprocess.PIPE,
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
    ``per-queue`` -- one pair per queue, in this process; ``process`` -- one pair per queue in a
    separate endpoint process (as production's remote endpoints); ``processes`` -- one endpoint
    process per queue (as separate ranks see it: no two queues' endpoint threads share a process).

    ``affinity``: ``none`` -- threads float; ``llc`` -- queue q's worker thread and its fake
    endpoint pair are pinned to L3 domain q mod D (utils/topology.py), so each queue's traffic
    stays on one CCD, as a rank per queue would (needs per-queue or process servers).

    Layout probes (profiles/README.md r02l): ``build_on_threads`` builds each queue's objects on a
    thread of its own (separate malloc arenas); ``clock_per_queue`` gives each queue its own
    clock object instead of one shared ``RealClock``."""

    def __init__(self, queues: int, mode: str = "scale", tls: bool = False, sqs_latency_ns: int = 0,
                 kube_latency_ns: int = 0, log_fd: Optional[int] = None, pipeline: bool = True,
                 busy_poll_ns: int = 0, servers: str = "shared", loggers: str = "shared", affinity: str = "none",
                 log_level: str = "info", sqs_protocol: str = "query", build_on_threads: bool = False,
                 clock_per_queue: bool = False):
        nat = native()
        self.nat = nat
        self.mode = mode
        self.pipeline = pipeline
        n_servers = 1 if servers == "shared" else queues
        self.remote = None
        cpus = worker_cpus = None
        if affinity == "llc":
            from ..utils.topology import plan

            cpus = worker_cpus = plan(queues)
            if servers == "shared" and queues > 1:
                raise ValueError("affinity=llc needs per-queue or process servers")
        elif affinity == "ccd":
            from ..utils.topology import plan_queue_ccds

            if servers == "shared" and queues > 1:
                raise ValueError("affinity=ccd needs per-queue or process servers")
            worker_cpus, cpus = plan_queue_ccds(queues)
        elif affinity.startswith("{"):
            # explicit placement (probes): {"workers": [[cpu, ...] per queue], "servers": [...]}
            import json

            spec = json.loads(affinity)
            worker_cpus, cpus = spec.get("workers"), spec.get("servers")
        elif affinity != "none":
            raise ValueError(f"affinity must be none, llc, ccd or a JSON placement, not {affinity!r}")
        self.cpus = cpus
        self.remotes = []
        if servers == "process":
            self.remote = RemoteEndpoints(queues, n_servers, tls, sqs_latency_ns, kube_latency_ns, cpus)
            self.remotes = [self.remote]
            self.sqs_servers, self.kube_servers = self.remote.sqs, self.remote.kube
        elif servers == "processes":
            self.remotes = [RemoteEndpoints(1, 1, tls, sqs_latency_ns, kube_latency_ns,
                                            [cpus[q]] if cpus is not None else None, offset=q) for q in range(queues)]
            self.remote = self.remotes[0]
            self.sqs_servers = [r.sqs[0] for r in self.remotes]
            self.kube_servers = [r.kube[0] for r in self.remotes]
        elif servers in ("shared", "per-queue"):
            self.sqs_servers, self.kube_servers = start_fake_endpoints(nat, queues, n_servers, tls, sqs_latency_ns,
                                                                       kube_latency_ns, cpus)
        else:
            raise ValueError(f"servers must be shared, per-queue, process or processes, not {servers!r}")
        self.sqs, self.kube = self.sqs_servers[0], self.kube_servers[0]
        self.clock = nat.RealClock()
        # loggers="per-queue": a logger and an open file of its own per queue (as one process
        # per queue has); "shared": one logger writing to one file, like the reference's global
        self._devnulls = []
        self.loggers = []
        for _ in range(queues if loggers == "per-queue" else 1):
            fd = log_fd
            if fd is None:
                fd = os.open(os.devnull, os.O_WRONLY)
                self._devnulls.append(fd)
            lg = nat.Logger()
            lg.set_sink_fd(fd)
            lg.set_level(log_level)
            self.loggers.append(lg)
        self.log = self.loggers[0]
        creds = static_provider(AKID, SECRET)
        self.runners = []
        self.kube_apis, self.sqs_apis = [], []
        self.targets = []
        self.server_of = []  # queue -> index of the server pair that serves it
        built = [None] * queues

        def build(q):
            si = q % n_servers
            sqs, kube, log = self.sqs_servers[si], self.kube_servers[si], self.loggers[q % len(self.loggers)]
            clock = nat.RealClock() if clock_per_queue else self.clock
            rest = RestConfig(host=kube.url, bearer_token=TOKEN, insecure=tls)
            sqs_tls = None
            if tls:
                sqs_tls = nat.TlsOptions()
                sqs_tls.ca_pem = sqs.cert_pem
                rest.insecure = False
                rest.ca_pem = kube.cert_pem
            url = queue_url(sqs.url, q)
            name = deployment_name(q)
            t = TargetConfig(queue_url=url, deployment=name, namespace="bench", poll_period_ns=0,
                             scale_up_cool_down_ns=0, scale_down_cool_down_ns=0, scale_up_messages=100,
                             scale_down_messages=10, max_pods=8, min_pods=1)
            kube_api = new_deployment_api(rest, "bench", mode, 30 * nat.SECOND, clock, busy_poll_ns=busy_poll_ns)
            scaler = new_pod_autoscaler(t, kube_api, log, clock)
            sqs_api = new_sqs_api(REGION, clock, endpoint=sqs.url, protocol=sqs_protocol, credentials=creds, tls=sqs_tls,
                                  busy_poll_ns=busy_poll_ns)
            client = new_sqs_client(t, sqs_api)
            cfg = nat.LoopConfig()
            cfg.poll_period_ns = 0
            cfg.scale_up_cool_down_ns = 0
            cfg.scale_down_cool_down_ns = 0
            cfg.scale_up_messages = 100
            cfg.scale_down_messages = 10
            cfg.prefetch = pipeline
            runner = nat.Runner(cfg, client, scaler, clock, log)
            if worker_cpus is not None:
                runner.cpus = worker_cpus[q]
            built[q] = (si, kube_api, sqs_api, runner, t)

        if build_on_threads and queues > 1:
            # each queue's objects built on a thread of its own, all alive together, so every
            # queue's heap allocations come from a separate malloc arena (scripts/arena_probe.py)
            import threading

            done = threading.Barrier(queues)

            def build_on_thread(q):
                build(q)
                done.wait()

            ts = [threading.Thread(target=build_on_thread, args=(q,)) for q in range(queues)]
            for th in ts:
                th.start()
            for th in ts:
                th.join()
        else:
            for q in range(queues):
                build(q)
        for si, kube_api, sqs_api, runner, t in built:
            self.server_of.append(si)
            self.kube_apis.append(kube_api)
            self.sqs_apis.append(sqs_api)
            self.runners.append(runner)
            self.targets.append(t)

    def run(self, iterations: int) -> float:
        """All workers run ``iterations`` polls concurrently; returns wall seconds."""
        sup = self.nat.Supervisor()
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


def measure_processes(queues: int, steps: int, warmup: int, mode: str = "scale", tls: bool = False,
                      pipeline: bool = True, busy_poll_ns: int = 0, sqs_latency_ns: int = 0, kube_latency_ns: int = 0,
                      affinity: str = "none", log_level: str = "info", **_ignored) -> LatencyResult:
    """``measure`` with every queue in a worker process of its own (``--worker-processes``,
    parallel/procfleet.py) against one endpoint process per queue. Each worker runs
    ``warmup + steps`` polls back to back and the last ``steps`` latencies of each are kept."""
    from ..parallel.procfleet import ProcessFleet

    nat = native()
    worker_cpus = endpoint_cpus = None
    if affinity == "ccd":
        from ..utils.topology import plan_queue_ccds

        worker_cpus, endpoint_cpus = plan_queue_ccds(queues)
    remotes = [RemoteEndpoints(1, 1, tls, sqs_latency_ns, kube_latency_ns,
                               [endpoint_cpus[q]] if endpoint_cpus is not None else None, offset=q)
               for q in range(queues)]
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
        fleet = ProcessFleet([build(q) for q in range(queues)], targets, worker_cpus)
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


# ---------------------------------------------------------------------------------------------
# Where does multi-queue latency go? Scheduler and kernel evidence around a measurement.


def _task_stats(pid: int) -> Dict[str, Dict[str, int]]:
    """Per thread name (``ksa-worker``, ``ksa-serve``, ...): CPU time, run-queue wait and
    timeslices from /proc/<pid>/task/*/schedstat, and context switches from .../status."""
    out: Dict[str, Dict[str, int]] = {}
    base = f"/proc/{pid}/task"
    try:
        tids = os.listdir(base)
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"{base}/{tid}/comm") as f:
                comm = f.read().strip()
            with open(f"{base}/{tid}/schedstat") as f:
                cpu, wait, slices = (int(x) for x in f.read().split()[:3])
            vol = invol = 0
            with open(f"{base}/{tid}/status") as f:
                for line in f:
                    if line.startswith("voluntary_ctxt_switches"):
                        vol = int(line.split()[1])
                    elif line.startswith("nonvoluntary_ctxt_switches"):
                        invol = int(line.split()[1])
        except (OSError, ValueError):
            continue
        d = out.setdefault(comm, {"threads": 0, "cpu_ns": 0, "runq_wait_ns": 0, "slices": 0, "vol_cs": 0,
                                  "invol_cs": 0})
        d["threads"] += 1
        d["cpu_ns"] += cpu
        d["runq_wait_ns"] += wait
        d["slices"] += slices
        d["vol_cs"] += vol
        d["invol_cs"] += invol
    return out


def _system_stats() -> Dict[str, int]:
    """cgroup v2 CPU throttling and the machine's TLB-shootdown IPIs (best effort)."""
    out: Dict[str, int] = {}
    for path in ("/sys/fs/cgroup/cpu.stat",):
        try:
            with open(path) as f:
                for line in f:
                    k, v = line.split()
                    if k in ("nr_periods", "nr_throttled", "throttled_usec", "usage_usec"):
                        out[k] = int(v)
        except (OSError, ValueError):
            pass
    try:
        with open("/proc/interrupts") as f:
            for line in f:
                name = line.split(":", 1)[0].strip()
                if name in ("TLB", "RES", "CAL"):
                    out[f"irq_{name}"] = sum(int(x) for x in line.split(":", 1)[1].split() if x.isdigit())
    except OSError:
        pass
    return out


def _delta(after, before):
    if isinstance(after, dict):
        return {k: _delta(v, before.get(k, 0 if not isinstance(v, dict) else {})) for k, v in after.items()}
    return after - before


def measure_detailed(queues: int, steps: int, warmup: int, mode: str = "scale", sync=None, **kw) -> Dict:
    """``measure`` plus, for the timed run: per-phase medians over all queues' spans, and the
    scheduler view of every thread group (this process and the endpoint process) per poll.
    ``sync``: called after the warm-up, right before the timed run (a barrier across ranks)."""
    import json
    import statistics
    import tempfile

    env = BenchEnv(queues, mode, **kw)
    try:
        if warmup:
            env.run(warmup)
        env.clear()
        if sync is not None:
            sync()
        pids = {"autoscaler": os.getpid()}
        for i, rem in enumerate(env.remotes):
            pids[f"endpoints{i}" if len(env.remotes) > 1 else "endpoints"] = rem.pid
        # one span file per worker: a shared one would serialise the workers on its file
        # position lock and perturb what is measured
        files = [tempfile.TemporaryFile() for _ in env.runners]
        try:
            for r, f in zip(env.runners, files):
                r.set_trace_fd(f.fileno())
            t_before = {k: _task_stats(p) for k, p in pids.items()}
            s_before = _system_stats()
            wall = env.run(steps)
            s_after = _system_stats()
            t_after = {k: _task_stats(p) for k, p in pids.items()}
            spans = []
            for r, f in zip(env.runners, files):
                r.set_trace_fd(-1)
                f.seek(0)
                spans += [json.loads(line) for line in f.read().decode().splitlines()]
        finally:
            for f in files:
                f.close()
        res = env.collect(steps, wall)
    finally:
        env.close()
    polls = max(1, queues * steps)
    med = lambda k: round(statistics.median(s[k] for s in spans) / 1e3, 2)
    sched = {}
    for proc, groups in t_after.items():
        for comm, d in groups.items():
            b = t_before[proc].get(comm, {})
            dd = _delta(d, b)
            sched[f"{proc}/{comm}"] = {
                "threads": d["threads"],
                "cpu_us_per_poll": round(dd["cpu_ns"] / polls / 1e3, 2),
                "runq_wait_us_per_poll": round(dd["runq_wait_ns"] / polls / 1e3, 3),
                "slices_per_poll": round(dd["slices"] / polls, 3),
                "vol_cs_per_poll": round(dd["vol_cs"] / polls, 3),
                "invol_cs_per_poll": round(dd["invol_cs"] / polls, 4),
            }
    w = env.last_thread_sched
    sched["autoscaler/ksa-worker"] = {
        "threads": w["threads"],
        "cpu_us_per_poll": round(w["cpu_ns"] / polls / 1e3, 2),
        "runq_wait_us_per_poll": round(w["runq_wait_ns"] / polls / 1e3, 3),
        "slices_per_poll": round(w["slices"] / polls, 3),
        "vol_cs_per_poll": round(w["vol_cs"] / polls, 3),
        "invol_cs_per_poll": round(w["invol_cs"] / polls, 4),
        "user_us_per_poll": round(w["utime_ns"] / polls / 1e3, 2),
        "sys_us_per_poll": round(w["stime_ns"] / polls / 1e3, 2),
        "minflt_per_poll": round(w["minflt"] / polls, 4),
    }
    sysd = _delta(s_after, s_before)
    return {"queues": queues, "mode": mode,
            **{k: v for k, v in kw.items() if k in ("servers", "pipeline", "busy_poll_ns", "affinity", "loggers",
                                                    "log_level")},
            "summary": res.summary(), "signature_failures": res.signature_failures,
            "phases_median_us": {"depth_us": med("depth_ns"), "get_wait_us": med("get_ns"), "write_us": med("update_ns"),
                                 "patch_us": med("patch_latency_ns")},
            "sched": sched, "system": sysd, "wall_s": round(wall, 4)}
