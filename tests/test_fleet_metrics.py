"""Multi-queue fleet isolation + Prometheus/health endpoints."""
import urllib.request

import pytest

from kube_sqs_autoscaler_amd.bench.latency import BenchEnv
from kube_sqs_autoscaler_amd.metrics import MetricsServer
from kube_sqs_autoscaler_amd.parallel.fleet import Fleet


class W:
    def __init__(self, runner, target, kube_api=None, sqs_api=None):
        self.runner, self.target = runner, target
        self.kube_api, self.sqs_api = kube_api, sqs_api


def test_fleet_runs_queues_independently(nat):
    env = BenchEnv(4)
    try:
        fleet = Fleet([W(r, t) for r, t in zip(env.runners, env.targets)])
        fleet.start(25)
        assert fleet.wait(30)
        fleet.join()
        stats = fleet.stats()
        assert [s["polls"] for s in stats] == [25] * 4
        # 200/0 alternation: 13 ups, 12 downs each, every one a write
        assert all(s["scale_ups"] == 13 and s["scale_downs"] == 12 for s in stats)
        assert env.sqs.signature_failures() == 0
        assert env.sqs.connections() == 4 and env.kube.connections() == 4  # one per worker
    finally:
        env.close()


def test_fleet_stop_interrupts_sleep(nat):
    env = BenchEnv(2)
    try:
        for r in env.runners:
            pass
        cfg = nat.LoopConfig()
        cfg.poll_period_ns = 3600 * nat.SECOND
        fleet = Fleet([W(nat.Runner(cfg, r.sqs, r.scaler, nat.RealClock(), env.log), t)
                       for r, t in zip(env.runners, env.targets)])
        fleet.start()
        assert not fleet.wait(0.2)
        fleet.stop()
        assert fleet.wait(5)
        fleet.join()
        assert all(s["polls"] == 0 for s in fleet.stats())
    finally:
        env.close()


def test_metrics_endpoints(nat):
    env = BenchEnv(2)
    try:
        fleet = Fleet([W(*a) for a in zip(env.runners, env.targets, env.kube_apis, env.sqs_apis)])
        m = MetricsServer(fleet, "127.0.0.1:0")
        m.start()
        try:
            base = f"http://127.0.0.1:{m.port}"
            with pytest.raises(urllib.error.HTTPError) as e:
                urllib.request.urlopen(base + "/readyz")
            assert e.value.code == 503
            fleet.start(10)
            fleet.join()
            body = urllib.request.urlopen(base + "/metrics").read().decode()
            assert 'ksa_polls_total{deployment="bench/gpu-worker-0"' in body
            assert "ksa_scale_ups_total" in body and "ksa_poll_to_patch_seconds_count" in body
            assert 'ksa_replicas{deployment="bench/gpu-worker-1"' in body
            # API load: every poll sends one speculative GET (pipelined reads) and one SQS call;
            # all 10 polls act on the 200/0 trace, so every speculative read is consumed
            q0 = '{deployment="bench/gpu-worker-0",queue='
            metric = {line.split("{")[0] + ("" if q0 in line else "#other"): float(line.rsplit(" ", 1)[1])
                      for line in body.splitlines() if line.startswith("ksa_") and q0 in line}
            assert metric["ksa_speculative_reads_total"] == 10 == metric["ksa_speculative_reads_used_total"]
            assert metric["ksa_sqs_calls_total"] == 10 and metric["ksa_apiserver_writes_total"] == 10
            assert metric["ksa_apiserver_gets_total"] == 10 and metric["ksa_apiserver_conflicts_total"] == 0
            assert metric["ksa_apiserver_throttled_total"] == 0 and metric["ksa_apiserver_throttle_seconds_total"] == 0
            assert metric["ksa_sqs_throttle_retries_total"] == 0 and metric["ksa_speculative_reads_skipped_total"] == 0
            # transport counters, per client: one keep-alive connection each; the apiserver
            # connection carries the 10 GETs and the 10 writes
            http = {(line.split("{")[0], line.split('client="')[1].split('"')[0]): float(line.rsplit(" ", 1)[1])
                    for line in body.splitlines() if line.startswith("ksa_http_") and 'deployment="bench/gpu-worker-0"' in line}
            assert http[("ksa_http_requests_total", "sqs")] == 10
            assert http[("ksa_http_requests_total", "apiserver")] == 20
            assert http[("ksa_http_connects_total", "sqs")] == 1 == http[("ksa_http_connects_total", "apiserver")]
            # back to back (no poll period): no warm-up, so nothing is staged
            assert http[("ksa_http_presends_total", "sqs")] == 0 == http[("ksa_http_presend_discards_total", "sqs")]
            assert "# TYPE ksa_http_idle_closed_total counter" in body
            # latency histogram: cumulative buckets ending at +Inf == count, same sum as the summary
            buckets = [(line.split('le="')[1].split('"')[0], float(line.rsplit(" ", 1)[1]))
                       for line in body.splitlines()
                       if line.startswith("ksa_poll_to_patch_latency_seconds_bucket")
                       and 'deployment="bench/gpu-worker-0"' in line]
            assert len(buckets) == 20 and buckets[-1] == ("+Inf", 10.0)
            assert all(a[1] <= b[1] for a, b in zip(buckets, buckets[1:]))
            assert metric["ksa_poll_to_patch_latency_seconds_count"] == 10
            assert metric["ksa_poll_to_patch_latency_seconds_sum"] == metric["ksa_poll_to_patch_seconds_sum"] > 0
            # the worker thread's CPU over its 10 polls (runner.h IterationRecord::cpu_ns)
            assert "# TYPE ksa_poll_cpu_seconds_total counter" in body
            assert 0 < metric["ksa_poll_cpu_seconds_total"] < 10 * 0.05
            assert urllib.request.urlopen(base + "/readyz").read() == b"ok"
            assert urllib.request.urlopen(base + "/healthz").status == 200
        finally:
            m.stop()
    finally:
        env.close()


def test_credential_fetches_family(nat):
    """ksa_aws_credential_fetches_total: one sample per region from the process's credential
    sources (cli.py passes the shared providers' or the broker's counts)."""
    from kube_sqs_autoscaler_amd.metrics import FleetCollector
    from kube_sqs_autoscaler_amd.parallel.fleet import Fleet

    body = FleetCollector(Fleet([]), credential_fetches=lambda: {"us-east-1": 2, "eu-west-1": 1}).exposition().decode()
    assert "# TYPE ksa_aws_credential_fetches_total counter" in body
    assert 'ksa_aws_credential_fetches_total{region="eu-west-1"} 1.0' in body
    assert 'ksa_aws_credential_fetches_total{region="us-east-1"} 2.0' in body
    assert "ksa_aws_credential_fetches_total" not in FleetCollector(Fleet([])).exposition().decode()


def test_pooled_scheduler_many_queues_few_threads(nat):
    """64 queues on 4 native threads: every queue polls, decisions match a dedicated loop."""
    env = BenchEnv(64)
    try:
        cfg = nat.LoopConfig()
        cfg.poll_period_ns = 2_000_000  # 2 ms between a queue's polls
        cfg.scale_up_cool_down_ns = 0
        cfg.scale_down_cool_down_ns = 0
        runners = [nat.Runner(cfg, r.sqs, r.scaler, nat.RealClock(), env.log) for r in env.runners]
        fleet = Fleet([W(r, t) for r, t in zip(runners, env.targets)], threads=4)
        assert fleet.pooled
        fleet.start(12)
        assert fleet.wait(60)
        fleet.join()
        stats = fleet.stats()
        assert all(s["polls"] == 12 for s in stats)
        # 200/0 alternation from the fake: 6 scale-ups then 6 scale-downs interleaved, per queue
        assert all(s["scale_ups"] == 6 and s["scale_downs"] == 6 for s in stats)
        assert [env.kube.replicas("bench", t.deployment) for t in env.targets] == [1] * 64
        assert env.sqs.signature_failures() == 0
    finally:
        env.close()


def test_pooled_scheduler_keeps_cadence(nat, tmp_path):
    """A queue's consecutive polls are at least one poll period apart (sleep-then-work)."""
    import json

    env = BenchEnv(8)
    try:
        cfg = nat.LoopConfig()
        cfg.poll_period_ns = 20_000_000
        trace = tmp_path / "spans.jsonl"
        fd = __import__("os").open(str(trace), __import__("os").O_WRONLY | __import__("os").O_CREAT)
        runners = []
        for r in env.runners:
            rr = nat.Runner(cfg, r.sqs, r.scaler, nat.RealClock(), env.log)
            rr.set_trace_fd(fd)
            runners.append(rr)
        fleet = Fleet([W(r, t) for r, t in zip(runners, env.targets)], threads=2)
        fleet.start(6)
        fleet.join()
        __import__("os").close(fd)
        spans = [json.loads(l) for l in trace.read_text().splitlines()]
        by_q = {}
        for s in spans:
            by_q.setdefault(s["deployment"], []).append(s)
        assert len(by_q) == 8 and all(len(v) == 6 for v in by_q.values())
        for v in by_q.values():
            v.sort(key=lambda s: s["poll"])
            for a, b in zip(v, v[1:]):
                # next poll starts >= period after the previous poll ended
                assert b["ts"] - (a["ts"]) >= 20_000_000 - 1_000_000
    finally:
        env.close()


@pytest.mark.parametrize("prewarm_ns", [0, 2_000_000])
def test_pooled_scheduler_runs_the_pre_poll_warm_up(nat, prewarm_ns):
    """--poll-prewarm under the pooled scheduler: a warm-up event of its own before each poll
    (no spinning on a shared thread). It dials the apiserver client before the first poll, so
    even that poll pipelines its GET; without it the first GET is synchronous (the on-wire GET
    never dials). Decisions are the same either way."""
    env = BenchEnv(8)
    try:
        cfg = nat.LoopConfig()
        cfg.poll_period_ns = 20_000_000
        cfg.scale_up_cool_down_ns = 0
        cfg.scale_down_cool_down_ns = 0
        cfg.prefetch = True
        cfg.prewarm_ns = prewarm_ns
        runners = [nat.Runner(cfg, r.sqs, r.scaler, nat.RealClock(), env.log) for r in env.runners]
        fleet = Fleet([W(r, t) for r, t in zip(runners, env.targets)], threads=2)
        assert fleet.pooled
        fleet.start(4)
        assert fleet.wait(60)
        fleet.join()
        stats = fleet.stats()
        assert all(s["polls"] == 4 and s["scale_ups"] == 2 and s["scale_downs"] == 2 for s in stats)
        want = 4 if prewarm_ns else 3
        assert all(s["speculative_reads_used"] == want for s in stats), [s["speculative_reads_used"] for s in stats]
        assert env.sqs.signature_failures() == 0
    finally:
        env.close()


def test_liveness_detects_a_wedged_worker(nat):
    """/healthz fails once a running worker makes no progress for longer than its budget
    (here an SQS call that takes 1.5 s against a 0.2 s budget)."""
    import time

    from kube_sqs_autoscaler_amd.metrics import Health

    env = BenchEnv(1, sqs_latency_ns=1_500_000_000)
    try:
        fleet = Fleet([W(*a) for a in zip(env.runners, env.targets, env.kube_apis, env.sqs_apis)])
        h = Health(fleet, [200_000_000])
        assert h.live() == (True, "ok")  # not started: nothing to judge yet
        fleet.start(1)
        time.sleep(0.5)
        ok, why = h.live()
        assert not ok and "made no progress" in why and "gpu-worker-0" in why
        assert not h.ready()[0]
        fleet.join()
        assert h.live() == (True, "ok")  # the poll completed: progress again
    finally:
        env.close()


def test_standby_replica_is_ready(nat):
    """Under --leader-elect a standby never polls; it must still be Ready, or a rolling update
    of the 2-replica Deployment would wait on it forever."""
    from kube_sqs_autoscaler_amd.metrics import Health

    env = BenchEnv(1)
    try:
        fleet = Fleet([W(*a) for a in zip(env.runners, env.targets, env.kube_apis, env.sqs_apis)])
        h = Health(fleet, [Health.budget_ns(0, 30 * nat.SECOND)], leader_elect=True)
        m = MetricsServer(fleet, "127.0.0.1:0", h)
        m.start()
        try:
            base = f"http://127.0.0.1:{m.port}"
            assert urllib.request.urlopen(base + "/readyz").read() == b"standby"
            assert urllib.request.urlopen(base + "/healthz").read() == b"ok"
            h.set_role("leader")  # acquired the lease: ready only after the first poll
            with pytest.raises(urllib.error.HTTPError) as e:
                urllib.request.urlopen(base + "/readyz")
            assert e.value.code == 503
            fleet.start(3)
            fleet.join()
            assert urllib.request.urlopen(base + "/readyz").read() == b"ok"
        finally:
            m.stop()
    finally:
        env.close()


def test_health_budget_covers_retries():
    from kube_sqs_autoscaler_amd.metrics import Health

    assert Health.budget_ns(5 * 10**9, 30 * 10**9) == (5 + 240 + 60) * 10**9


@pytest.mark.parametrize("pooled", [False, True])
def test_stop_cancels_in_flight_calls(nat, pooled):
    """SIGTERM path: stopping the fleet aborts a worker's in-flight SQS call ("request canceled")
    instead of waiting for its 30 s timeout, so the process exits well inside the pod's grace
    period. (The reference has no graceful shutdown at all, main.go:36.)"""
    import time

    env = BenchEnv(2, sqs_latency_ns=20 * 10**9)  # the fake sits on every SQS call for 20 s
    try:
        fleet = Fleet([W(*a) for a in zip(env.runners, env.targets, env.kube_apis, env.sqs_apis)],
                      threads=1 if pooled else 0)
        fleet.start()
        time.sleep(0.3)  # both workers are now blocked inside GetQueueAttributes
        t0 = time.perf_counter()
        fleet.stop()
        assert fleet.wait(5)
        fleet.join()
        assert time.perf_counter() - t0 < 2.0
        assert all(s["depth_errors"] >= 1 for s in fleet.stats()[: 1 if pooled else 2])
    finally:
        env.close()


def test_latency_sum_and_buckets_cover_every_sample(nat):
    """The summary's sum and the histogram count every sample since start, not only the ones
    the latency ring still holds (the ring keeps the latest 65536)."""
    env = BenchEnv(1)
    try:
        env.run(50)
        env.clear()  # empties the ring; the cumulative sum and buckets stay
        env.run(50)
        st = env.runners[0].stats()
        assert st["latency_samples"] == 100 == sum(st["latency_buckets"])
        assert st["latency_sum_ns"] > sum(env.runners[0].latencies()) > 0
        assert len(nat.latency_bucket_le_ns) == len(st["latency_buckets"]) - 1
    finally:
        env.close()


def _readiness_env(nat, fail):
    env = BenchEnv(1)
    fail(env)
    fleet = Fleet([W(*a) for a in zip(env.runners, env.targets, env.kube_apis, env.sqs_apis)])
    from kube_sqs_autoscaler_amd.metrics import Health

    h = Health(fleet, [Health.budget_ns(0, 30 * nat.SECOND)], failure_window_ns=150_000_000)
    m = MetricsServer(fleet, "127.0.0.1:0", h)
    m.start()
    return env, fleet, m


def _get(url):
    try:
        r = urllib.request.urlopen(url)
        return r.status, r.read().decode()
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode()


@pytest.mark.parametrize("kind", ["sqs", "apiserver"])
def test_readyz_fails_while_every_poll_fails(nat, kind):
    """--readiness-failure-window: a queue that can never be read (SQS refuses the role) or a
    Deployment that can never be written (RBAC refuses /scale and the Deployment fallback too)
    turns /readyz to 503 after the window, while /healthz stays 200 (the loop is alive and
    retrying, as the reference's does); one good poll makes it ready again."""
    import time

    def fail(env):
        if kind == "sqs":
            env.sqs.inject(50000, nat.InjectedFault(403, "<ErrorResponse><Error><Type>Sender</Type><Code>AccessDenied</Code>"
                                                         "<Message>not authorized</Message></Error></ErrorResponse>",
                                                    "text/xml"))
        else:
            env.kube.set_rbac([])

    env, fleet, m = _readiness_env(nat, fail)
    base = f"http://127.0.0.1:{m.port}"
    try:
        fleet.start()
        deadline = time.time() + 10
        while "every poll failed" not in _get(base + "/readyz")[1]:
            assert time.time() < deadline, _get(base + "/readyz")
            time.sleep(0.02)
        code, why = _get(base + "/readyz")
        assert code == 503 and "every poll failed for" in why and "gpu-worker-0" in why
        assert ("AccessDenied" in why) if kind == "sqs" else ("forbidden" in why)
        assert _get(base + "/healthz") == (200, "ok")
        text = _get(base + "/metrics")[1]
        streak = [l for l in text.splitlines() if l.startswith("ksa_consecutive_failed_polls{")]
        assert streak and float(streak[0].rsplit(" ", 1)[1]) > 1
        assert any(l.startswith("ksa_failing_seconds{") and float(l.rsplit(" ", 1)[1]) >= 0.15 for l in text.splitlines())
        if kind == "apiserver":  # recovery: the next good poll makes the pod ready again
            env.kube.set_rbac(["*"])
            deadline = time.time() + 10
            while _get(base + "/readyz")[0] != 200:
                assert time.time() < deadline
                time.sleep(0.02)
            assert fleet.stats()[0]["consecutive_failed_polls"] == 0
    finally:
        fleet.stop()
        fleet.join()
        m.stop()
        env.close()


def test_readiness_window_zero_disables(nat):
    import time

    from kube_sqs_autoscaler_amd.metrics import Health

    env = BenchEnv(1)
    env.kube.set_rbac([])
    try:
        fleet = Fleet([W(*a) for a in zip(env.runners, env.targets, env.kube_apis, env.sqs_apis)])
        h = Health(fleet, [Health.budget_ns(0, 30 * nat.SECOND)], failure_window_ns=0)
        fleet.start(50)
        fleet.join()
        time.sleep(0.01)
        assert env.runners[0].failing_ns() > 0
        assert h.ready() == (True, "ok")
    finally:
        env.close()


def test_fleet_staggers_queue_starts(nat, tmp_path):
    """Four queues at one poll period start a quarter period apart (Supervisor.stagger): their
    polls do not arrive together every period. Each queue still polls one period after its own
    start (main.go:37-41)."""
    import json
    import os

    env = BenchEnv(4, poll_period_ns=200_000_000)
    try:
        trace = tmp_path / "t.jsonl"
        fd = os.open(trace, os.O_WRONLY | os.O_CREAT | os.O_APPEND)
        for r in env.runners:
            r.set_trace_fd(fd)
        fleet = Fleet([W(r, t) for r, t in zip(env.runners, env.targets)])
        fleet.start(2)
        assert fleet.wait(10)
        fleet.join()
        os.close(fd)
        spans = [json.loads(l) for l in trace.read_text().splitlines()]
    finally:
        env.close()
    first = sorted((s["ts"] - s["total_ns"]) for s in spans if s["poll"] == 1)
    gaps = [(b - a) / 1e6 for a, b in zip(first, first[1:])]
    assert len(first) == 4 and all(35 < g < 65 for g in gaps), gaps  # 50 ms apart


def test_metrics_listen_addresses():
    """Go-style listen addresses: ``:port`` listens on every interface (dual-stack where the host
    has IPv6, so an IPv6-only cluster reaches it), ``[::1]:port`` an IPv6 literal; a bad
    --metrics-addr is a flag error, not a traceback at start-up."""
    import socket

    from kube_sqs_autoscaler_amd.config import config_from_flags, new_flag_set
    from kube_sqs_autoscaler_amd.metrics import parse_addr
    from kube_sqs_autoscaler_amd.utils.goflag import FlagError

    assert parse_addr(":9090") == ("", 9090) and parse_addr("[::1]:80") == ("::1", 80)
    assert parse_addr("127.0.0.1:0") == ("127.0.0.1", 0)
    for bad in ("9090", "host:port", "::1:80", ":70000"):
        fs = new_flag_set("kube-sqs-autoscaler")
        fs.parse([f"--metrics-addr={bad}"])
        with pytest.raises(FlagError, match="metrics-addr"):
            config_from_flags(fs, {})

    class _Fleet:
        workers, stopped, started = [], False, False

        def stats(self):
            return []

    addrs = [":0", "127.0.0.1:0"] + (["[::1]:0"] if socket.has_ipv6 else [])
    for addr in addrs:
        try:
            m = MetricsServer(_Fleet(), addr)
        except OSError:  # no IPv6 loopback in this sandbox
            assert addr.startswith("[")
            continue
        m.start()
        try:
            host = "[::1]" if addr.startswith("[") else "127.0.0.1"  # ":0" takes IPv4 too
            assert urllib.request.urlopen(f"http://{host}:{m.port}/healthz", timeout=5).status == 200
        finally:
            m.stop()


@pytest.mark.slow
@pytest.mark.serial  # binds the container's resolver port: nothing else may resolve names meanwhile
def test_stop_cancels_a_hung_name_lookup(nat, tmp_path):
    """A poll dialling while the DNS server is silent waits in getaddrinfo on a helper thread
    (http.cc resolve(), bounded by --api-timeout); a stop ends that wait too, not only the
    socket waits. Needs a resolver at 127.0.0.1 this process may impersonate (the dev container,
    as root); skipped elsewhere."""
    import os
    import signal
    import socket
    import subprocess
    import sys
    import time

    import yaml

    try:
        with open("/etc/resolv.conf") as f:
            servers = [line.split()[1] for line in f if line.startswith("nameserver")]
    except OSError:
        servers = []
    if servers[:1] != ["127.0.0.1"]:
        pytest.skip("the resolver is not 127.0.0.1")
    dns = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        dns.bind(("127.0.0.1", 53))  # a DNS server that never answers
    except OSError as e:
        dns.close()
        pytest.skip(f"cannot stand in for the resolver: {e}")
    kube = nat.FakeKubeServer()
    kube.start()
    try:
        kube.add_deployment("default", "w", 2)
        kc = tmp_path / "kubeconfig"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": "t"}}],
            "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = dict(os.environ, AWS_ACCESS_KEY_ID="AKID", AWS_SECRET_ACCESS_KEY="secret", KUBE_CONFIG_PATH=str(kc),
                   HOME=str(tmp_path))
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        child = subprocess.Popen([sys.executable, "-m", "kube_sqs_autoscaler_amd", "--aws-region=us-east-1",
                                  "--sqs-endpoint=http://sqs.hung-dns.example.com", "--poll-period=100ms",
                                  "--sqs-queue-url=http://sqs.hung-dns.example.com/1/q", "--kubernetes-deployment=w",
                                  "--api-timeout=30s", "--log-level=error"], cwd=root, env=env,
                                 stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        deadline = time.monotonic() + 60
        dns.settimeout(1.0)
        while time.monotonic() < deadline:  # wait for the poll's lookup to reach the "server"
            try:
                dns.recvfrom(512)
                break
            except socket.timeout:
                assert child.poll() is None
        time.sleep(0.5)  # past the warm-up's 100 ms dial: the poll's own lookup is waiting now
        t0 = time.monotonic()
        child.send_signal(signal.SIGTERM)
        _, err = child.communicate(timeout=60)
        took = time.monotonic() - t0
        assert child.returncode == 0, err[-2000:]
        assert took < 2.0, took  # not the rest of the 30 s lookup budget
    finally:
        dns.close()
        kube.stop()
