"""One AWS credential source per process and region.

The reference builds one session per process (/root/reference/sqs/sqs.go:36), so one credential
fetch per expiry. Round 4 gave every tracked queue a chain of its own: N queues made N STS / ECS /
IMDS fetches at every expiry, each a Python urllib call on a worker thread. The CLI's queues
(threads or processes) now read one broker's sets from shared memory (parallel/credbroker.py,
cred_slot.h); a library user sharing a ``credentials_cache`` between ``new_runner`` calls gets
one ``SharedCredentialsProvider`` (sigv4.h) per region instead.
"""
import json
import threading
from datetime import datetime, timedelta, timezone
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest
import yaml

SEC = 1_000_000_000
AKID, SECRET, REGION, TOKEN = "ASIASHARED", "shared/secret", "us-east-1", "kube-token"


def test_shared_provider_fetches_once_per_expiry(nat):
    clock = nat.VirtualClock()
    calls = []

    class Inner(nat.CredentialsProvider):
        def retrieve(self):
            calls.append(clock.unix_nanos())
            return nat.Credentials("AKID", "secret", f"tok-{len(calls)}", clock.unix_nanos() + 600 * SEC, "Test")

    shared = nat.SharedCredentialsProvider(Inner(), clock)  # 5-minute expiry window
    got = [shared.retrieve() for _ in range(8)]
    assert len(calls) == 1 and {c.session_token for c in got} == {"tok-1"}
    clock.advance(299 * SEC)  # 301 s left: still outside the window
    assert shared.retrieve().session_token == "tok-1" and len(calls) == 1
    clock.advance(2 * SEC)  # 299 s left: inside it -> one fetch for every asker
    assert {shared.retrieve().session_token for _ in range(8)} == {"tok-2"} and len(calls) == 2
    # ExpiredToken seen by one client: the set is dropped once; a report about an older set is ignored
    old = got[0]
    shared.stale(old)
    assert shared.retrieve().session_token == "tok-2" and len(calls) == 2
    shared.stale(shared.retrieve())
    assert shared.retrieve().session_token == "tok-3" and len(calls) == 3
    assert shared.fetches() == 3


class _Ecs(BaseHTTPRequestHandler):
    """A container-credentials endpoint (AWS_CONTAINER_CREDENTIALS_FULL_URI): the first set
    expires 5 min + 1.5 s from now (so it enters every client's 5-minute refresh window 1.5 s
    into the run), later ones in an hour."""

    fetches = 0
    lock = threading.Lock()

    def do_GET(self):  # noqa: N802
        with _Ecs.lock:
            _Ecs.fetches += 1
            n = _Ecs.fetches
        left = timedelta(minutes=5, seconds=1.5) if n == 1 else timedelta(hours=1)
        body = json.dumps({"AccessKeyId": AKID, "SecretAccessKey": SECRET, "Token": f"session-{n}",
                           "Expiration": (datetime.now(timezone.utc) + left).strftime("%Y-%m-%dT%H:%M:%S.%fZ")}).encode()
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def log_message(self, *a):
        pass


@pytest.mark.slow
def test_eight_queues_one_fetch_per_expiry(nat, tmp_path):
    from kube_sqs_autoscaler_amd.cli import main

    _Ecs.fetches = 0
    ecs = ThreadingHTTPServer(("127.0.0.1", 0), _Ecs)
    threading.Thread(target=ecs.serve_forever, daemon=True).start()
    sqs = nat.FakeSqsServer()
    sqs.require_signature(AKID, SECRET, REGION)
    sqs.start()
    kube = nat.FakeKubeServer()
    kube.require_token(TOKEN)
    kube.start()
    try:
        kc = tmp_path / "kubeconfig"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": TOKEN}}],
            "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = {"HOME": str(tmp_path), "KUBE_CONFIG_PATH": str(kc), "AWS_EC2_METADATA_DISABLED": "true",
               "AWS_CONTAINER_CREDENTIALS_FULL_URI": f"http://127.0.0.1:{ecs.server_address[1]}/creds"}
        specs = []
        for i in range(8):
            url = f"{sqs.url}/123/q{i}"
            sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500" if i % 2 == 0 else "0"})
            kube.add_deployment("gpu", f"w{i}", 4)
            specs += ["--queue", f"url={url},deployment=w{i},namespace=gpu,attribute-names=ApproximateNumberOfMessages"]
        rc = main([f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=100ms",
                   "--scale-up-cool-down=0s", "--scale-down-cool-down=0s", "--log-level=error", *specs],
                  environ=env, max_iterations=25)  # 2.5 s: across the first set's refresh point
        assert rc == 0
        assert _Ecs.fetches == 2  # the first set, then its one refresh -- not 8 of each
        assert sqs.signature_failures() == 0
        # decisions are the reference's: each queue scaled to its bound
        assert [kube.replicas("gpu", f"w{i}") for i in range(8)] == [8, 1] * 4
        tokens = [v for k, v in sqs.last_headers() if k.lower() == "x-amz-security-token"]
        assert tokens == ["session-2"]  # the last poll signed with the refreshed set
    finally:
        ecs.shutdown()
        sqs.stop()
        kube.stop()


@pytest.mark.slow
def test_library_workers_share_one_provider(nat, tmp_path):
    """A library user building workers with ``new_runner(..., credentials_cache=cache)`` (not the
    CLI, which uses the broker) gets one ``SharedCredentialsProvider`` per region: 8 queues, one
    ECS fetch per expiry, decisions unchanged."""
    from kube_sqs_autoscaler_amd import autoscaler
    from kube_sqs_autoscaler_amd.config import parse_args
    from kube_sqs_autoscaler_amd.parallel.fleet import Fleet
    from kube_sqs_autoscaler_amd.utils.log import make_logger

    _Ecs.fetches = 0
    ecs = ThreadingHTTPServer(("127.0.0.1", 0), _Ecs)
    threading.Thread(target=ecs.serve_forever, daemon=True).start()
    sqs = nat.FakeSqsServer()
    sqs.require_signature(AKID, SECRET, REGION)
    sqs.start()
    kube = nat.FakeKubeServer()
    kube.require_token(TOKEN)
    kube.start()
    try:
        kc = tmp_path / "kubeconfig"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": TOKEN}}],
            "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = {"HOME": str(tmp_path), "KUBE_CONFIG_PATH": str(kc), "AWS_EC2_METADATA_DISABLED": "true",
               "AWS_CONTAINER_CREDENTIALS_FULL_URI": f"http://127.0.0.1:{ecs.server_address[1]}/creds"}
        specs = []
        for i in range(8):
            url = f"{sqs.url}/123/q{i}"
            sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500" if i % 2 == 0 else "0"})
            kube.add_deployment("gpu", f"w{i}", 4)
            specs += ["--queue", f"url={url},deployment=w{i},namespace=gpu,attribute-names=ApproximateNumberOfMessages"]
        cfg = parse_args([f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=100ms",
                          "--scale-up-cool-down=0s", "--scale-down-cool-down=0s", *specs], env)
        rest = autoscaler.load_rest_config(cfg, env)
        cache: dict = {}
        workers = [autoscaler.new_runner(t, cfg, rest, make_logger("error", "text"), nat.RealClock(), environ=env,
                                         credentials_cache=cache) for t in cfg.targets]
        assert list(cache) == [REGION] and isinstance(cache[REGION], nat.SharedCredentialsProvider)
        fleet = Fleet(workers)
        fleet.start(25)  # 2.5 s: across the first set's refresh point (5 min + 1.5 s)
        fleet.join()
        assert _Ecs.fetches == 2 == cache[REGION].fetches()
        assert sqs.signature_failures() == 0
        assert [kube.replicas("gpu", f"w{i}") for i in range(8)] == [8, 1] * 4
    finally:
        ecs.shutdown()
        sqs.stop()
        kube.stop()


def test_credential_slot_between_processes(nat):
    """cred_slot.h: the supervisor publishes a set, a worker reads it, asks for the next when its
    copy nears expiry, and gets it once the supervisor publishes; an error reaches the waiter."""
    from kube_sqs_autoscaler_amd.parallel.credbroker import CredentialBroker

    clock = nat.VirtualClock()
    calls = []

    class Inner(nat.CredentialsProvider):
        def retrieve(self):
            calls.append(1)
            if len(calls) == 3:
                raise RuntimeError("STS said no")
            return nat.Credentials("AKID", "secret", f"tok-{len(calls)}", clock.unix_nanos() + 3600 * SEC, "Test")

    broker = CredentialBroker(["us-east-1"], clock=clock, providers={"us-east-1": Inner()})
    try:
        addr = broker.addrs["us-east-1"]
        assert nat.read_credential_slot(addr)[2] == 0 and broker.serve_once() == 1 and len(calls) == 1
        worker = nat.SlotCredentialsProvider(addr, clock, 300 * SEC, 2 * SEC)
        assert worker.retrieve().session_token == "tok-1"
        assert broker.serve_once() == 0  # nothing asked, nothing due
        clock.advance(3300 * SEC)  # 300 s left: inside the worker's window (and the broker's lead)
        t = threading.Thread(target=lambda: broker.serve_once())
        t.start()
        assert worker.retrieve().session_token == "tok-2"
        t.join()
        assert len(calls) == 2
        worker.stale(worker.retrieve())  # the service rejected tok-2: the next fetch fails
        assert broker.serve_once() == 1
        with pytest.raises(nat.NativeError, match="STS said no"):
            worker.retrieve()
        assert broker.serve_once() == 1  # the failed worker asked again
        assert worker.retrieve().session_token == "tok-4"
    finally:
        broker.close()


@pytest.mark.slow
def test_worker_processes_share_one_fetch_per_expiry(nat, tmp_path):
    """--worker-processes: 4 worker processes, one ECS fetch per expiry between them (the
    supervisor's broker), decisions unchanged."""
    from kube_sqs_autoscaler_amd.cli import main

    _Ecs.fetches = 0
    ecs = ThreadingHTTPServer(("127.0.0.1", 0), _Ecs)
    threading.Thread(target=ecs.serve_forever, daemon=True).start()
    sqs = nat.FakeSqsServer()
    sqs.require_signature(AKID, SECRET, REGION)
    sqs.start()
    kube = nat.FakeKubeServer()
    kube.require_token(TOKEN)
    kube.start()
    try:
        kc = tmp_path / "kubeconfig"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": TOKEN}}],
            "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = {"HOME": str(tmp_path), "KUBE_CONFIG_PATH": str(kc), "AWS_EC2_METADATA_DISABLED": "true",
               "AWS_CONTAINER_CREDENTIALS_FULL_URI": f"http://127.0.0.1:{ecs.server_address[1]}/creds"}
        specs = []
        for i in range(4):
            url = f"{sqs.url}/123/q{i}"
            sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500" if i % 2 == 0 else "0"})
            kube.add_deployment("gpu", f"w{i}", 4)
            specs += ["--queue", f"url={url},deployment=w{i},namespace=gpu,attribute-names=ApproximateNumberOfMessages"]
        rc = main([f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=100ms", "--worker-processes",
                   "--scale-up-cool-down=0s", "--scale-down-cool-down=0s", "--log-level=error", *specs],
                  environ=env, max_iterations=25)
        assert rc == 0
        assert _Ecs.fetches == 2  # the first set, then its one refresh -- not 4 of each
        assert sqs.signature_failures() == 0
        assert [kube.replicas("gpu", f"w{i}") for i in range(4)] == [8, 1] * 2
        tokens = [v for k, v in sqs.last_headers() if k.lower() == "x-amz-security-token"]
        assert tokens == ["session-2"]
    finally:
        ecs.shutdown()
        sqs.stop()
        kube.stop()


def test_refresh_lead():
    """credbroker.refresh_due_at: halfway between the fetch and the queues' 5-minute window, at
    least 1 and at most 15 minutes before the window -- an hour-long set is refreshed 20 minutes
    before it expires (a credential endpoint may be down 15 minutes without a poll failing), a
    15-minute one 10 minutes before; a set shorter than that minimum at once (MIN_REFRESH_NS
    apart); one that does not expire never."""
    from kube_sqs_autoscaler_amd.parallel.credbroker import refresh_due_at

    m = 60 * SEC
    assert refresh_due_at(0, 60 * m) == 40 * m
    assert refresh_due_at(0, 15 * m) == 5 * m
    assert refresh_due_at(0, 8 * m) == 90 * SEC  # halfway through the 3 minutes before the window
    assert refresh_due_at(0, 6 * m + 30 * SEC) == 30 * SEC  # the 1-minute minimum lead, not 45 s
    assert refresh_due_at(0, 6 * m) == 0  # at once
    assert refresh_due_at(0, 4 * m) == -1 * m  # already inside the window: at once
    assert refresh_due_at(0, 0) is None


def test_failed_refresh_ahead_of_time_keeps_the_set(nat):
    """The broker refreshes a set ahead of the workers' window; when that fetch fails (an
    ECS / IMDS hiccup) the set in the slot, still good, stays -- republished with the fetch's
    error, so a worker reading the slot still gets it -- and the refresh is tried again later. An
    error reaches the slot only when a worker waits for a new set and none still signs (here: the
    service rejected it)."""
    from kube_sqs_autoscaler_amd.parallel.credbroker import MIN_REFRESH_NS, CredentialBroker

    clock = nat.VirtualClock()
    calls = []

    class Flaky(nat.CredentialsProvider):
        def retrieve(self):
            calls.append(1)
            if len(calls) in (2, 4):
                raise RuntimeError("EC2RoleRequestError: connection refused")
            return nat.Credentials("AKID", "secret", f"tok-{len(calls)}", clock.unix_nanos() + 3600 * SEC, "Test")

    warned = []
    broker = CredentialBroker(["us-east-1"], clock=clock, providers={"us-east-1": Flaky()},
                              log=lambda lvl, m: warned.append((lvl, m)))
    try:
        addr = broker.addrs["us-east-1"]
        assert broker.serve_once() == 1 and nat.read_credential_slot(addr)[2] == 1
        clock.advance(3600 * SEC - 330 * SEC)  # 5.5 min left: the broker's lead, not yet the workers' window
        assert broker.serve_once() == 1 and broker.refresh_errors == 1  # fetch 2 fails
        creds, err, gen = nat.read_credential_slot(addr)
        assert (creds.session_token, err, gen) == ("tok-1", "", 2)  # kept, marked with the refresh's error
        assert "connection refused" in nat.credential_slot_info(addr)["refresh_error"]
        assert len(warned) == 1 and warned[0][0] == "warning" and "keep signing" in warned[0][1]
        worker = nat.SlotCredentialsProvider(addr, clock, 300 * SEC, 2 * SEC)
        assert worker.retrieve().session_token == "tok-1"
        assert broker.serve_once() == 0  # not again before MIN_REFRESH_NS
        clock.advance(MIN_REFRESH_NS)
        assert broker.serve_once() == 1 and nat.read_credential_slot(addr)[0].session_token == "tok-3"
        assert nat.credential_slot_info(addr)["refresh_error"] == ""
        # a worker that waits for a new set after a rejection gets the error of a failing fetch
        worker.stale(worker.retrieve())
        assert broker.serve_once() == 1  # fetch 4 fails, asked for; the rejected set is not kept
        with pytest.raises(nat.NativeError, match="EC2RoleRequestError"):
            worker.retrieve()
        assert len(warned) == 1
    finally:
        broker.close()


def test_credential_slot_limits_and_regions(nat):
    """A set too large for the slot reaches the workers as an error, not a torn read; each region
    has a slot of its own, fetched with its own chain."""
    from kube_sqs_autoscaler_amd.parallel.credbroker import CredentialBroker

    clock = nat.VirtualClock()
    seen = []

    def chain(region, token):
        class Inner(nat.CredentialsProvider):
            def retrieve(self):
                seen.append(region)
                return nat.Credentials("AKID-" + region, "secret", token, 0, "Test")
        return Inner()

    broker = CredentialBroker(["eu-west-1", "us-east-1", "us-east-1"], clock=clock,
                              providers={"eu-west-1": chain("eu-west-1", "t" * 20_000),
                                         "us-east-1": chain("us-east-1", "small")})
    try:
        assert broker.regions == ["eu-west-1", "us-east-1"]
        assert broker.serve_once() == 2 and sorted(seen) == ["eu-west-1", "us-east-1"]
        creds, err, gen = nat.read_credential_slot(broker.addrs["eu-west-1"])
        assert gen == 1 and "do not fit" in err
        with pytest.raises(nat.NativeError, match="do not fit"):
            nat.SlotCredentialsProvider(broker.addrs["eu-west-1"], clock, 300 * SEC, 1 * SEC).retrieve()
        us = nat.SlotCredentialsProvider(broker.addrs["us-east-1"], clock, 300 * SEC, 1 * SEC).retrieve()
        assert us.access_key_id == "AKID-us-east-1" and us.session_token == "small"
        assert broker.serve_once() == 1  # the failed eu-west-1 worker asked again; us-east-1 never expires
    finally:
        broker.close()


class _HungEcs(BaseHTTPRequestHandler):
    """A container-credentials endpoint that never answers within the chain's 5 s timeout."""

    asked = threading.Event()

    def do_GET(self):  # noqa: N802
        _HungEcs.asked.set()
        threading.Event().wait(8)

    def log_message(self, *a):
        pass


@pytest.mark.slow
@pytest.mark.serial  # a stop's wall time: a loaded host (xdist) slows the processes' exit
@pytest.mark.parametrize("mode,queues,limit_s", [("processes", 2, 1.8), ("threads", 3, 1.8)])
def test_stop_while_waiting_for_credentials(nat, tmp_path, mode, queues, limit_s):
    """SIGTERM while the queues wait for credentials from a hung endpoint (the chain's ECS
    fetch times out after 5 s). The CLI's queues -- worker threads or worker processes -- wait
    for the broker's first set (cred_slot.h); the waits are cancelled with their API calls
    (Runner::stop -> SlotCredentialsProvider::cancel) and the broker's thread, inside the fetch,
    is not waited for, so the process exits at once (round 5 before the broker served the thread
    fleet: 7.4 s with 2 queues, each queueing a fetch of its own; then 2.4 s, the queues sharing
    the one fetch in flight)."""
    import os
    import signal
    import subprocess
    import sys
    import time

    _HungEcs.asked.clear()
    ecs = ThreadingHTTPServer(("127.0.0.1", 0), _HungEcs)
    ecs.daemon_threads = True
    threading.Thread(target=ecs.serve_forever, daemon=True).start()
    sqs = nat.FakeSqsServer()
    sqs.start()
    kube = nat.FakeKubeServer()
    kube.require_token(TOKEN)
    kube.start()
    try:
        kc = tmp_path / "kubeconfig"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": TOKEN}}],
            "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = {k: v for k, v in os.environ.items() if not k.startswith("AWS_")}
        env.update(HOME=str(tmp_path), KUBE_CONFIG_PATH=str(kc), AWS_EC2_METADATA_DISABLED="true",
                   AWS_CONTAINER_CREDENTIALS_FULL_URI=f"http://127.0.0.1:{ecs.server_address[1]}/creds")
        specs = []
        for i in range(queues):
            kube.add_deployment("gpu", f"w{i}", 2)
            specs.append(f"--queue=url={sqs.url}/123/q{i},deployment=w{i},namespace=gpu")
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        extra = ["--worker-processes"] if mode == "processes" else []
        child = subprocess.Popen([sys.executable, "-m", "kube_sqs_autoscaler_amd", f"--aws-region={REGION}",
                                  f"--sqs-endpoint={sqs.url}", "--poll-period=200ms", *extra,
                                  "--log-level=error", *specs], cwd=root, env=env,
                                 stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        assert _HungEcs.asked.wait(60), "the credential endpoint was never asked"
        time.sleep(0.5)  # every queue is waiting for that fetch now
        assert child.poll() is None
        t0 = time.monotonic()
        child.send_signal(signal.SIGTERM)
        _, err = child.communicate(timeout=60)
        took = time.monotonic() - t0
        assert child.returncode == 0, err[-2000:]
        assert took < limit_s, took
        assert sqs.requests() == 0  # nothing was signed without credentials
    finally:
        ecs.shutdown()
        sqs.stop()
        kube.stop()
