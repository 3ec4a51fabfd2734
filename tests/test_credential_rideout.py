"""Credential outages and per-region isolation of the CLI's credential broker.

* A refresh that fails while the set still signs keeps that set: the queues sign with it past the
  SDK's 5-minute window until a refresh succeeds or the set is a minute from Expiration
  (parallel/credbroker.py, cred_slot.h). Round 5's soak with a 90 s outage and 60 s-lead sets
  failed 92 of 2838 polls where the set was still valid (profiles/r05ah); the reference would have
  decided the same on a successful read (/root/reference/sqs/sqs.go:51, main.go:47-53).
* A set the service rejected is never signed with again, even before the broker replaces it.
* Each region has its own serving thread: one region's hung endpoint does not delay another's
  fetch (/root/reference/sqs/sqs.go:35-43: the client per queue's region).
"""
import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest
import yaml

SEC = 1_000_000_000
AKID, SECRET, TOKEN = "ASIARIDE", "ride/secret", "kube-token"


def _short_sets(nat, clock, outage, life_s=420):
    """A chain whose sets live ``life_s`` (a 60 s refresh lead) and that fails inside
    ``outage`` = (start_s, end_s) of the virtual clock's seconds since ``t0``."""
    t0 = clock.unix_nanos()
    calls = []

    class Chain(nat.CredentialsProvider):
        def retrieve(self):
            now = clock.unix_nanos()
            calls.append(now)
            if outage[0] * SEC <= now - t0 < outage[1] * SEC:
                raise RuntimeError("EcsCredentialsError: 500 agent restarting")
            return nat.Credentials(AKID, SECRET, f"tok-{len(calls)}", now + life_s * SEC, "EcsProvider")

    return Chain(), calls


def test_outage_longer_than_the_lead_fails_no_poll(nat):
    """Round 5's r05ah case on a virtual clock: 7-minute sets (the broker refreshes 60 s after a
    fetch) and a 90 s outage starting at that refresh. The queues enter their 5-minute window
    at 120 s, 30 s into the outage: every poll still signs, 30 of them with the kept set, and the
    first refresh after the outage replaces it."""
    from kube_sqs_autoscaler_amd.parallel.credbroker import CredentialBroker

    clock = nat.VirtualClock()
    chain, calls = _short_sets(nat, clock, (60, 150))
    warned = []
    broker = CredentialBroker(["us-east-1"], clock=clock, providers={"us-east-1": chain},
                              log=lambda lvl, m: warned.append(m))
    try:
        addr = broker.addrs["us-east-1"]
        worker = nat.SlotCredentialsProvider(addr, clock, 300 * SEC, 1 * SEC)
        tokens, kept = [], []
        for s in range(0, 200):
            broker.serve_once()
            c = worker.retrieve()  # raises on a failed poll
            tokens.append(c.session_token)
            kept.append(c.kept_after_failed_refresh)
            clock.advance(1 * SEC)
        assert tokens[:150] == ["tok-1"] * 150 and set(tokens[150:]) == {"tok-11"}
        assert len(calls) == 11  # 1 fetch, 9 failed refreshes 10 s apart (60..140 s), 1 that worked
        assert [s for s, k in enumerate(kept) if k] == list(range(120, 150))  # inside the window
        assert len(warned) == 1 and "EcsCredentialsError" in warned[0]
        assert nat.credential_slot_info(addr)["wanted"] == 0  # no queue had to ask
    finally:
        broker.close()


@pytest.mark.slow
def test_fleet_polls_ride_out_a_failing_refresh(nat, tmp_path):
    """End to end: a queue whose set is inside its 5-minute window from the start (200 s left)
    while every refresh fails. Each poll's ask gets the kept set back at once; every poll reads
    the depth and scales as the reference would (4 -> 8 at 500 messages, one pod per poll), and
    every signed SQS request is counted in ksa_aws_credential_stale_signs_total."""
    from kube_sqs_autoscaler_amd import autoscaler
    from kube_sqs_autoscaler_amd.config import parse_args
    from kube_sqs_autoscaler_amd.metrics import FleetCollector
    from kube_sqs_autoscaler_amd.parallel.credbroker import CredentialBroker
    from kube_sqs_autoscaler_amd.parallel.fleet import Fleet
    from kube_sqs_autoscaler_amd.utils.log import make_logger

    clock = nat.RealClock()
    calls = []

    class Failing(nat.CredentialsProvider):
        def retrieve(self):
            calls.append(1)
            if len(calls) > 1:
                raise RuntimeError("EcsCredentialsError: 500 agent restarting")
            return nat.Credentials(AKID, SECRET, "only", clock.unix_nanos() + 200 * SEC, "EcsProvider")

    sqs = nat.FakeSqsServer()
    sqs.require_signature(AKID, SECRET, "us-east-1")
    sqs.start()
    kube = nat.FakeKubeServer()
    kube.require_token(TOKEN)
    kube.start()
    warned = []
    broker = CredentialBroker(["us-east-1"], clock=clock, providers={"us-east-1": Failing()},
                              log=lambda lvl, m: warned.append(m))
    fleet = None
    try:
        kc = tmp_path / "kubeconfig"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": TOKEN}}],
            "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = {"HOME": str(tmp_path), "KUBE_CONFIG_PATH": str(kc)}
        url = f"{sqs.url}/123/q"
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500"})
        kube.add_deployment("gpu", "w", 4)
        cfg = parse_args(["--aws-region=us-east-1", f"--sqs-endpoint={sqs.url}", "--poll-period=50ms",
                          "--scale-up-cool-down=0s", "--scale-down-cool-down=0s", "--max-pods=8",
                          f"--queue=url={url},deployment=w,namespace=gpu,attribute-names=ApproximateNumberOfMessages"],
                         env)
        rest = autoscaler.load_rest_config(cfg, env)
        workers = [autoscaler.new_runner(t, cfg, rest, make_logger("error", "text"), clock, environ=env,
                                         credentials=broker.provider_for("us-east-1")) for t in cfg.targets]
        broker.start()
        fleet = Fleet(workers)
        fleet.start(10)
        fleet.join()
        st = fleet.stats()[0]
        assert st["polls"] == 10 and st["depth_errors"] == 0 and kube.replicas("gpu", "w") == 8
        assert sqs.signature_failures() == 0 and sqs.requests() == 10
        stale = broker.stale_signs_by_region()["us-east-1"]
        assert stale == 10, stale  # every signed request, warm-ups not counted
        text = FleetCollector(fleet, credential_stale_signs=broker.stale_signs_by_region).exposition().decode()
        assert 'ksa_aws_credential_stale_signs_total{region="us-east-1"} 10' in text
        assert len(warned) == 1 and "keep signing" in warned[0]
    finally:
        if fleet is not None:
            fleet.stop()
            fleet.join()
        broker.close()
        sqs.stop()
        kube.stop()


def test_a_set_past_its_skew_fails_with_the_chains_error(nat):
    """The other half: an outage that outlasts the set. The kept set signs until a minute before
    its Expiration; then a poll asks, the broker's fetch fails, and the poll fails with the
    chain's own error text."""
    from kube_sqs_autoscaler_amd.parallel.credbroker import CredentialBroker

    clock = nat.VirtualClock()
    chain, calls = _short_sets(nat, clock, (60, 10_000))
    broker = CredentialBroker(["us-east-1"], clock=clock, providers={"us-east-1": chain})
    try:
        addr = broker.addrs["us-east-1"]
        worker = nat.SlotCredentialsProvider(addr, clock, 300 * SEC, 2 * SEC)
        broker.serve_once()
        clock.advance(120 * SEC)
        for _ in range(239):  # 120 .. 358 s: inside the window, the refresh failing, the set kept
            broker.serve_once()
            assert worker.retrieve().session_token == "tok-1"
            clock.advance(1 * SEC)
        clock.advance(2 * SEC)  # 361 s: 59 s before Expiration, inside the skew
        served = threading.Thread(target=lambda: [time.sleep(0.05), broker.serve_once()])
        served.start()
        with pytest.raises(nat.NativeError, match="EcsCredentialsError: 500 agent restarting"):
            worker.retrieve()
        served.join()
        assert nat.credential_slot_info(addr)["error"].startswith("EcsCredentialsError")
    finally:
        broker.close()


def test_a_rejected_set_is_not_signed_with_before_its_replacement(nat):
    """after ExpiredToken (stale()), the next retrieve() must not hand back the
    rejected set while the broker has not replaced it yet (round 5: it looked every 200 ms, an SQS
    retry comes after 30-120 ms): it waits for the replacement, and without one it fails rather
    than re-sign with the rejected key."""
    from kube_sqs_autoscaler_amd.parallel.credbroker import CredentialBroker

    clock = nat.RealClock()
    n = []

    class Chain(nat.CredentialsProvider):
        def retrieve(self):
            n.append(1)
            return nat.Credentials(AKID, SECRET, f"tok-{len(n)}", clock.unix_nanos() + 3600 * SEC, "Test")

    broker = CredentialBroker(["us-east-1"], clock=clock, providers={"us-east-1": Chain()})
    try:
        addr = broker.addrs["us-east-1"]
        broker.serve_once()
        worker = nat.SlotCredentialsProvider(addr, clock, 300 * SEC, 300_000_000)  # 0.3 s wait
        first = worker.retrieve()
        worker.stale(first)
        assert nat.credential_slot_info(addr)["rejected"] == 1
        with pytest.raises(nat.NativeError, match="NoCredentialProviders"):
            worker.retrieve()  # nobody serves: no replacement, and the rejected set is not used
        other = nat.SlotCredentialsProvider(addr, clock, 300 * SEC, 5 * SEC)  # another queue of the slot
        t = threading.Thread(target=lambda: [time.sleep(0.05), broker.serve_once()])
        t.start()
        assert other.retrieve().session_token == "tok-2"
        t.join()
        assert worker.retrieve().session_token == "tok-2"
    finally:
        broker.close()


def test_one_regions_hung_endpoint_does_not_delay_another(nat):
    """Region A's credential endpoint hangs (30 s); region B's queue holds a set about to expire
    and asks for a new one: B's serving thread fetches it within a second (its ask wakes that
    thread at once: typically a millisecond), because A's fetch blocks only A's thread."""
    from kube_sqs_autoscaler_amd.parallel.credbroker import CredentialBroker

    clock = nat.RealClock()
    release = threading.Event()
    entered = threading.Event()
    b_calls = []

    class Hung(nat.CredentialsProvider):
        def retrieve(self):
            entered.set()
            release.wait(30)
            raise RuntimeError("RequestError: send request failed (timeout)")

    class Fine(nat.CredentialsProvider):
        def retrieve(self):
            b_calls.append(1)
            life = 2 * SEC if len(b_calls) == 1 else 3600 * SEC  # the first set is about to expire
            return nat.Credentials(AKID, SECRET, f"b-{len(b_calls)}", clock.unix_nanos() + life, "Test")

    broker = CredentialBroker(["eu-west-1", "us-east-1"], clock=clock,
                              providers={"eu-west-1": Hung(), "us-east-1": Fine()})
    try:
        broker.start()
        assert entered.wait(5)
        deadline = time.monotonic() + 5
        while not b_calls and time.monotonic() < deadline:
            time.sleep(0.01)
        b = broker.provider_for("us-east-1", clock)
        t0 = time.monotonic()
        got = b.retrieve()  # b-1 is inside the window (expires in 2 s): ask, wait for b-2
        took = time.monotonic() - t0
        assert got.session_token == "b-2" and took < 1.0, took
        assert not release.is_set() and broker.fetches_by_region["eu-west-1"] == 1  # A is still hung
    finally:
        release.set()
        broker.close()


@pytest.mark.slow
def test_two_region_fleet_decides_while_one_region_hangs(nat, tmp_path):
    """The CLI's wiring end to end: two queues in two regions, region A's credential chain hung
    for the whole run. Region B's queue asks for a fresh set on its first poll (its first one
    expires in 2 s), gets it at once, and makes the reference's decisions: 500 messages scale its
    Deployment from 4 to the max of 8, one pod per poll. A's queue never signs."""
    from kube_sqs_autoscaler_amd import autoscaler
    from kube_sqs_autoscaler_amd.config import parse_args
    from kube_sqs_autoscaler_amd.parallel.credbroker import CredentialBroker
    from kube_sqs_autoscaler_amd.parallel.fleet import Fleet
    from kube_sqs_autoscaler_amd.utils.log import make_logger

    clock = nat.RealClock()
    release = threading.Event()
    b_calls = []

    class Hung(nat.CredentialsProvider):
        def retrieve(self):
            release.wait(30)
            raise RuntimeError("RequestError: send request failed (timeout)")

    class Fine(nat.CredentialsProvider):
        def retrieve(self):
            b_calls.append(time.monotonic())
            life = 2 * SEC if len(b_calls) == 1 else 3600 * SEC
            return nat.Credentials(AKID, SECRET, f"b-{len(b_calls)}", clock.unix_nanos() + life, "Test")

    sqs = nat.FakeSqsServer()
    sqs.require_signature(AKID, SECRET, "us-east-1")
    sqs.start()
    kube = nat.FakeKubeServer()
    kube.require_token(TOKEN)
    kube.start()
    broker = CredentialBroker(["eu-west-1", "us-east-1"], clock=clock,
                              providers={"eu-west-1": Hung(), "us-east-1": Fine()})
    fleet = None
    try:
        kc = tmp_path / "kubeconfig"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": TOKEN}}],
            "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = {"HOME": str(tmp_path), "KUBE_CONFIG_PATH": str(kc)}
        specs = []
        for name, region in (("wa", "eu-west-1"), ("wb", "us-east-1")):
            url = f"{sqs.url}/123/{name}"
            sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500"})
            kube.add_deployment("gpu", name, 4)
            specs += ["--queue", f"url={url},deployment={name},namespace=gpu,region={region},"
                                 "attribute-names=ApproximateNumberOfMessages"]
        cfg = parse_args(["--aws-region=us-east-1", f"--sqs-endpoint={sqs.url}", "--poll-period=100ms",
                          "--scale-up-cool-down=0s", "--scale-down-cool-down=0s", "--max-pods=8", *specs], env)
        rest = autoscaler.load_rest_config(cfg, env)
        log = make_logger("error", "text")
        workers = [autoscaler.new_runner(t, cfg, rest, log, clock, environ=env,
                                         credentials=broker.provider_for(t.region)) for t in cfg.targets]
        broker.start()
        fleet = Fleet(workers)
        t0 = time.monotonic()
        fleet.start(8)
        deadline = time.monotonic() + 20
        while kube.replicas("gpu", "wb") < 8 and time.monotonic() < deadline:
            time.sleep(0.02)
        took = time.monotonic() - t0
        assert kube.replicas("gpu", "wb") == 8 and took < 3.0, took  # 4 scaling polls, 100 ms apart
        assert len(b_calls) == 2 and sqs.signature_failures() == 0
        assert kube.replicas("gpu", "wa") == 4  # A never got a set: no decision, no write
    finally:
        if fleet is not None:
            fleet.stop()
            fleet.join()
        release.set()
        broker.close()
        sqs.stop()
        kube.stop()


def test_broker_close_and_stop_are_idempotent(nat):
    """close() unmaps the slots once; a later stop() or close() (a second signal, a finally
    after an exception) must not touch them."""
    from kube_sqs_autoscaler_amd.parallel.credbroker import CredentialBroker

    class Chain(nat.CredentialsProvider):
        def retrieve(self):
            return nat.Credentials(AKID, SECRET, "t", 0, "Test")

    broker = CredentialBroker(["us-east-1", "eu-west-1"], providers={"us-east-1": Chain(), "eu-west-1": Chain()})
    broker.start()
    broker.close()
    assert broker.stop() is True
    broker.close()


class _EcsThenDown(BaseHTTPRequestHandler):
    """A container-credentials endpoint that hands out one set with 200 s left (inside every
    queue's 5-minute window from the start) and then answers 500 (an agent restart)."""

    fetches = 0
    failed = 0
    lock = threading.Lock()

    def do_GET(self):  # noqa: N802
        from datetime import datetime, timedelta, timezone

        with _EcsThenDown.lock:
            _EcsThenDown.fetches += 1
            first = _EcsThenDown.fetches == 1
            if not first:
                _EcsThenDown.failed += 1
        if first:
            body = json.dumps({"AccessKeyId": AKID, "SecretAccessKey": SECRET, "Token": "only-set",
                               "Expiration": (datetime.now(timezone.utc) + timedelta(seconds=200))
                               .strftime("%Y-%m-%dT%H:%M:%SZ")}).encode()
            self.send_response(200)
        else:
            body = b'{"code":"InternalError","message":"agent restarting"}'
            self.send_response(500)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def log_message(self, *a):
        pass


@pytest.mark.slow
@pytest.mark.parametrize("processes", [False, True])
def test_cli_rides_out_a_credential_outage(nat, tmp_path, processes, capfd):
    """The CLI (threads, or --worker-processes sharing the slot across processes) with its only
    credential set inside the window and the endpoint down: every poll reads the depth and the
    Deployments scale to their max; the kept set signs every request and the log carries one
    warning."""
    from kube_sqs_autoscaler_amd.cli import main

    _EcsThenDown.fetches = _EcsThenDown.failed = 0
    ecs = ThreadingHTTPServer(("127.0.0.1", 0), _EcsThenDown)
    threading.Thread(target=ecs.serve_forever, daemon=True).start()
    sqs = nat.FakeSqsServer()
    sqs.require_signature(AKID, SECRET, "us-east-1")
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
        for i in range(3):
            url = f"{sqs.url}/123/q{i}"
            sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500"})
            kube.add_deployment("gpu", f"w{i}", 4)
            specs += ["--queue", f"url={url},deployment=w{i},namespace=gpu,attribute-names=ApproximateNumberOfMessages"]
        extra = ["--worker-processes"] if processes else []
        rc = main(["--aws-region=us-east-1", f"--sqs-endpoint={sqs.url}", "--poll-period=100ms", *extra,
                   "--scale-up-cool-down=0s", "--scale-down-cool-down=0s", "--max-pods=8", "--log-level=warning",
                   *specs], environ=env, max_iterations=6)
        err = capfd.readouterr().err
        assert rc == 0, err[-2000:]
        assert [kube.replicas("gpu", f"w{i}") for i in range(3)] == [8, 8, 8]
        assert sqs.requests() == 18 and sqs.signature_failures() == 0  # every poll read the depth
        assert "Failed to get SQS messages" not in err
        assert err.count("keep signing with the current set") == 1
        assert "AWS credential refresh for us-east-1 failed: NoCredentialProviders" in err
        assert _EcsThenDown.failed >= 1
    finally:
        ecs.shutdown()
        sqs.stop()
        kube.stop()
