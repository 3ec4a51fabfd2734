"""Lease leader election (extension; the reference can only run one replica, README.md:27)."""
import json
import os
import subprocess
import sys
import threading
import time

import pytest
import yaml

from kube_sqs_autoscaler_amd.kube.config import RestConfig
from kube_sqs_autoscaler_amd.kube.leader import LeaderElector, LeaseLock

TOKEN = "lease-token"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def kube(nat):
    k = nat.FakeKubeServer()
    k.require_token(TOKEN)
    k.start()
    yield k
    k.stop()


class FakeMono:
    def __init__(self):
        self.t = 100.0

    def __call__(self):
        return self.t


def elector(kube, ident, mono):
    lock = LeaseLock(RestConfig(host=kube.url, bearer_token=TOKEN), "ml", "ksa")
    return LeaderElector(lock, ident, 15, 10, 2, monotonic=mono, wall=lambda: 1_700_000_000 + mono())


def lease(kube):
    return json.loads(kube.lease_json("ml", "ksa"))


def test_acquire_creates_and_renews(kube):
    m = FakeMono()
    a = elector(kube, "a", m)
    assert a.try_acquire_or_renew()
    spec = lease(kube)["spec"]
    assert spec["holderIdentity"] == "a" and spec["leaseDurationSeconds"] == 15 and spec["leaseTransitions"] == 0
    acquired = spec["acquireTime"]
    m.t += 2
    assert a.try_acquire_or_renew()
    spec = lease(kube)["spec"]
    assert spec["acquireTime"] == acquired and spec["renewTime"] != acquired and spec["leaseTransitions"] == 0


def test_standby_waits_until_lease_expires_by_local_clock(kube):
    m = FakeMono()
    a, b = elector(kube, "a", m), elector(kube, "b", m)
    assert a.try_acquire_or_renew()
    assert not b.try_acquire_or_renew()
    m.t += 14
    assert not b.try_acquire_or_renew()  # still valid (observed 14 s ago)
    m.t += 2
    assert b.try_acquire_or_renew()  # a stopped renewing: expired
    spec = lease(kube)["spec"]
    assert spec["holderIdentity"] == "b" and spec["leaseTransitions"] == 1


def test_renewals_keep_standby_out(kube):
    m = FakeMono()
    a, b = elector(kube, "a", m), elector(kube, "b", m)
    assert a.try_acquire_or_renew()
    for _ in range(20):
        m.t += 2
        assert a.try_acquire_or_renew()
        assert not b.try_acquire_or_renew()  # every renewal resets b's observation time


def test_release_lets_standby_in_immediately(kube):
    m = FakeMono()
    a, b = elector(kube, "a", m), elector(kube, "b", m)
    assert a.try_acquire_or_renew()
    a._leader = True
    assert a.release()
    assert lease(kube)["spec"]["holderIdentity"] == ""
    assert b.try_acquire_or_renew()


def test_simultaneous_candidates_one_wins(kube):
    m = FakeMono()
    es = [elector(kube, f"c{i}", m) for i in range(6)]
    wins = []
    barrier = threading.Barrier(len(es))

    def go(e):
        barrier.wait()
        if e.try_acquire_or_renew():
            wins.append(e.identity)

    ts = [threading.Thread(target=go, args=(e,)) for e in es]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert len(wins) == 1 and lease(kube)["spec"]["holderIdentity"] == wins[0]


def test_renew_loop_reports_loss(kube):
    m = FakeMono()
    a = LeaderElector(LeaseLock(RestConfig(host=kube.url, bearer_token=TOKEN), "ml", "ksa"), "a", 0.6, 0.3, 0.05)
    assert a.try_acquire_or_renew()
    a._leader = True
    kube.inject(1000, __import__("kube_sqs_autoscaler_amd.ops", fromlist=["fakes"]).fakes().InjectedFault(500, "down"))
    lost = threading.Event()
    stop = threading.Event()
    t = threading.Thread(target=a.renew_loop, args=(stop, lost.set))
    t.start()
    assert lost.wait(5)
    stop.set()
    t.join()
    assert not a.is_leader


def test_invalid_timings():
    with pytest.raises(ValueError):
        LeaderElector(None, "x", 10, 10, 2)


def test_two_processes_failover(nat, kube, tmp_path):
    sqs = nat.FakeSqsServer()
    sqs.start()
    try:
        url = sqs.url + "/1/q"
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": "0"})
        kube.add_deployment("ml", "w", 3)
        kc = tmp_path / "kc"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": TOKEN}}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = dict(os.environ, AWS_ACCESS_KEY_ID="a", AWS_SECRET_ACCESS_KEY="b", KUBE_CONFIG_PATH=str(kc))
        args = [sys.executable, "-m", "kube_sqs_autoscaler_amd", f"--sqs-queue-url={url}", "--kubernetes-deployment=w",
                "--kubernetes-namespace=ml", "--aws-region=us-east-1", f"--sqs-endpoint={sqs.url}", "--poll-period=50ms",
                "--scale-down-cool-down=0s", "--attribute-names=ApproximateNumberOfMessages", "--leader-elect",
                "--leader-elect-lease-duration=3s", "--leader-elect-renew-deadline=2s", "--leader-elect-retry-period=200ms"]

        def start(ident):
            return subprocess.Popen(args + [f"--leader-elect-identity={ident}"], cwd=ROOT, env=env,
                                    stderr=subprocess.PIPE, text=True)

        def wait_for(p, text, timeout=60):
            buf = ""
            deadline = time.time() + timeout
            while text not in buf and time.time() < deadline:
                line = p.stderr.readline()
                if not line:
                    break
                buf += line
            return text in buf

        a = start("a")
        b = None
        try:
            assert wait_for(a, "Starting kube-sqs-autoscaler")
            b = start("b")
            assert wait_for(b, "attempting to acquire leader lease")
            time.sleep(1.0)
            assert json.loads(kube.lease_json("ml", "kube-sqs-autoscaler"))["spec"]["holderIdentity"] == "a"
            a.terminate()
            assert a.wait(timeout=20) == 0  # graceful: releases the lease
            assert wait_for(b, "Starting kube-sqs-autoscaler", timeout=20)  # took over without waiting 3 s lease
            assert json.loads(kube.lease_json("ml", "kube-sqs-autoscaler"))["spec"]["holderIdentity"] == "b"
        finally:
            for p in (a, b):
                if p is not None and p.poll() is None:
                    p.kill()
        assert kube.replicas("ml", "w") == 1
    finally:
        sqs.stop()


def test_hanging_renewal_loses_leadership_at_the_deadline(nat, kube):
    """a renewal that hangs must not stretch leadership past renew_deadline. The lease
    calls get only the time left before the deadline, and a watchdog ends leadership when it
    passes, long before the lease client's own 10 s timeout."""
    a = LeaderElector(LeaseLock(RestConfig(host=kube.url, bearer_token=TOKEN), "ml", "ksa", timeout_s=10.0),
                      "a", 1.2, 0.6, 0.1)
    assert a.try_acquire_or_renew()
    a._leader = True
    lost_at = []
    stop = threading.Event()
    t0 = time.monotonic()
    kube.set_latency(5_000_000_000)  # every apiserver call now hangs for 5 s
    th = threading.Thread(target=a.renew_loop, args=(stop, lambda: lost_at.append(time.monotonic())))
    th.start()
    try:
        deadline = time.monotonic() + 4
        while not lost_at and time.monotonic() < deadline:
            time.sleep(0.01)
        assert lost_at, "leadership not given up"
        assert lost_at[0] - t0 < 0.6 + 0.4  # renew_deadline (+ scheduling slack), not 10 s
        assert not a.is_leader
    finally:
        stop.set()
        kube.set_latency(0)
        th.join(timeout=10)
    assert not th.is_alive()
    assert len(lost_at) == 1


def test_lock_deadline_uses_the_electors_clock():
    """The renew deadline handed to the lock and the lock's per-call limit share one time base
    (an injected clock far from time.monotonic must not expire every call)."""
    from kube_sqs_autoscaler_amd.kube.leader import LeaderElector

    class Lock:
        deadline = None
        monotonic = None
        calls = []

        def describe(self):
            return "ns/lease"

        def get(self):
            # the time left before the deadline, on the lock's clock, as _call computes it
            self.calls.append(self.deadline - self.monotonic() if self.deadline is not None else None)
            return None

        def create(self, rec):
            pass

    clock = [1e9]  # nowhere near time.monotonic()
    lock = Lock()
    el = LeaderElector(lock, "me", 15, 10, 0.01, monotonic=lambda: clock[0], wall=lambda: 0.0)
    assert lock.monotonic() == 1e9
    import threading

    stop = threading.Event()
    t = threading.Thread(target=el.renew_loop, args=(stop, lambda: None))
    t.start()
    import time

    time.sleep(0.1)
    stop.set()
    t.join()
    assert lock.calls and all(c is not None and 0 < c <= 10 for c in lock.calls)
