"""Fault tolerance over the real wire path (the reference's error paths were never tested,
SURVEY.md §4): random 5xx, dropped connections, write conflicts and hung calls must never crash
the loop, never push replicas outside [min, max], and the loop must converge once faults stop."""
import random

import pytest

from kube_sqs_autoscaler_amd.autoscaler import new_deployment_api, new_sqs_api
from kube_sqs_autoscaler_amd.kube.config import RestConfig
from kube_sqs_autoscaler_amd.sqs.credentials import static_provider
from kube_sqs_autoscaler_amd.utils.log import capture_logger

AKID, SECRET, REGION, TOKEN = "AKIDCHAOS", "chaos-secret", "us-east-1", "chaos-token"


def make_loop(nat, sqs, kube, mode, prefetch, timeout_ns=2 * 10**9, lines=None):
    url = sqs.url + "/1/chaos"
    api = new_sqs_api(REGION, nat.RealClock(), endpoint=sqs.url, credentials=static_provider(AKID, SECRET),
                      timeout_ns=timeout_ns, retry_delays_ns=(1_000_000, 5_000_000))  # SDK back-off, shortened
    client = nat.SqsClient(api, url, ["ApproximateNumberOfMessages"])
    dep = new_deployment_api(RestConfig(host=kube.url, bearer_token=TOKEN), "ml", mode, timeout_ns)
    log = capture_logger(lines if lines is not None else [])
    scaler = nat.PodAutoScaler(dep, "w", "ml", 8, 2, 1, 1, log, nat.RealClock())
    cfg = nat.LoopConfig()
    cfg.poll_period_ns = 0
    cfg.scale_up_cool_down_ns = 0
    cfg.scale_down_cool_down_ns = 0
    cfg.prefetch = prefetch
    r = nat.Runner(cfg, client, scaler, nat.RealClock(), log)
    r.arm()
    return r, url


@pytest.mark.parametrize("mode,prefetch,seed", [("scale", True, 1), ("deployment", False, 2), ("patch", True, 3), ("scale", False, 4)])
def test_random_faults_keep_invariants(nat, mode, prefetch, seed):
    rng = random.Random(seed)
    sqs, kube = nat.FakeSqsServer(), nat.FakeKubeServer()
    sqs.require_signature(AKID, SECRET, REGION)
    kube.require_token(TOKEN)
    sqs.start()
    kube.start()
    try:
        kube.add_deployment("ml", "w", 5)
        lines = []
        r, url = make_loop(nat, sqs, kube, mode, prefetch, lines=lines)
        for step in range(300):
            sqs.set_attributes(url, {"ApproximateNumberOfMessages": str(rng.choice([0, 5, 50, 150, 500]))})
            f = rng.random()
            if f < 0.08:
                sqs.inject(rng.randint(1, 5), nat.InjectedFault(rng.choice([500, 503]), "sqs down"))
            elif f < 0.14:
                kube.inject(1, nat.InjectedFault(rng.choice([500, 503, 429]), "apiserver hiccup"))
            elif f < 0.18:
                kube.conflict_next(1)
            elif f < 0.21:
                kube.drop_connections()
            elif f < 0.24:
                sqs.drop_connections()
            elif f < 0.26:
                kube.inject(1, nat.InjectedFault(0, "", "text/plain", True))  # close without responding
            rec = r.step()
            reps = kube.replicas("ml", "w")
            assert 2 <= reps <= 8, (step, rec)
        st = r.stats()
        assert st["polls"] == 300
        assert st["failed_ups"] + st["failed_downs"] + st["depth_errors"] > 0  # faults really happened
        assert any("level=error" in l for l in lines)
        # faults stop: the loop converges to the bound the backlog dictates
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500"})
        r.steps(10)
        assert kube.replicas("ml", "w") == 8
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": "0"})
        r.steps(10)
        assert kube.replicas("ml", "w") == 2
    finally:
        sqs.stop()
        kube.stop()


def test_hung_apiserver_times_out_and_loop_continues(nat):
    sqs, kube = nat.FakeSqsServer(), nat.FakeKubeServer()
    sqs.require_signature(AKID, SECRET, REGION)
    sqs.start()
    kube.require_token(TOKEN)
    kube.start()
    try:
        kube.add_deployment("ml", "w", 3)
        lines = []
        r, url = make_loop(nat, sqs, kube, "scale", True, timeout_ns=200_000_000, lines=lines)
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500"})
        kube.set_latency(1_000_000_000)  # 1 s > 200 ms timeout
        rec = r.step()
        assert rec["up"] == "failed" and "timeout" in rec["error"]
        kube.set_latency(0)
        recs = r.steps(3)
        assert recs[0]["up"] == "scaled"  # the failed attempt did not refresh the timer
        assert kube.replicas("ml", "w") >= 4
    finally:
        sqs.stop()
        kube.stop()


def test_hung_sqs_times_out(nat):
    sqs, kube = nat.FakeSqsServer(), nat.FakeKubeServer()
    sqs.require_signature(AKID, SECRET, REGION)
    sqs.start()
    kube.require_token(TOKEN)
    kube.start()
    try:
        kube.add_deployment("ml", "w", 3)
        r, url = make_loop(nat, sqs, kube, "scale", True, timeout_ns=150_000_000)
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": "0"})
        sqs.set_latency(1_000_000_000)
        rec = r.step()
        assert not rec["depth_ok"] and "Failed to get messages in SQS" in rec["error"]
        assert kube.replicas("ml", "w") == 3  # nothing scaled on a failed depth read
    finally:
        sqs.set_latency(0)
        sqs.stop()
        kube.stop()
