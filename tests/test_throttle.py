"""Client-side kube-apiserver throttle: client-go's default rest client (QPS 5, burst 10 through
flowcontrol.NewTokenBucketRateLimiter, client-go v0.19 per /root/reference/go.mod:17). The
reference's clientset has it, so a fast poll period is throttled there too; here it is per tracked
queue (one reference process per queue) and `--kube-api-qps=0` switches it off."""
import time

import pytest

from kube_sqs_autoscaler_amd.autoscaler import new_deployment_api
from kube_sqs_autoscaler_amd.kube.config import RestConfig

S = 1_000_000_000


def test_token_bucket_starts_full_then_paces(nat):
    clock = nat.VirtualClock(0)
    b = nat.TokenBucket(5.0, 10, clock)
    assert [b.reserve() for _ in range(10)] == [0] * 10      # burst
    assert b.reserve() == S // 5                              # 11th waits one token (200 ms)
    assert b.reserve() == 2 * S // 5                          # reservations queue behind it
    clock.advance(S)                                          # 1 s refills 5 tokens: debt 2 -> 3 available
    assert [b.reserve() for _ in range(3)] == [0, 0, 0]
    assert b.reserve() == S // 5


def test_token_bucket_take_sleeps_on_the_clock(nat):
    clock = nat.VirtualClock(0)
    b = nat.TokenBucket(2.0, 1, clock)
    assert b.take() == 0 and clock.now() == 0
    assert b.take() == S // 2 and clock.now() == S // 2
    assert b.take() == S // 2 and clock.now() == S


def test_kube_client_is_throttled_over_the_wire(nat):
    kube = nat.FakeKubeServer()
    kube.require_token("t")
    kube.start()
    try:
        kube.add_deployment("ml", "w", 3)
        rc = RestConfig(host=kube.url, bearer_token="t")
        # the throttle runs on a VirtualClock: its waits are exact and a slow (loaded) test
        # runner cannot refill the bucket between requests
        clock = nat.VirtualClock(0)
        api = new_deployment_api(rc, "ml", "scale", 5 * S, clock=clock, qps=50.0, burst=2)
        for _ in range(6):
            assert api.get("w").replicas == 3
        st = api.stats()
        assert st["throttled"] == 4 and st["throttle_ns"] == 4 * S // 50 and clock.now() == 4 * S // 50
        free = new_deployment_api(rc, "ml", "scale", 5 * S)  # qps 0: unthrottled (bench path)
        for _ in range(20):
            free.get("w")
        assert free.stats()["throttled"] == 0
    finally:
        kube.stop()


def test_cli_default_matches_client_go():
    from kube_sqs_autoscaler_amd.config import parse_args

    cfg = parse_args(["--sqs-queue-url=q", "--kubernetes-deployment=d"], {})
    assert (cfg.kube_api_qps, cfg.kube_api_burst) == (5.0, 10)
    cfg = parse_args(["--sqs-queue-url=q", "--kubernetes-deployment=d", "--kube-api-qps=0"], {})
    assert cfg.kube_api_qps == 0


def test_throttled_loop_keeps_reference_decisions(nat):
    """A poll period far below the throttle's pace: the loop slows down as the reference's would
    (client-go blocks in Accept before each request); the decisions stay the reference's."""
    from kube_sqs_autoscaler_amd.bench.latency import BenchEnv

    env = BenchEnv(1)
    try:
        rc = RestConfig(host=env.kube.url, bearer_token="bench-bearer-token")
        api = new_deployment_api(rc, "bench", "scale", 5 * S, qps=100.0, burst=4)
        scaler = nat.PodAutoScaler(api, "gpu-worker-0", "bench", 8, 1, 1, 1, env.log, env.clock)
        cfg = nat.LoopConfig()
        cfg.poll_period_ns = 0
        cfg.scale_up_cool_down_ns = 0
        cfg.scale_down_cool_down_ns = 0
        cfg.scale_up_messages = 100
        cfg.scale_down_messages = 10
        cfg.prefetch = True
        r = nat.Runner(cfg, env.runners[0].sqs, scaler, env.clock, env.log)
        r.arm()
        recs = [r.poll_once() for _ in range(12)]
        assert [x["up"] for x in recs[::2]] == ["scaled"] * 6 and [x["down"] for x in recs[1::2]] == ["scaled"] * 6
        assert api.stats()["throttled"] >= 10
    finally:
        env.close()


@pytest.mark.parametrize("always", [True, False])
def test_speculative_read_never_waits_for_the_throttle(nat, always):
    """With prefetch_always a GET goes out with every poll, which the reference does not send.
    Once the bucket is empty the speculative GET is skipped rather than delayed, and only the
    reference's own GET (when a decision needs one) waits. The default gate sends none here:
    no poll can get past its cool-down."""
    from kube_sqs_autoscaler_amd.bench.latency import BenchEnv

    env = BenchEnv(1)
    try:
        rc = RestConfig(host=env.kube.url, bearer_token="bench-bearer-token")
        api = new_deployment_api(rc, "bench", "scale", 5 * S, qps=1.0, burst=3)
        scaler = nat.PodAutoScaler(api, "gpu-worker-0", "bench", 8, 1, 1, 1, env.log, env.clock)
        cfg = nat.LoopConfig()
        cfg.poll_period_ns = 0
        cfg.scale_up_cool_down_ns = 3600 * S  # every poll is a cool-down skip: no GET needed
        cfg.scale_down_cool_down_ns = 3600 * S
        cfg.scale_up_messages = 100
        cfg.scale_down_messages = 10
        cfg.prefetch = True
        cfg.prefetch_always = always
        r = nat.Runner(cfg, env.runners[0].sqs, scaler, env.clock, env.log)
        r.arm()
        scaler.warm()  # connected, as --poll-prewarm leaves it (the pipelined GET never dials)
        t0 = time.perf_counter()
        recs = [r.poll_once() for _ in range(20)]
        assert time.perf_counter() - t0 < 0.5  # no poll waited for a token
        st = api.stats()
        if always:
            assert sum(x["prefetched"] for x in recs) == 3 and st["speculative_skipped"] == 17
        else:
            assert all(x["prefetch_gated"] and x["gets"] == 0 for x in recs) and st["gets"] == 0
        assert st["throttled"] == 0
    finally:
        env.close()
