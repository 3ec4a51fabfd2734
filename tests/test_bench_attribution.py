"""The bench's attribution instrumentation (bench/latency.py): client HttpTiming and the fakes'
per-request wake-up/service times are recorded only when asked for -- the fake's receive-time
stamp costs syscalls on every round trip, so the latency rows run without it."""
import pytest

from kube_sqs_autoscaler_amd.bench.latency import BenchEnv, measure_cadenced


@pytest.mark.parametrize("timing", [False, True])
def test_fake_server_timings_only_when_enabled(nat, timing):
    import time

    env = BenchEnv(1, timing=timing)
    try:
        env.run(20)
        served = {"sqs": [], "kube": []}
        deadline = time.monotonic() + 2
        while True:  # a request is recorded after its response is written: the last may lag
            for k, v in env.server_timings().items():
                served[k] += v
            if not timing or (len(served["sqs"]) >= 20 and len(served["kube"]) >= 20) or time.monotonic() > deadline:
                break
            time.sleep(0.01)
    finally:
        env.close()
    if not timing:
        assert served == {"sqs": [], "kube": []}
        return
    assert len(served["sqs"]) >= 20 and len(served["kube"]) >= 20
    assert all(wake >= 0 and service > 0 for wake, service in served["sqs"] + served["kube"])


@pytest.mark.parametrize("servers", ["shared", "process", "split"])
def test_cadenced_rows_attribute_only_the_timed_runs(nat, servers):
    plain = measure_cadenced(20_000_000, 6, queues=4, busy_poll_ns=25_000, servers=servers, prewarm_ns=200_000)
    timed = measure_cadenced(20_000_000, 6, queues=4, busy_poll_ns=25_000, servers=servers, prewarm_ns=200_000,
                             timing=True)
    for r in (plain, timed):
        assert r["samples"] >= 12 and r["errors"] == 0 and r["signature_failures"] == 0
        assert r["p50_ms"] > 0
    assert "call_phase_median_us" not in plain and "endpoint_median_us" not in plain
    calls = timed["call_phase_median_us"]
    assert {"sign", "write", "wait", "read", "parse"} <= set(calls["sqs"])
    assert {"write", "wait"} <= set(calls["write"])
    assert timed["endpoint_median_us"]["sqs"]["service"] > 0
    assert timed["endpoint_median_us"]["kube"]["service"] > 0


def test_bench_workers_dial_their_own_connections(nat):
    """LoopConfig.connect_at_start: nothing is dialled while the bench environment is built (on
    the harness's thread); each worker connects both clients when it starts, so even its first
    poll sends the Deployment GET with the SQS request."""
    env = BenchEnv(2)
    try:
        assert env.kube_servers[0].connections() == 0 and env.sqs_servers[0].connections() == 0
        env.run(3)
        assert env.kube_servers[0].connections() == 2 and env.sqs_servers[0].connections() == 2
        for r in env.runners:
            st = r.stats()
            assert st["polls"] == 3 and st["speculative_reads"] == 3 and st["speculative_reads_used"] == 3
    finally:
        env.close()


US = 1_000


@pytest.mark.parametrize("busy_poll,ewma,budget,window", [
    (0, 50 * US, 10_000 * US, 0),              # --busy-poll=0s: never spin
    (25 * US, -1, 0, 25 * US),                 # no response-time sample yet: try the window
    (25 * US, 100 * US, 0, 25 * US),           # a fast peer (EWMA <= 4x window): the window
    (25 * US, 101 * US, 0, 0),                 # slower, no budget (pooled thread / back to back)
    (25 * US, 40 * US, 80 * US, 80 * US),      # near peer, 2x EWMA fits the budget: spin through it
    (25 * US, 40 * US, 79 * US, 25 * US),      # ... and does not: the window
    (25 * US, 150 * US, 1_000 * US, 200 * US),  # spin through capped at the 200 us ceiling
    (25 * US, 201 * US, 10**9, 0),             # slower than the ceiling: never, whatever the budget
    (25 * US, 15_000 * US, 37_500 * US, 0),    # a 15 ms WAN peer at the 5 s default period's budget
])
def test_spin_window_decision(nat, busy_poll, ewma, budget, window):
    """HttpClient::spin_window_for, the spin/no-spin decision of every response read, on injected
    EWMA and budget values (deterministic; the end-to-end checks below are load-dependent)."""
    assert nat.http_spin_window(busy_poll, ewma, budget) == window
    assert nat.http_spin_window(busy_poll, ewma, budget) <= nat.HTTP_MAX_SPIN_THROUGH_NS


@pytest.mark.slow
@pytest.mark.serial
@pytest.mark.parametrize("period_ms", [1000, 0])
def test_worker_never_spins_through_a_slow_answer(nat, period_ms):
    """End to end: an answer slower than HttpClient::kMaxSpinThrough (the fakes answer after
    0.4 ms plus their timer slack) is waited for in poll(2), never spun through -- even at a
    cadence with a worker budget of 10 % of the period (75 ms for the SQS call), far above
    2 x EWMA. Round 4 spun through such answers whenever 2 x EWMA fitted the budget, which
    burns a remote endpoint's whole round trip of CPU under a 100m CPU limit."""
    import json
    import tempfile

    env = BenchEnv(1, busy_poll_ns=25_000, poll_period_ns=period_ms * 1_000_000, timing=True,
                   sqs_latency_ns=400_000, kube_latency_ns=400_000, spin_budget_ppm=100_000)
    f = tempfile.TemporaryFile()
    try:
        env.runners[0].set_trace_fd(f.fileno())
        env.run(8)
        env.runners[0].set_trace_fd(-1)
        f.seek(0)
        spans = [json.loads(line) for line in f.read().decode().splitlines()][3:]  # EWMA settled
    finally:
        f.close()
        env.close()
    sqs = [s["detail"]["sqs"] for s in spans if s.get("detail") and s["detail"].get("sqs")]
    assert len(sqs) >= 4
    assert sum(1 for c in sqs if c["spun"]) == 0, sqs


def test_cli_queues_share_one_spin_budget(nat):
    """autoscaler.loop_config: a process's queues share --busy-poll-budget of their poll period
    (runner.h LoopConfig.spin_budget_ppm), so a large fleet's spinning stays bounded; the default
    is 0, the --busy-poll window only."""
    from kube_sqs_autoscaler_amd.autoscaler import DEFAULT_SPIN_BUDGET_PPM, loop_config
    from kube_sqs_autoscaler_amd.config import TargetConfig, parse_args

    t = TargetConfig(queue_url="https://sqs.us-east-1.amazonaws.com/1/q", deployment="d")
    assert DEFAULT_SPIN_BUDGET_PPM == 0 and parse_args(["--sqs-queue-url=u"]).busy_poll_budget_pct == 0.0
    assert loop_config(t).spin_budget_ppm == 0 and nat.LoopConfig().spin_budget_ppm == 0
    assert parse_args(["--sqs-queue-url=u", "--busy-poll-budget=1"]).busy_poll_budget_pct == 1.0
    assert loop_config(t, spin_budget_pct=1.0).spin_budget_ppm == 10_000
    assert loop_config(t, queues=16, spin_budget_pct=1.0).spin_budget_ppm == 625
    assert loop_config(t, queues=64, spin_budget_pct=1.0).spin_budget_ppm == 156
    assert loop_config(t, spin_budget_pct=0.25).spin_budget_ppm == 2_500
