"""Decision parity: oracle vs SURVEY.md Appendix C goldens, and native loop vs oracle."""
import pytest

from kube_sqs_autoscaler_amd.models import oracle, parity, traces
from kube_sqs_autoscaler_amd.utils.goflag import SECOND


@pytest.mark.parametrize("sc", traces.baseline_scenarios(), ids=lambda s: s.name)
def test_oracle_reproduces_appendix_c(sc):
    ev = oracle.simulate(sc.params, sc.trace, sc.names, sc.polls, sc.init_replicas, sc.latency)
    assert traces.golden_from_events(ev, sc.params.poll_ns) == sc.golden


@pytest.mark.parametrize("sc", traces.baseline_scenarios(), ids=lambda s: s.name)
def test_native_loop_matches_oracle(sc):
    r = parity.compare(sc)
    assert r.ok, r.mismatches[:3]


def test_c1_never_writes():
    sc = traces.c1_noop()
    ev = oracle.simulate(sc.params, sc.trace, sc.names, sc.polls, sc.init_replicas, sc.latency)
    assert all(e.up == "none" and e.down in ("cooldown", "noop") for e in ev)
    # down-no-op at min every 30 s re-arms the timer: polls 6, 12, 18 ...
    noops = [e.index for e in ev if e.down == "noop"]
    assert noops[:3] == [6, 12, 18]


def test_c3_timers_armed_at_start_skip_early_bursts():
    sc = traces.c3_cooldown_bursty()
    ev = oracle.simulate(sc.params, sc.trace, sc.names, sc.polls, sc.init_replicas, sc.latency)
    early = [e for e in ev if e.t_poll_ns < 300 * SECOND and e.depth and e.depth >= 100]
    assert early and all(e.up == "cooldown" for e in early)


@pytest.mark.parametrize("name,case", list(traces.reference_test_scenarios().items()))
def test_reference_main_test_scenarios_virtual_clock(name, case):
    """The six /root/reference/main_test.go loop tests, in microseconds instead of 56 s."""
    p = case["params"]
    a, b, c = case["depth"]
    trace = [(0, traces.attrs(a, b, c))]
    polls = int(case["check_s"] * SECOND // p.poll_ns)
    sc = traces.Scenario(name, name, p, traces.DEFAULT_NAMES, trace, case["init"], polls,
                         latency=oracle.Latency(0, 0, 0))
    ref = oracle.simulate(p, trace, sc.names, polls, case["init"], sc.latency)
    assert ref[-1].replicas == case["expect"]
    got = parity.run_native(sc)
    assert got[-1].replicas == case["expect"]
    assert [e.key() for e in got] == [e.key() for e in ref]


def test_fault_injection_parity():
    sc = traces.c2_step()
    f = oracle.Faults(sqs={3, 7, 50}, up_get={14}, up_update={17}, down_get={36}, down_update={43})
    r = parity.compare(sc, f)
    assert r.ok, r.mismatches[:3]
    ev = oracle.simulate(sc.params, sc.trace, sc.names, sc.polls, sc.init_replicas, sc.latency, f)
    by = {e.index: e for e in ev}
    assert by[50].depth is None and by[3].depth is None  # SQS error: iteration skipped
    # a failed GET/PUT does not refresh the timer, so the very next poll retries
    assert by[14].up == "failed" and by[15].up == "scaled"
    assert by[17].up == "failed" and by[18].up == "scaled"
    assert by[36].down == "failed" and by[37].down == "scaled"
    assert by[43].down == "failed" and by[44].down == "scaled"


@pytest.mark.parametrize("sc", traces.baseline_scenarios(), ids=lambda s: s.name)
def test_pipelined_reads_parity_and_goldens(sc):
    """--pipeline-reads: the native loop matches the pipelined-time oracle, and the decisions
    are still the reference's Appendix C goldens."""
    r = parity.compare(sc, prefetch=True)
    assert r.ok, r.mismatches[:3]
    ev = oracle.simulate(sc.params, sc.trace, sc.names, sc.polls, sc.init_replicas, sc.latency, prefetch=True)
    assert traces.golden_from_events(ev, sc.params.poll_ns) == sc.golden


@pytest.mark.parametrize("sc", traces.baseline_scenarios(), ids=lambda s: s.name)
def test_gated_prefetch_reads_what_the_reference_reads(sc):
    """--pipeline-reads on the Appendix C traces sends exactly the reference's Deployment GETs
    (C1: 20 in 120 polls, one per down-no-op at min), where sending one with every poll would
    read on every poll."""
    r = parity.compare(sc, prefetch=True)
    assert r.ok, r.mismatches[:3]
    ref = oracle.simulate(sc.params, sc.trace, sc.names, sc.polls, sc.init_replicas, sc.latency)
    ev = oracle.simulate(sc.params, sc.trace, sc.names, sc.polls, sc.init_replicas, sc.latency, prefetch=True)
    assert sum(e.gets for e in ev) == oracle.reference_gets(ref) == sum(e.gets for e in ref)
    always = oracle.simulate(sc.params, sc.trace, sc.names, sc.polls, sc.init_replicas, sc.latency, prefetch=True,
                             prefetch_always=True)
    assert sum(e.gets for e in always) == sc.polls
    if sc.name.startswith("c1"):
        assert oracle.reference_gets(ref) == 20 and sc.polls == 120
