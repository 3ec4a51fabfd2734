"""Hypothesis: random policies/traces/faults -> the native loop agrees with the oracle poll by poll."""
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from kube_sqs_autoscaler_amd.models import oracle, parity, traces
from kube_sqs_autoscaler_amd.utils.goflag import MILLISECOND, SECOND

periods = st.sampled_from([0, 1 * MILLISECOND, 500 * MILLISECOND, 1 * SECOND, 5 * SECOND, 7 * SECOND])
cools = st.sampled_from([0, 1 * SECOND, 4 * SECOND, 5 * SECOND, 10 * SECOND, 12 * SECOND, 30 * SECOND, 300 * SECOND])


@st.composite
def scenarios(draw, with_faults=False):
    p = oracle.Params(
        poll_ns=draw(periods), up_cool_ns=draw(cools), down_cool_ns=draw(cools),
        up_msgs=draw(st.integers(-5, 300)), down_msgs=draw(st.integers(-5, 300)),  # overlapping thresholds allowed
        up_pods=draw(st.integers(0, 7)), down_pods=draw(st.integers(0, 7)),
        max_pods=draw(st.integers(0, 12)), min_pods=draw(st.integers(0, 12)),  # min > max allowed, like the reference
    )
    n_seg = draw(st.integers(1, 6))
    starts = sorted(draw(st.lists(st.integers(0, 400), min_size=n_seg, max_size=n_seg)))
    trace = [(0 if i == 0 else s * SECOND, traces.attrs(draw(st.integers(0, 400)), draw(st.integers(0, 50)),
                                                       draw(st.integers(0, 50)))) for i, s in enumerate(starts)]
    lat_ms = draw(st.sampled_from([0, 1, 3]))
    sc = traces.Scenario("prop", "hypothesis", p, list(draw(st.sampled_from([traces.DEFAULT_NAMES, traces.C5_NAMES]))),
                         trace, draw(st.integers(0, 14)), draw(st.integers(1, 80)),
                         latency=oracle.Latency(lat_ms * MILLISECOND, lat_ms * MILLISECOND, lat_ms * MILLISECOND))
    faults = None
    if with_faults:
        pick = st.sets(st.integers(1, sc.polls), max_size=6)
        faults = oracle.Faults(draw(pick), draw(pick), draw(pick), draw(pick), draw(pick))
    return sc, faults


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(scenarios(), st.sampled_from(["off", "gated", "always"]))
def test_native_equals_oracle(case, prefetch):
    """Poll-by-poll agreement, including (with --pipeline-reads) whether the gate sent the
    speculative GET and how many GETs the poll made."""
    sc, _ = case
    r = parity.compare(sc, prefetch=prefetch != "off", prefetch_always=prefetch == "always")
    assert r.ok, r.mismatches[:2]


def _depth_class(d, p):
    return "up" if d >= p.up_msgs else ("down" if d <= p.down_msgs else "band")


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(scenarios())
def test_prefetch_gate_costs_the_reference_api_reads(case):
    """The gated speculative GET goes out exactly on the polls that call ScaleUp/ScaleDown
    whenever the depth stayed in the same threshold class as the previous read, so the
    apiserver sees the reference's reads plus at most one per class change -- never one per
    poll (120 GETs vs the reference's 20 on an idle queue)."""
    sc, _ = case
    p = sc.params
    ref = oracle.simulate(p, sc.trace, sc.names, sc.polls, sc.init_replicas, sc.latency)
    ev = oracle.simulate(p, sc.trace, sc.names, sc.polls, sc.init_replicas, sc.latency, prefetch=True)
    called = ("scaled", "noop", "failed")
    prev = None
    changes = 0
    for e in ev:
        if e.depth is None:
            changes += 1  # a failed read: a prefetch sent with it is drained
            continue
        if prev is not None and _depth_class(e.depth, p) == _depth_class(prev, p):
            assert e.prefetched == (e.up in called or e.down in called), e
        elif prev is not None:
            changes += 1
        prev = e.depth
    ref_gets = oracle.reference_gets(ref)
    gated = sum(e.gets for e in ev)
    if p.poll_ns >= 500 * MILLISECOND:  # same decisions as the reference (see below)
        assert ref_gets <= gated <= ref_gets + changes + 1


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(scenarios())
def test_pipelined_reads_keep_reference_decisions(case):
    """With API latency far below the poll period (ms vs s), overlapping the GET with the SQS
    call changes no decision: same depth, actions and replicas at every poll -- up to the poll
    where the two schedules first read different depths. A pipelined poll ends earlier, so later
    polls start a little earlier than the sequential ones (by the overlapped GETs' latency, summed
    over the polls so far); once that drift carries one schedule's poll across a trace boundary
    the other does not cross yet, they sample different queues, as two reference processes
    started a few ms apart would."""
    sc, _ = case
    if sc.params.poll_ns < 500 * MILLISECOND:
        return
    a = oracle.simulate(sc.params, sc.trace, sc.names, sc.polls, sc.init_replicas, sc.latency)
    b = oracle.simulate(sc.params, sc.trace, sc.names, sc.polls, sc.init_replicas, sc.latency, prefetch=True)
    same = next((i for i, (x, y) in enumerate(zip(a, b)) if x.depth != y.depth), min(len(a), len(b)))
    assert [e.key() for e in a[:same]] == [e.key() for e in b[:same]]
    assert len(a) == len(b)


@settings(max_examples=120, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(scenarios(with_faults=True))
def test_native_equals_oracle_with_faults(case):
    sc, f = case
    r = parity.compare(sc, f)
    assert r.ok, r.mismatches[:2]


@settings(max_examples=200, deadline=None)
@given(st.integers(-20, 40), st.integers(0, 20), st.integers(0, 20), st.integers(0, 10), st.integers(0, 10))
def test_clamp_invariants(cur, max_, min_, up, down):
    """scale.go:62-69,89-97: a scale-up never exceeds max unless it was already above it; a
    scale-down never goes below min unless it was already below it."""
    p = oracle.Params(poll_ns=SECOND, up_cool_ns=0, down_cool_ns=0, up_msgs=10, down_msgs=0, up_pods=up,
                      down_pods=down, max_pods=max_, min_pods=min_)
    hi = oracle.simulate(p, [(0, traces.attrs(100))], traces.DEFAULT_NAMES, 1, cur, oracle.Latency(0, 0, 0))[0]
    lo = oracle.simulate(p, [(0, traces.attrs(0))], traces.DEFAULT_NAMES, 1, cur, oracle.Latency(0, 0, 0))[0]
    if cur >= max_:
        assert hi.up == "noop" and hi.replicas == cur
    else:
        assert hi.up == "scaled" and hi.replicas == min(cur + up, max_)
    if cur <= min_:
        assert lo.down == "noop" and lo.replicas == cur
    else:
        assert lo.down == "scaled" and lo.replicas == max(cur - down, min_)
