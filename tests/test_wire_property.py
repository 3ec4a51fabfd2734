"""Hypothesis over the production wire path: random policies and traces, every scale mode,
pipelined reads on or off -- ``Runner`` + SigV4 ``HttpSqsApi`` + ``KubeRestDeployments`` over
HTTP to the fakes must agree with the zero-latency oracle poll by poll (decisions, replicas,
poll times, GETs per poll). The apiserver sees the reference's GETs, plus -- with pipelined
reads -- a speculative one only where the depth moved since the previous poll
(/root/reference/main.go:35-78, scale/scale.go:55,82)."""
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from kube_sqs_autoscaler_amd.models import oracle, parity, traces
from kube_sqs_autoscaler_amd.utils.goflag import MILLISECOND, SECOND

periods = st.sampled_from([0, 1 * MILLISECOND, 1 * SECOND, 5 * SECOND, 7 * SECOND])
cools = st.sampled_from([0, 1 * SECOND, 5 * SECOND, 10 * SECOND, 30 * SECOND, 300 * SECOND])


@st.composite
def wire_scenarios(draw):
    p = oracle.Params(
        poll_ns=draw(periods), up_cool_ns=draw(cools), down_cool_ns=draw(cools),
        up_msgs=draw(st.integers(-5, 300)), down_msgs=draw(st.integers(-5, 300)),
        up_pods=draw(st.integers(0, 7)), down_pods=draw(st.integers(0, 7)),
        max_pods=draw(st.integers(0, 12)), min_pods=draw(st.integers(0, 12)),
    )
    n_seg = draw(st.integers(1, 5))
    starts = sorted(draw(st.lists(st.integers(0, 300), min_size=n_seg, max_size=n_seg)))
    trace = [(0 if i == 0 else s * SECOND, traces.attrs(draw(st.integers(0, 400)), draw(st.integers(0, 50)),
                                                       draw(st.integers(0, 50)))) for i, s in enumerate(starts)]
    names = list(draw(st.sampled_from([traces.DEFAULT_NAMES, traces.C5_NAMES])))
    return traces.Scenario("wireprop", "hypothesis", p, names, trace, draw(st.integers(0, 14)),
                           draw(st.integers(1, 40)), latency=oracle.Latency(0, 0, 0))


@pytest.fixture(scope="module")
def servers(nat):
    s, k = nat.FakeSqsServer(), nat.FakeKubeServer()
    s.start("127.0.0.1", 0, False)
    k.start("127.0.0.1", 0, False)
    yield s, k
    s.stop()
    k.stop()


@settings(max_examples=200, deadline=None, suppress_health_check=[HealthCheck.too_slow,
                                                                  HealthCheck.function_scoped_fixture])
@given(wire_scenarios(), st.sampled_from(["scale", "deployment", "patch"]), st.booleans())
def test_wire_path_equals_oracle(servers, sc, mode, prefetch):
    r = parity.run_wire(sc, mode, prefetch, servers=servers)
    assert r.ok, r.mismatches[:3]
    # The pipelined GET is sent on the previous poll's depth (Runner::action_likely): it is wasted
    # only on the first poll (no depth yet) or when the depth has moved since the previous poll.
    moves = sum(1 for a, b in zip(r.events, r.events[1:]) if a.depth != b.depth)
    assert r.reference_gets <= r.apiserver_gets <= r.reference_gets + (1 + moves if prefetch else 0)
    assert r.signature_failures == 0 and r.sqs_requests == sc.polls
