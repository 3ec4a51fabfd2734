"""Decision parity over the production wire path (VERDICT r01 "next round" #3).

The five Appendix C scenarios run through ``Runner`` + ``HttpSqsApi`` (SigV4 verified by the
fake) + ``KubeRestDeployments`` against ``FakeSqsServer`` / ``FakeKubeServer`` on a
``VirtualClock``, and are compared poll by poll with the zero-latency oracle -- including
whether the pipelined GET was sent and how many GETs each poll made -- and with the
SURVEY.md Appendix C goldens. The apiserver's own counters must show exactly the Deployment
GETs the reference sends on the same trace (/root/reference/scale/scale.go:55,82).
"""
import pytest

from kube_sqs_autoscaler_amd.models import parity, traces


@pytest.fixture(scope="module")
def servers(nat):
    s, k = nat.FakeSqsServer(), nat.FakeKubeServer()
    s.start("127.0.0.1", 0, False)
    k.start("127.0.0.1", 0, False)
    yield s, k
    s.stop()
    k.stop()


@pytest.mark.parametrize("mode,prefetch", [("scale", True), ("scale", False), ("deployment", False),
                                           ("deployment", True), ("patch", True)])
@pytest.mark.parametrize("sc", traces.baseline_scenarios(), ids=lambda s: s.name)
def test_wire_parity(servers, sc, mode, prefetch):
    r = parity.run_wire(sc, mode, prefetch, servers=servers)
    assert r.ok, r.mismatches[:3]
    assert traces.golden_from_events(r.events, sc.params.poll_ns) == sc.golden
    assert r.apiserver_gets == r.reference_gets  # no speculative reads beyond the reference's
    assert r.signature_failures == 0 and r.sqs_requests == sc.polls


def test_c1_idle_queue_apiserver_footprint(servers):
    sc = traces.c1_noop()
    gated = parity.run_wire(sc, "scale", True, servers=servers)
    every = parity.run_wire(sc, "scale", True, servers=servers, prefetch_always=True)
    assert gated.ok and every.ok
    assert (gated.apiserver_gets, gated.reference_gets, every.apiserver_gets) == (20, 20, 120)


def test_wire_summary_shape(nat):
    out = parity.wire_summary(configs=(("scale", True, False),))
    assert out["scale_pipelined"]["agree"] == "500/500"
    c1 = out["scale_pipelined"]["scenarios"]["c1_constant_zero_min_eq_max"]
    assert c1["apiserver_gets"] == c1["reference_gets"] == 20
