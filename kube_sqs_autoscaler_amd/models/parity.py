"""Decision-parity harness: native control loop vs the reference-semantics oracle.

The native side is the production code path -- ``Runner`` (csrc/core/runner.cc), the real
``SqsClient`` attribute summing (csrc/core/sqs.cc) and ``PodAutoScaler`` clamp arithmetic
(csrc/core/kube.cc) -- driven by a ``VirtualClock`` and in-memory fakes with the same latency
model as :mod:`.oracle`. A scenario passes when every poll agrees on
``(index, depth, up action, down action, replicas after)``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

from ..ops import fakes, native
from .oracle import Event, Faults, Latency, depth_of, simulate
from .traces import Scenario

def _records_to_events(recs: Sequence[dict], init_replicas: int) -> List[Event]:
    out = []
    replicas = init_replicas
    for r in recs:
        # the native record carries replicas as read/written during the poll (-1: no GET)
        if r["replicas_after"] >= 0:
            replicas = r["replicas_after"]
        ev = Event(
            index=r["index"],
            t_poll_ns=r["t_poll"],
            depth=r["depth"] if r["depth_ok"] else None,
            up=r["up"],
            down=r["down"],
            replicas=replicas,
            prefetched=r["prefetched"],
            gets=r["gets"],
        )
        if r["up"] == "scaled" and r["down"] != "scaled":  # else the record holds the post-down count
            ev.up_replicas = replicas
        out.append(ev)
    return out


class _PollCounter:
    def __init__(self) -> None:
        self.poll = 0
        self.depth: Optional[int] = None
        self.gets_this_poll = 0


def _faulty_fakes(nat, clock, scenario: Scenario, faults: Faults, counter: _PollCounter):
    """Python fakes (plugged into the native seams) that fail on specific polls."""
    trace = sorted(scenario.trace, key=lambda s: s[0])
    lat = scenario.latency
    params = scenario.params

    class Sqs(nat.SqsApi):
        def get_queue_attributes(self, url, names):
            counter.poll += 1
            counter.gets_this_poll = 0
            t = clock.now()
            cur = {}
            for start, a in trace:
                if start <= t:
                    cur = a
                else:
                    break
            clock.advance(lat.sqs_ns)
            if counter.poll in faults.sqs:
                raise RuntimeError("injected SQS failure")
            return dict(cur)

    class Deployments(nat.DeploymentApi):
        def __init__(self, replicas: int):
            super().__init__()
            self.replicas = replicas
            self.rv = 1
            self.direction = "up"

        def get(self, name):
            counter.gets_this_poll += 1
            clock.advance(lat.get_ns)
            # first GET of a poll is the scale-up one iff the up branch ran
            self.direction = "up" if (counter.gets_this_poll == 1 and self._up_branch()) else "down"
            if counter.poll in (faults.up_get if self.direction == "up" else faults.down_get):
                raise RuntimeError("injected GET failure")
            return nat.ScaleObject(self.replicas, True, str(self.rv), "")

        def _up_branch(self) -> bool:
            return counter.depth is not None and counter.depth >= params.up_msgs

        def update(self, name, obj, replicas):
            clock.advance(lat.update_ns)
            if counter.poll in (faults.up_update if self.direction == "up" else faults.down_update):
                raise RuntimeError("injected PUT failure")
            self.replicas = replicas
            self.rv += 1

    return Sqs(), Deployments


def run_native(
    scenario: Scenario,
    faults: Optional[Faults] = None,
    log_sink=None,
    prefetch: bool = False,
    prefetch_always: bool = False,
) -> List[Event]:
    """Runs ``scenario`` through the native control loop and returns per-poll events."""
    nat = native()
    p = scenario.params
    lat = scenario.latency
    clock = nat.VirtualClock(0)
    log = nat.Logger()
    log.set_time_source(clock)
    if log_sink is None:
        log.set_level("panic")
    else:
        log.set_sink(log_sink)

    if faults is None:
        sqs_api = fakes().TraceSqsApi(clock, [(t, dict(a)) for t, a in scenario.trace], lat.sqs_ns)
        kube = fakes().FakeDeployments("default")
        kube.add("target", scenario.init_replicas)
        kube.set_latency(clock, lat.get_ns)
        kube.enable_pipelining(prefetch)
        if lat.update_ns != lat.get_ns:
            raise ValueError("FakeDeployments models one latency for GET and PUT")
        counter = None
    else:
        if prefetch:
            raise ValueError("fault-injection parity runs without pipelined reads")
        counter = _PollCounter()
        sqs_api, dep_cls = _faulty_fakes(nat, clock, scenario, faults, counter)
        kube = dep_cls(scenario.init_replicas)

    sqs = nat.SqsClient(sqs_api, "https://sqs.local/000000000000/parity", list(scenario.names))
    scaler = nat.PodAutoScaler(kube, "target", "default", p.max_pods, p.min_pods, p.up_pods, p.down_pods, log, clock)
    cfg = nat.LoopConfig()
    cfg.poll_period_ns = p.poll_ns
    cfg.scale_up_cool_down_ns = p.up_cool_ns
    cfg.scale_down_cool_down_ns = p.down_cool_ns
    cfg.scale_up_messages = p.up_msgs
    cfg.scale_down_messages = p.down_msgs
    cfg.prefetch = prefetch
    cfg.prefetch_always = prefetch_always
    runner = nat.Runner(cfg, sqs, scaler, clock, log)
    runner.arm()
    if counter is None:
        recs = runner.steps(scenario.polls)
    else:
        recs = []
        for _ in range(scenario.polls):
            # the depth the fake will report is needed to attribute GETs to a direction
            t_next = clock.now() + max(p.poll_ns, 0)
            cur = {}
            for start, a in sorted(scenario.trace, key=lambda s: s[0]):
                if start <= t_next:
                    cur = a
            try:
                counter.depth = depth_of(cur, scenario.names)
            except (ValueError, TypeError):
                counter.depth = None
            recs.append(runner.step())
    return _records_to_events(recs, scenario.init_replicas)


@dataclass
class ParityResult:
    scenario: str
    polls: int
    agree: int
    mismatches: List[Tuple[Event, Event]] = field(default_factory=list)
    scale_events: int = 0

    @property
    def fraction(self) -> float:
        return self.agree / self.polls if self.polls else 1.0

    @property
    def ok(self) -> bool:
        return self.agree == self.polls


def compare(scenario: Scenario, faults: Optional[Faults] = None, prefetch: bool = False,
            prefetch_always: bool = False) -> ParityResult:
    """Poll-by-poll agreement; with ``prefetch`` the gate's send/skip choice must agree too."""
    ref = simulate(
        scenario.params, scenario.trace, scenario.names, scenario.polls, scenario.init_replicas, scenario.latency, faults,
        prefetch=prefetch, prefetch_always=prefetch_always,
    )
    got = run_native(scenario, faults, prefetch=prefetch, prefetch_always=prefetch_always)
    res = ParityResult(scenario=scenario.name, polls=len(ref), agree=0)
    for a, b in zip(ref, got):
        if a.key() == b.key() and a.t_poll_ns == b.t_poll_ns and a.prefetched == b.prefetched \
                and a.gets == b.gets:
            res.agree += 1
        else:
            res.mismatches.append((a, b))
        res.scale_events += (a.up == "scaled") + (a.down == "scaled")
    if len(got) != len(ref):
        res.agree = min(res.agree, len(got))
    return res


# ---------------------------------------------------------------------------------------
# Wire-path parity: the production clients against the localhost fake endpoints.

WIRE_LATENCY = Latency(0, 0, 0)


@dataclass
class WireParityResult(ParityResult):
    mode: str = "scale"
    prefetch: bool = False
    apiserver_gets: int = 0        # GETs the fake apiserver served
    apiserver_writes: int = 0
    reference_gets: int = 0        # what the reference would send on this trace
    sqs_requests: int = 0
    signature_failures: int = 0
    events: List[Event] = field(default_factory=list)

    @property
    def apiserver_requests_per_poll(self) -> float:
        return (self.apiserver_gets + self.apiserver_writes) / self.polls if self.polls else 0.0


def run_wire(scenario: Scenario, mode: str = "scale", prefetch: bool = True, servers=None,
             prefetch_always: bool = False) -> WireParityResult:
    """Runs ``scenario`` through the production wire path and compares it with the oracle.

    ``Runner`` + SigV4-signing ``HttpSqsApi`` + ``KubeRestDeployments`` (``mode``: ``scale``,
    ``deployment`` or ``patch``; ``prefetch``: --pipeline-reads) talk HTTP to
    ``FakeSqsServer`` (signature verified) and ``FakeKubeServer``. Time is a ``VirtualClock``
    that only the poll sleeps advance, so the reference model is the zero-latency oracle;
    before each poll the fake SQS is set to the trace's attributes at that poll's time (the
    per-poll attribute schedule). Agreement is per poll on (depth, up/down action, replicas),
    poll time, whether the pipelined GET was sent and how many GETs the poll made; the
    apiserver's own request counters must add up to the same GETs and writes.
    """
    from ..autoscaler import new_deployment_api, new_sqs_api
    from ..config import DEFAULT_POLL_PREWARM_NS
    from ..kube.config import RestConfig
    from ..sqs.credentials import static_provider
    from .oracle import reference_gets, sample

    nat = native()
    akid, secret, region, token = "AKIDPARITY", "parity/secret", "us-east-1", "parity-token"
    own = servers is None
    if own:
        sqs_srv = fakes().FakeSqsServer()
        sqs_srv.start("127.0.0.1", 0, False)
        kube_srv = fakes().FakeKubeServer()
        kube_srv.start("127.0.0.1", 0, False)
    else:
        sqs_srv, kube_srv = servers
    sqs_srv.require_signature(akid, secret, region)
    kube_srv.require_token(token)
    p = scenario.params
    try:
        clock = nat.VirtualClock(0)
        log = nat.Logger()
        log.set_time_source(clock)
        log.set_level("panic")
        ns = "parity"
        name = f"{scenario.name}-{mode}-{int(prefetch)}"
        kube_srv.add_deployment(ns, name, scenario.init_replicas)
        url = f"{sqs_srv.url}/000000000000/{name}"
        kube_api = new_deployment_api(RestConfig(host=kube_srv.url, bearer_token=token), ns, mode, clock=clock)
        sqs_api = new_sqs_api(region, clock, endpoint=sqs_srv.url, credentials=static_provider(akid, secret),
                              environ={})
        sqs = nat.SqsClient(sqs_api, url, list(scenario.names))
        scaler = nat.PodAutoScaler(kube_api, name, ns, p.max_pods, p.min_pods, p.up_pods, p.down_pods, log, clock)
        cfg = nat.LoopConfig()
        cfg.poll_period_ns = p.poll_ns
        cfg.scale_up_cool_down_ns = p.up_cool_ns
        cfg.scale_down_cool_down_ns = p.down_cool_ns
        cfg.scale_up_messages = p.up_msgs
        cfg.scale_down_messages = p.down_msgs
        cfg.prefetch = prefetch
        cfg.prefetch_always = prefetch_always
        cfg.prewarm_ns = DEFAULT_POLL_PREWARM_NS  # the CLI's pre-poll warm-up (dials before the pipelined GET)
        runner = nat.Runner(cfg, sqs, scaler, clock, log)
        trace = sorted(scenario.trace, key=lambda s: s[0])
        gets0, writes0, sqs0, sig0 = kube_srv.gets(), kube_srv.writes(), sqs_srv.requests(), sqs_srv.signature_failures()
        runner.arm()
        recs = []
        for _ in range(scenario.polls):
            sqs_srv.set_attributes(url, dict(sample(trace, clock.now() + max(p.poll_ns, 0))))
            recs.append(runner.step())
        got = _records_to_events(recs, scenario.init_replicas)
        for e, r in zip(got, recs):
            e.gets = r["gets"]
        ref = simulate(p, trace, scenario.names, scenario.polls, scenario.init_replicas, WIRE_LATENCY, prefetch=prefetch,
                       prefetch_always=prefetch_always)
        res = WireParityResult(scenario=scenario.name, polls=len(ref), agree=0, mode=mode, prefetch=prefetch)
        res.events = got
        for a, b in zip(ref, got):
            if (a.key() == b.key() and a.t_poll_ns == b.t_poll_ns and a.prefetched == b.prefetched
                    and a.gets == b.gets):
                res.agree += 1
            else:
                res.mismatches.append((a, b))
            res.scale_events += (a.up == "scaled") + (a.down == "scaled")
        res.apiserver_gets = kube_srv.gets() - gets0
        res.apiserver_writes = kube_srv.writes() - writes0
        res.sqs_requests = sqs_srv.requests() - sqs0
        res.signature_failures = sqs_srv.signature_failures() - sig0
        res.reference_gets = reference_gets(simulate(p, trace, scenario.names, scenario.polls, scenario.init_replicas,
                                                     WIRE_LATENCY))
        expected_writes = sum((e.up == "scaled") + (e.down == "scaled") for e in ref)
        if (res.apiserver_gets != sum(e.gets for e in got) or res.apiserver_writes != expected_writes
                or res.sqs_requests != scenario.polls or res.signature_failures):
            res.agree = min(res.agree, res.polls - 1)  # the servers saw traffic the records do not explain
        return res
    finally:
        if own:
            sqs_srv.stop()
            kube_srv.stop()


WIRE_CONFIGS = (("scale", True, False), ("scale", False, False), ("deployment", False, False),
                ("scale", True, True))


def wire_summary(configs=WIRE_CONFIGS) -> dict:
    """Wire-path parity over the five Appendix C scenarios for each (mode, pipelined,
    pipelined-on-every-poll) config, with the apiserver traffic next to what the reference
    would send. The last default row is the round-1 behaviour (a speculative GET per poll)."""
    from . import traces

    nat = native()
    sqs_srv, kube_srv = fakes().FakeSqsServer(), fakes().FakeKubeServer()
    sqs_srv.start("127.0.0.1", 0, False)
    kube_srv.start("127.0.0.1", 0, False)
    out = {}
    try:
        for mode, pf, always in configs:
            key = f"{mode}{'_pipelined' if pf else ''}{'_every_poll' if always else ''}"
            rows, agree, polls = {}, 0, 0
            for sc in traces.baseline_scenarios():
                r = run_wire(sc, mode, pf, servers=(sqs_srv, kube_srv), prefetch_always=always)
                rows[sc.name] = {"agree": f"{r.agree}/{r.polls}", "apiserver_gets": r.apiserver_gets,
                                 "reference_gets": r.reference_gets, "writes": r.apiserver_writes,
                                 "apiserver_requests_per_poll": round(r.apiserver_requests_per_poll, 4)}
                agree += r.agree
                polls += r.polls
            out[key] = {"agree": f"{agree}/{polls}", "scenarios": rows}
    finally:
        sqs_srv.stop()
        kube_srv.stop()
    return out
