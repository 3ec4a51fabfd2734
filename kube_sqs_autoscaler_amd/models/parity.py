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

from ..ops import native
from .oracle import Event, Faults, depth_of, simulate
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
        sqs_api = nat.TraceSqsApi(clock, [(t, dict(a)) for t, a in scenario.trace], lat.sqs_ns)
        kube = nat.FakeDeployments("default")
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
