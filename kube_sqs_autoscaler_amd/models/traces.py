"""Synthetic queue-depth traces for the five BASELINE.json configs.

Each :class:`Scenario` is a complete, self-describing parity case: policy parameters, the
attribute names requested, a piecewise-constant SQS attribute trace, the initial replica
count and the number of polls to run. ``golden`` holds the scale events SURVEY.md Appendix C
derives by hand from /root/reference/main.go:35-78 -- the tests assert the oracle reproduces
them before the oracle is trusted to judge the native loop.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from ..config import DEFAULT_ATTRIBUTE_NAMES
from ..utils.goflag import MINUTE, SECOND
from .oracle import AttrMap, Latency, Params

DEFAULT_NAMES: List[str] = DEFAULT_ATTRIBUTE_NAMES.split(",")
C5_NAMES: List[str] = ["ApproximateNumberOfMessages", "ApproximateNumberOfMessagesNotVisible"]


def attrs(visible: int, delayed: int = 0, not_visible: int = 0) -> AttrMap:
    return {
        "ApproximateNumberOfMessages": str(visible),
        "ApproximateNumberOfMessagesDelayed": str(delayed),
        "ApproximateNumberOfMessagesNotVisible": str(not_visible),
    }


@dataclass
class Scenario:
    name: str
    description: str
    params: Params
    names: List[str]
    trace: List[Tuple[int, AttrMap]]
    init_replicas: int
    polls: int
    latency: Latency = field(default_factory=Latency)
    # (direction, poll time in whole seconds, replicas after) from SURVEY.md Appendix C
    golden: Optional[List[Tuple[str, int, int]]] = None


def _defaults(**kw) -> Params:
    base = dict(
        poll_ns=5 * SECOND,
        up_cool_ns=10 * SECOND,
        down_cool_ns=30 * SECOND,
        up_msgs=100,
        down_msgs=10,
        up_pods=1,
        down_pods=1,
        max_pods=8,
        min_pods=1,
    )
    base.update(kw)
    return Params(**base)


def c1_noop() -> Scenario:
    return Scenario(
        name="c1_constant_zero_min_eq_max",
        description="mock-SQS + fake kube, constant 0 msgs, min=max=1 (no-op plumbing loop)",
        params=_defaults(max_pods=1, min_pods=1),
        names=DEFAULT_NAMES,
        trace=[(0, attrs(0))],
        init_replicas=1,
        polls=120,
        golden=[],
    )


def c2_step() -> Scenario:
    up = [("up", 60 + 10 * i, 2 + i) for i in range(7)]
    down = [("down", 180 + 30 * i, 7 - i) for i in range(7)]
    return Scenario(
        name="c2_step_0_200_0",
        description="single queue step trace 0->200->0 msgs, scale-up-messages=100 / scale-down-messages=10",
        params=_defaults(),
        names=DEFAULT_NAMES,
        trace=[(0, attrs(0)), (60 * SECOND, attrs(200)), (180 * SECOND, attrs(0))],
        init_replicas=1,
        polls=100,
        golden=up + down,
    )


def c3_cooldown_bursty() -> Scenario:
    trace: List[Tuple[int, AttrMap]] = []
    for base in range(0, 1000, 100):
        trace.append((base * SECOND, attrs(500)))
        trace.append(((base + 20) * SECOND, attrs(0)))
    return Scenario(
        name="c3_cooldown_bursty",
        description="poll-period=5s, scale-up-cool-down=5m, scale-down-cool-down=30s, bursty trace",
        params=_defaults(up_cool_ns=5 * MINUTE, down_cool_ns=30 * SECOND),
        names=DEFAULT_NAMES,
        trace=trace,
        init_replicas=1,
        polls=140,
        golden=[("up", 300, 2), ("down", 320, 1), ("up", 600, 2), ("down", 620, 1)],
    )


def c4_clamp() -> Scenario:
    return Scenario(
        name="c4_clamp_10k_backlog",
        description="min-pods=1 max-pods=8 clamp under 10k-msg backlog (8xMI355X GPU-worker pod cap)",
        params=_defaults(),
        names=DEFAULT_NAMES,
        trace=[(0, attrs(10_000))],
        init_replicas=1,
        polls=40,
        golden=[("up", 10 * (i + 1), 2 + i) for i in range(7)],
    )


def c5_multi_attr() -> Scenario:
    # Delayed is large throughout but NOT requested, so it must not count. Visible+NotVisible
    # is 0 -> 150 (60..180 s) -> 5, i.e. C2-shaped on the two-attribute sum.
    trace = [
        (0, attrs(0, delayed=5000, not_visible=0)),
        (60 * SECOND, attrs(100, delayed=5000, not_visible=50)),
        (180 * SECOND, attrs(3, delayed=5000, not_visible=2)),
    ]
    up = [("up", 60 + 10 * i, 2 + i) for i in range(7)]
    down = [("down", 180 + 30 * i, 7 - i) for i in range(7)]
    return Scenario(
        name="c5_multi_attribute_sum",
        description="attribute-names=ApproximateNumberOfMessages,ApproximateNumberOfMessagesNotVisible multi-attr sum",
        params=_defaults(),
        names=C5_NAMES,
        trace=trace,
        init_replicas=1,
        polls=100,
        golden=up + down,
    )


def baseline_scenarios() -> List[Scenario]:
    return [c1_noop(), c2_step(), c3_cooldown_bursty(), c4_clamp(), c5_multi_attr()]


def reference_test_scenarios() -> Dict[str, dict]:
    """The six loop tests of /root/reference/main_test.go as (params, depth, check time, expect).

    The mocks start at 100/100/100 and each test replaces the attributes right after
    ``go Run``; the first poll is one period later (main.go:41), so the depth is constant for
    the whole observation window.
    """
    S = SECOND
    one = dict(poll_ns=1 * S, up_cool_ns=1 * S, down_cool_ns=1 * S)
    five = dict(poll_ns=5 * S, up_cool_ns=10 * S, down_cool_ns=10 * S)
    return {
        # main_test.go:19-54
        "TestRunReachMinReplicas": dict(params=Params(**one, up_msgs=100, down_msgs=3, max_pods=5, min_pods=1),
                                        depth=(1, 1, 1), init=3, check_s=10, expect=1),
        # main_test.go:56-91
        "TestRunReachMaxReplicas": dict(params=Params(**one, up_msgs=300, down_msgs=10, max_pods=5, min_pods=1),
                                        depth=(100, 100, 100), init=3, check_s=10, expect=5),
        # main_test.go:93-127
        "TestRunScaleUpCoolDown": dict(params=Params(**five, up_msgs=300, down_msgs=10, max_pods=5, min_pods=1),
                                       depth=(100, 100, 100), init=3, check_s=15, expect=4),
        # main_test.go:129-163
        "TestRunScaleDownCoolDown": dict(params=Params(**five, up_msgs=100, down_msgs=3, max_pods=5, min_pods=1),
                                         depth=(1, 1, 1), init=3, check_s=15, expect=2),
        # main_test.go:165-201
        "TestRunReachMinReplicasWithScalingPodNum": dict(
            params=Params(**one, up_msgs=100, down_msgs=3, up_pods=100, down_pods=100, max_pods=100, min_pods=1),
            depth=(1, 1, 1), init=100, check_s=3, expect=1),
        # main_test.go:203-239
        "TestRunReachMaxReplicasWithScalingPodNum": dict(
            params=Params(**one, up_msgs=100, down_msgs=3, up_pods=100, down_pods=100, max_pods=100, min_pods=1),
            depth=(100, 100, 100), init=3, check_s=3, expect=100),
    }


def golden_from_events(events: Sequence, poll_ns: int) -> List[Tuple[str, int, int]]:
    """Scale events with poll times rounded down to whole seconds (drift is < 1 s)."""
    out = []
    for e in events:
        t = e.t_poll_ns // SECOND
        if e.up == "scaled":
            out.append(("up", t, e.up_replicas))
        if e.down == "scaled":
            out.append(("down", t, e.replicas))
    return out
