"""Reference-semantics oracle: the decision model of the reference, in its simplest form.

This is a deliberately naive, I/O-free restatement of /root/reference/main.go:35-78 plus
/root/reference/scale/scale.go:54-107 over a virtual clock. It shares no code with the native
control loop (csrc/core/runner.cc) so the parity harness compares two independent
implementations of SURVEY.md §3.3:

1. timers armed at ``Run()`` entry (main.go:37-38);
2. independent up/down timers;
3. a no-op at a bound refreshes that direction's timer (scale.go:62-65,89-92 + main.go:62,76);
4. a failure does not refresh it (main.go:57-60,71-74);
5. a cool-down skip or failed scale-up ``continue``s past the scale-down check (main.go:54,59);
6. proceed iff ``now >= last + cool`` (``After`` is strict; main.go:52,66), ``now`` re-read at
   every comparison, so API latency moves later comparisons;
7. asymmetric clamping with Go int32 arithmetic (scale.go:62-69,89-97);
8. depth is the 64-bit sum of the requested attributes (sqs.go:56-64);
9. the first poll happens one period after start (main.go:41), sleep-then-work (no ticker).

Time model (shared with the native in-memory fakes): the SQS trace is sampled at call start,
then every API call advances the clock by its latency.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Set, Tuple

INT32_MIN = -(1 << 31)


def int32(v: int) -> int:
    """Go ``int32(v)`` (two's-complement wrap)."""
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


def atoi(s: str) -> int:
    """strconv.Atoi on a 64-bit platform; raises ValueError like the reference's error path."""
    if s is None:
        raise ValueError("missing attribute")
    t = s
    if t[:1] in ("+", "-"):
        t = t[1:]
    if not t or not t.isascii() or not t.isdigit():
        raise ValueError(f'strconv.Atoi: parsing "{s}": invalid syntax')
    v = int(s)
    if v < -(1 << 63) or v > (1 << 63) - 1:
        raise ValueError(f'strconv.Atoi: parsing "{s}": value out of range')
    return v


@dataclass(frozen=True)
class Params:
    poll_ns: int
    up_cool_ns: int
    down_cool_ns: int
    up_msgs: int
    down_msgs: int
    up_pods: int = 1
    down_pods: int = 1
    max_pods: int = 8
    min_pods: int = 1


@dataclass(frozen=True)
class Latency:
    sqs_ns: int = 1_000_000
    get_ns: int = 1_000_000
    update_ns: int = 1_000_000


AttrMap = Dict[str, str]
Trace = Sequence[Tuple[int, AttrMap]]  # piecewise-constant (start_ns, attributes), sorted


@dataclass
class Event:
    """One poll, in the vocabulary the native runner reports (runner.h IterationRecord)."""

    index: int
    t_poll_ns: int
    depth: Optional[int]  # None when the depth read failed
    up: str = "none"  # none | cooldown | scaled | noop | failed
    down: str = "none"
    replicas: int = 0  # Deployment replicas after the poll
    up_replicas: Optional[int] = None  # replicas right after a scale-up write
    prefetched: bool = False  # a pipelined GET went out with this poll
    gets: int = 0  # Deployment GETs sent during the poll (pipelined + synchronous)

    def key(self) -> Tuple:
        return (self.index, self.depth, self.up, self.down, self.replicas)


@dataclass
class Faults:
    """Injected failures keyed by 1-based poll index."""

    sqs: Set[int] = field(default_factory=set)
    up_get: Set[int] = field(default_factory=set)
    up_update: Set[int] = field(default_factory=set)
    down_get: Set[int] = field(default_factory=set)
    down_update: Set[int] = field(default_factory=set)


def sample(trace: Trace, t: int) -> AttrMap:
    cur: AttrMap = {}
    for start, attrs in trace:
        if start <= t:
            cur = attrs
        else:
            break
    return cur


def depth_of(attrs: AttrMap, names: Sequence[str]) -> int:
    total = 0
    for n in names:
        total += atoi(attrs.get(n))  # type: ignore[arg-type]
    # Go int is 64-bit and wraps
    total &= (1 << 64) - 1
    return total - (1 << 64) if total >= 1 << 63 else total


def simulate(
    p: Params,
    trace: Trace,
    names: Sequence[str],
    polls: int,
    init_replicas: int,
    lat: Latency = Latency(),
    faults: Optional[Faults] = None,
    prefetch: bool = False,
    prefetch_always: bool = False,
) -> List[Event]:
    """Runs ``polls`` iterations of the reference loop on a virtual clock.

    ``prefetch`` models the pipelined read (``--pipeline-reads``): the Deployment GET is sent
    with the SQS call, so the first GET of a poll costs ``max(0, get - sqs)`` extra instead of
    ``get``, and an unused prefetch is drained at the end of the poll. The decision rules are
    unchanged -- only when ``now`` is read moves. The GET is only sent on polls whose gates
    would open on the previous depth (``prefetch_always`` sends it on every poll): see
    :func:`_likely`, restated from the rule in runner.h, not shared with it.
    """
    f = faults or Faults()
    import bisect

    starts = [start for start, _ in trace]

    def sample_at(t: int) -> AttrMap:  # sample() in O(log n): long traces (GPU sweep checks)
        i = bisect.bisect_right(starts, t) - 1
        return trace[i][1] if i >= 0 else {}

    st = {"now": 0, "last_up": 0, "last_down": 0, "replicas": int32(init_replicas)}  # main.go:37-38
    out: List[Event] = []
    seen = {"depth": None, "rtt": 0}  # prefetch gate inputs: last depth read, last SQS latency

    def _likely(t0: int) -> bool:
        at = t0 + seen["rtt"]
        up_open = st["last_up"] + p.up_cool_ns <= at
        down_open = st["last_down"] + p.down_cool_ns <= at
        d = seen["depth"]
        if d is None:
            return up_open or down_open
        if d >= p.up_msgs:  # the up gate either reads or `continue`s past the down check
            return up_open
        return down_open if d <= p.down_msgs else False

    def read(k: int, ev: Event, pf: dict, fail_set: Set[int]) -> bool:
        """One GET; returns False when it fails (injected fault)."""
        if pf["pending"]:
            pf["pending"] = False
            st["now"] = max(st["now"], pf["done"])
        else:
            st["now"] += lat.get_ns
            ev.gets += 1
        return k not in fail_set

    def scale(k: int, ev: Event, up: bool, pf: dict) -> bool:
        """ScaleUp/ScaleDown + timer refresh; False means `continue` (failure)."""
        if not read(k, ev, pf, f.up_get if up else f.down_get):
            setattr(ev, "up" if up else "down", "failed")
            return False
        r = st["replicas"]
        if up:
            if r >= int32(p.max_pods):  # scale.go:62
                ev.up = "noop"
            else:
                nxt = int32(r + int32(p.up_pods))
                nxt = int32(p.max_pods) if nxt > int32(p.max_pods) else nxt
                st["now"] += lat.update_ns
                if k in f.up_update:
                    ev.up = "failed"
                    return False
                st["replicas"] = nxt
                ev.up = "scaled"
                ev.up_replicas = nxt
            st["last_up"] = st["now"]  # main.go:62
        else:
            if r <= int32(p.min_pods):  # scale.go:89
                ev.down = "noop"
            else:
                nxt = int32(r - int32(p.down_pods))
                nxt = int32(p.min_pods) if nxt < int32(p.min_pods) else nxt
                st["now"] += lat.update_ns
                if k in f.down_update:
                    ev.down = "failed"
                    return False
                st["replicas"] = nxt
                ev.down = "scaled"
            st["last_down"] = st["now"]  # main.go:76
        return True

    def poll(k: int, ev: Event, pf: dict) -> None:
        attrs = sample_at(st["now"])
        st["now"] += lat.sqs_ns
        seen["rtt"] = lat.sqs_ns
        if k in f.sqs:
            return
        try:
            n = depth_of(attrs, names)
        except (ValueError, TypeError):
            return  # main.go:44-47
        ev.depth = n
        seen["depth"] = n
        if n >= p.up_msgs:  # main.go:51
            if st["last_up"] + p.up_cool_ns > st["now"]:  # main.go:52
                ev.up = "cooldown"
                return
            if not scale(k, ev, True, pf):
                return
        if n <= p.down_msgs:  # main.go:65
            if st["last_down"] + p.down_cool_ns > st["now"]:  # main.go:66
                ev.down = "cooldown"
                return
            scale(k, ev, False, pf)

    for k in range(1, polls + 1):
        st["now"] += max(p.poll_ns, 0)  # main.go:41 time.Sleep (<= 0: no sleep)
        ev = Event(index=k, t_poll_ns=st["now"], depth=None)
        out.append(ev)
        pf = {"pending": prefetch and (prefetch_always or _likely(st["now"])), "done": st["now"] + lat.get_ns}
        ev.prefetched = pf["pending"]
        ev.gets = int(ev.prefetched)
        poll(k, ev, pf)
        if pf["pending"]:  # drain an unused prefetch
            st["now"] = max(st["now"], pf["done"])
        ev.replicas = st["replicas"]
    return out


def reference_gets(events: Sequence[Event]) -> int:
    """Deployment GETs the reference sends on these polls: one per ScaleUp/ScaleDown call,
    i.e. per direction that got past its threshold and cool-down gates (scale.go:55,82)."""
    called = ("scaled", "noop", "failed")
    return sum((e.up in called) + (e.down in called) for e in events)


def scale_events(events: Sequence[Event]) -> List[Tuple[str, int, int]]:
    """(direction, poll index, replicas after) for every write -- the compact golden form."""
    out = []
    for e in events:
        if e.up == "scaled":
            out.append(("up", e.index, e.up_replicas))
        if e.down == "scaled":
            out.append(("down", e.index, e.replicas))
    return out
