"""Replay recorded polls (``--trace-file`` spans) against the reference's decision rules.

The parity harness (models/parity.py) drives the loop on a virtual clock, where every input is
known in advance. A real run -- a soak against endpoints that fail, throttle and conflict --
has inputs no model can predict: the depth each poll read, which calls failed, what the
Deployment held when it was read, and the real time of every step. This module takes those
inputs from the spans and checks that every *decision* the loop made from them is the one the
reference makes (/root/reference/main.go:40-78, scale/scale.go:54-107):

* a depth read that failed ends the poll with no scale call (main.go:44-47);
* depth >= scale-up-messages: a cool-down skip iff ``last_up + C_up > now`` at the comparison
  (main.go:52, strict ``After``), which also skips the down check (``continue``, main.go:54);
  otherwise one ScaleUp call; a no-op only at or above max (scale.go:62), else
  ``min(before + up_pods, max)`` (scale.go:66-69); a failure ``continue``s (main.go:57-60);
  the timer is refreshed after a success or no-op (main.go:62), never after a failure;
* the same for depth <= scale-down-messages (main.go:65-77, scale.go:89-97);
* timers start at ``Run()`` entry, one poll period before the first poll (main.go:37-41).

``now`` at a comparison is the poll's start plus its SQS call (the span's ``depth_ns``); a timer
is refreshed at the end of its scale call. Both come from the spans to within microseconds, so a
comparison whose margin is under ``boundary_ns`` is not judged (either outcome is the
reference's for some scheduling of the same run) and is counted instead. Thresholds must not
overlap (up > down): with overlap one poll makes two calls whose split of the span's time is
not recorded.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from .oracle import Params, int32


@dataclass
class ReplayResult:
    queue: str
    polls: int = 0
    checked: int = 0           # polls whose every decision was judged
    boundary: int = 0          # cool-down comparisons within boundary_ns (not judged)
    depth_errors: int = 0
    failed_calls: int = 0      # scale calls that failed (an input: the endpoint's doing)
    scale_writes: int = 0
    mismatches: List[Tuple[int, str]] = field(default_factory=list)

    @property
    def ok(self) -> bool:
        return not self.mismatches


def _cool_gate(last: int, cool: int, now: int, boundary_ns: int) -> Optional[bool]:
    """True: proceed (now >= last + cool); False: cool-down skip; None: too close to call."""
    margin = now - (last + cool)
    if abs(margin) < boundary_ns:
        return None
    return margin >= 0


def replay_queue(p: Params, spans: Sequence[dict], boundary_ns: int = 2_000_000, queue: str = "") -> ReplayResult:
    """Checks one queue's spans (in poll order) against the reference's rules; see the module
    docstring. ``spans``: ``--trace-file`` objects (runner.cc ``iteration_json``)."""
    if p.up_msgs <= p.down_msgs:
        raise ValueError("replay needs non-overlapping thresholds (scale-up-messages > scale-down-messages)")
    res = ReplayResult(queue=queue)
    if not spans:
        return res
    t0_first = spans[0]["ts"] - spans[0]["total_ns"]
    last_up = last_down = t0_first - p.poll_ns  # Run() entry, main.go:37-38
    max_p, min_p = int32(p.max_pods), int32(p.min_pods)
    for s in spans:
        res.polls += 1
        k = s["poll"]
        t0 = s["ts"] - s["total_ns"]
        t_cmp = t0 + s["depth_ns"]
        t_end = t0 + s["total_ns"]
        judged = True

        def bad(msg: str) -> None:
            res.mismatches.append((k, msg))

        if s["depth"] is None:  # main.go:44-47
            res.depth_errors += 1
            if s["up"] != "none" or s["down"] != "none":
                bad(f"depth read failed but up={s['up']} down={s['down']}")
            res.checked += 1
            continue
        n = s["depth"]
        for direction, want in (("up", n >= p.up_msgs), ("down", n <= p.down_msgs)):
            got = s[direction]
            if not want:
                if got != "none":
                    bad(f"depth {n}: {direction}={got} but its threshold does not hold")
                continue
            last, cool = (last_up, p.up_cool_ns) if direction == "up" else (last_down, p.down_cool_ns)
            gate = _cool_gate(last, cool, t_cmp, boundary_ns)
            if gate is None:
                res.boundary += 1
                judged = False
            elif gate and got == "cooldown":
                bad(f"{direction} skipped for cool-down although {(t_cmp - last - cool) / 1e6:.3f} ms past it")
            elif not gate and got != "cooldown":
                bad(f"{direction}={got} although the cool-down has {(last + cool - t_cmp) / 1e6:.3f} ms left")
            if got == "cooldown":
                continue
            if got == "failed":
                res.failed_calls += 1
                continue  # main.go:57-60 / 71-74: no timer refresh
            before, after = s["replicas_before"], s["replicas_after"]
            if got == "noop":
                if direction == "up" and before >= 0 and before < max_p:
                    bad(f"up no-op at {before} replicas, below max {max_p}")
                if direction == "down" and before >= 0 and before > min_p:
                    bad(f"down no-op at {before} replicas, above min {min_p}")
            elif got == "scaled":
                res.scale_writes += 1
                if direction == "up":
                    want_after = max_p if int32(before + int32(p.up_pods)) > max_p else int32(before + int32(p.up_pods))
                    if before >= max_p:
                        bad(f"up wrote at {before} replicas, at or above max {max_p}")
                else:
                    want_after = min_p if int32(before - int32(p.down_pods)) < min_p else int32(before - int32(p.down_pods))
                    if before <= min_p:
                        bad(f"down wrote at {before} replicas, at or below min {min_p}")
                if after != want_after:
                    bad(f"{direction} wrote {after} replicas from {before}; the reference writes {want_after}")
            else:
                bad(f"unexpected {direction} outcome {got!r}")
                continue
            # main.go:62 / 76: refreshed after the call returned (the end of this poll: with
            # non-overlapping thresholds it makes one call)
            if direction == "up":
                last_up = t_end
            else:
                last_down = t_end
            break  # one direction per poll without overlap
        if judged:
            res.checked += 1
    return res


def group_spans(spans: Iterable[dict]) -> Dict[str, List[dict]]:
    """Spans by queue URL, each list in poll order."""
    out: Dict[str, List[dict]] = {}
    for s in spans:
        out.setdefault(s["queue"], []).append(s)
    for v in out.values():
        v.sort(key=lambda s: s["poll"])
    return out
