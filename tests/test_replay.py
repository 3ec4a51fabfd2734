"""models/replay.py: recorded spans checked against the reference's decision rules."""
import json

import pytest

from kube_sqs_autoscaler_amd.models.oracle import Params
from kube_sqs_autoscaler_amd.models.replay import group_spans, replay_queue

MS = 1_000_000
P = Params(poll_ns=100 * MS, up_cool_ns=250 * MS, down_cool_ns=350 * MS, up_msgs=100, down_msgs=10, max_pods=4, min_pods=1)


def span(k, t0_ms, depth, up="none", down="none", before=-1, after=-1, total_ms=1, depth_ms=0.5):
    return {"poll": k, "ts": int((t0_ms + total_ms) * MS), "total_ns": int(total_ms * MS), "depth_ns": int(depth_ms * MS),
            "depth": depth, "up": up, "down": down, "replicas_before": before, "replicas_after": after, "queue": "q"}


def test_accepts_the_reference_sequence():
    # arm at 0; polls every ~101 ms; up cool-down 250 ms: polls 1-2 skip, poll 3 scales
    spans = [span(1, 100, 500, "cooldown"), span(2, 201, 500, "cooldown"), span(3, 302, 500, "scaled", before=1, after=2),
             span(4, 403, 500, "cooldown"), span(5, 504, 500, "cooldown"), span(6, 605, 500, "scaled", before=2, after=3),
             span(7, 706, 50), span(8, 807, None), span(9, 908, 0, down="scaled", before=3, after=2),
             span(10, 1009, 0, down="cooldown")]
    r = replay_queue(P, spans)
    assert r.ok and r.polls == 10 and r.checked == 10 and r.scale_writes == 3 and r.depth_errors == 1


@pytest.mark.parametrize("bad,msg", [
    (span(3, 302, 500, "cooldown"), "skipped for cool-down although"),
    (span(3, 240, 500, "scaled", before=1, after=2), "cool-down has"),
    (span(3, 302, 500, "scaled", before=1, after=3), "the reference writes 2"),
    (span(3, 302, 500, "noop", before=2), "below max"),
    (span(3, 302, 50, "scaled", before=1, after=2), "threshold does not hold"),
    (span(3, 302, None, "failed"), "depth read failed"),
])
def test_flags_decisions_the_reference_would_not_make(bad, msg):
    r = replay_queue(P, [span(1, 100, 500, "cooldown"), span(2, 201, 500, "cooldown"), bad])
    assert not r.ok and msg in r.mismatches[0][1]


def test_failed_call_does_not_refresh_the_timer_and_boundaries_are_counted():
    spans = [span(1, 100, 500, "cooldown"), span(2, 201, 500, "cooldown"), span(3, 302, 500, "failed"),
             span(4, 403, 500, "scaled", before=1, after=2)]  # the failure left the timer alone
    r = replay_queue(P, spans)
    assert r.ok and r.failed_calls == 1
    # a comparison 0.5 ms from the edge is not judged either way
    edge = [span(1, 100, 500, "cooldown"), span(2, 249.0, 500, "scaled", before=1, after=2, depth_ms=0.5)]
    r = replay_queue(P, edge, boundary_ns=2 * MS)
    assert r.ok and r.boundary == 1


def test_wire_run_replays_clean(nat, tmp_path):
    """A real-clock run over the wire (fakes, pipelined /scale), spans from the trace file."""
    from kube_sqs_autoscaler_amd.bench.latency import BenchEnv

    env = BenchEnv(2, poll_period_ns=20 * MS, prewarm_ns=200_000)
    try:
        trace = tmp_path / "t.jsonl"
        import os

        fd = os.open(trace, os.O_WRONLY | os.O_CREAT | os.O_APPEND)
        for r in env.runners:
            r.set_trace_fd(fd)
        env.run(40)
        os.close(fd)
        spans = [json.loads(l) for l in trace.read_text().splitlines()]
    finally:
        env.close()
    groups = group_spans(spans)
    assert len(groups) == 2
    p = Params(poll_ns=20 * MS, up_cool_ns=0, down_cool_ns=0, up_msgs=100, down_msgs=10, max_pods=8, min_pods=1)
    for q, ss in groups.items():
        r = replay_queue(p, ss)
        assert r.ok, r.mismatches[:3]
        assert r.polls == 40 and r.scale_writes == 40
