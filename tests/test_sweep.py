"""What-if policy sweep: the native simulator (CPU path here, gfx950 kernel in test_gpu.py)
must reproduce the reference-semantics oracle exactly."""
import json

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from kube_sqs_autoscaler_amd.tune import sweep
from kube_sqs_autoscaler_amd.tune.__main__ import main as tune_main, parse_values
from kube_sqs_autoscaler_amd.utils.goflag import SECOND, parse_duration

S = SECOND


def step_trace():
    return sweep.Trace.from_segments([(0, 0), (60 * S, 200), (180 * S, 0), (400 * S, 5000), (500 * S, 3)])


def test_grid_shape_and_order():
    p = sweep.grid(poll_ns=[1 * S, 5 * S], up_msgs=[10, 20, 30])
    assert p.shape == (9, 6)
    assert list(p[0]) == [S, S, S, 5 * S, 5 * S, 5 * S]  # poll period outermost
    assert list(p[3]) == [10, 20, 30, 10, 20, 30]
    assert (p[7] == 8).all()  # default max-pods


def test_reference_defaults_match_appendix_c2():
    """Defaults on the C2 step trace: 7 ups (60..120 s) then 7 downs -- SURVEY.md Appendix C."""
    tr = sweep.Trace.from_segments([(0, 0), (60 * S, 200), (180 * S, 0)])
    r = sweep.run(tr, sweep.grid(), 1, 500 * S, device="cpu").row(0)
    assert r["ups"] == 7 and r["downs"] == 7 and r["first_up_ns"] // S == 60 and r["final_replicas"] == 1


def test_cpu_equals_oracle_on_a_grid():
    tr = step_trace()
    p = sweep.grid(poll_ns=[1 * S, 5 * S], up_cool_ns=[0, 10 * S, 300 * S], down_cool_ns=[10 * S, 30 * S],
                   up_msgs=[50, 300], down_msgs=[3, 10], up_pods=[1, 3], max_pods=[4, 8])
    res = sweep.run(tr, p, 1, 900 * S, device="cpu")
    for i in range(len(res)):
        o = sweep.oracle_row(tr, res.config(i), 1, 900 * S, (10**6, 10**6, 10**6))
        assert {k: res.row(i)[k] for k in o} == o, res.config(i)


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(
    segs=st.lists(st.tuples(st.integers(1, 600), st.integers(0, 600)), min_size=0, max_size=8),
    d0=st.integers(0, 600),
    poll=st.sampled_from([500_000_000, S, 5 * S, 7 * S]),
    up_cool=st.sampled_from([0, S, 10 * S, 60 * S]), down_cool=st.sampled_from([0, 5 * S, 30 * S]),
    up_msgs=st.integers(-5, 400), down_msgs=st.integers(-5, 400), up_pods=st.integers(-2, 5),
    down_pods=st.integers(-2, 5), max_pods=st.integers(0, 12), min_pods=st.integers(0, 12),
    init=st.integers(0, 14), lat_ms=st.sampled_from([0, 1, 3]), horizon_s=st.integers(1, 900),
)
def test_cpu_equals_oracle_property(segs, d0, poll, up_cool, down_cool, up_msgs, down_msgs, up_pods, down_pods,
                                    max_pods, min_pods, init, lat_ms, horizon_s):
    tr = sweep.Trace.from_segments([(0, d0)] + sorted((t * S, d) for t, d in segs))
    cfg = dict(poll_ns=[poll], up_cool_ns=[up_cool], down_cool_ns=[down_cool], up_msgs=[up_msgs],
               down_msgs=[down_msgs], up_pods=[up_pods], down_pods=[down_pods], max_pods=[max_pods], min_pods=[min_pods])
    lat = (lat_ms * 10**6,) * 3
    o = None
    for skip in ("on", "off"):  # the steady-stretch skip adds a stretch at once: same results
        res = sweep.run(tr, sweep.grid(**cfg), init, horizon_s * S, lat, device="cpu", skip=skip)
        o = o or sweep.oracle_row(tr, res.config(0), init, horizon_s * S, lat)
        assert {k: res.row(0)[k] for k in o} == o, skip


def test_work_budget_guard():
    with pytest.raises(ValueError, match="sweep too large"):
        sweep.run(step_trace(), sweep.grid(poll_ns=[1], up_msgs=list(range(5000))), 1, 10**18, (0, 0, 0), device="cpu")
    with pytest.raises(ValueError, match="zero poll period"):
        sweep.run(step_trace(), sweep.grid(poll_ns=[0]), 1, 10 * S, (0, 0, 0), device="cpu")


def test_trace_loaders(tmp_path):
    spans = tmp_path / "s.jsonl"
    spans.write_text("\n".join(json.dumps({"ts": 10**12 + i * 5 * S, "depth": d, "queue": "q", "deployment": "ns/d"})
                               for i, d in enumerate([0, 0, 200, 200, 0])) + "\n")
    tr = sweep.Trace.from_spans(str(spans))
    assert list(tr.t_ns) == [0, 5 * S, 10 * S, 15 * S, 20 * S] and list(tr.depth) == [0, 0, 200, 200, 0]
    csv = tmp_path / "t.csv"
    csv.write_text("seconds,depth\n100,5\n160,50\n")
    tr = sweep.Trace.from_csv(str(csv))
    assert list(tr.t_ns) == [0, 60 * S] and list(tr.depth) == [5, 50]


def test_parse_values():
    assert parse_values("10s:30s:10s", parse_duration) == [10 * S, 20 * S, 30 * S]
    from kube_sqs_autoscaler_amd.utils.goflag import parse_int

    assert parse_values("1,0x10", parse_int) == [1, 16]


def test_tune_cli(tmp_path, capsys):
    csv = tmp_path / "t.csv"
    csv.write_text("0,0\n60,200\n180,0\n400,5000\n500,3\n")
    rc = tune_main(["--trace", str(csv), "--horizon", "15m", "--grid", "scale-up-cool-down=0s:60s:10s",
                    "--grid", "scale-up-messages=50,100,300", "--grid", "max-pods=4,8", "--objective", "pod_ms",
                    "--top", "3", "--device", "cpu", "--json"])
    assert rc == 0
    lines = [json.loads(l) for l in capsys.readouterr().out.splitlines()]
    assert lines[0]["configs"] == 7 * 3 * 2 and lines[0]["reference_defaults"]["ups"] > 0
    assert lines[0]["steady_skip"] is True  # 5 segments over 900 s: 180 s each under the 5 s poll
    pods = [l["pod_ms"] for l in lines[1:]]
    assert len(pods) == 3 and pods == sorted(pods)


def test_pareto_front():
    pod = np.array([5, 1, 3, 2, 4, 1])
    bl = np.array([1, 9, 4, 8, 2, 7])
    f = sweep.pareto_front(pod, bl)
    # (pod, backlog): (1,7) (3,4) (4,2) (5,1); (1,9) and (2,8) are dominated by (1,7)
    assert list(f) == [5, 2, 4, 0]


def test_extreme_cool_downs_and_periods_do_not_overflow(nat):
    """Cool-downs and poll periods near the int64 limit: the simulator clamps them (no signed
    overflow) and still agrees with the oracle, which has unbounded integers."""
    import numpy as np

    from kube_sqs_autoscaler_amd.tune import sweep

    S = 1_000_000_000
    tr = sweep.Trace.from_segments([(0, 500), (60 * S, 0)])
    big = 2**63 - 1
    grid = sweep.grid(poll_ns=[5 * S, big], up_cool_ns=[0, big, -big], down_cool_ns=[0, big], max_pods=[8])
    r = sweep.run(tr, grid, 1, 300 * S, device="cpu")
    for j in range(grid.shape[1]):
        want = sweep.oracle_row(tr, r.config(j), 1, 300 * S, (1_000_000, 1_000_000, 1_000_000))
        got = {k: int(r.out[k][j]) for k in want}
        assert got == want, (r.config(j), got, want)
    assert np.all(r.out["polls"][grid[0] == big] == 0)


# ---- millisecond clock (policy_sim.h simulate_ms) against the nanosecond one ----------------


def _both_clocks(tr, grid, init, horizon, lat):
    """Both clocks, each with and without the steady-stretch skip: the same results."""
    a = sweep.run(tr, grid, init, horizon, lat, device="cpu", clock="auto", skip="on")
    assert a.skip
    for clock, skip in (("ns", "on"), ("auto", "off"), ("ns", "off")):
        b = sweep.run(tr, grid, init, horizon, lat, device="cpu", clock=clock, skip=skip)
        assert b.ms_clock == (clock == "auto" and a.ms_clock) and b.skip == (skip == "on")
        for k in a.out:
            assert np.array_equal(a.out[k], b.out[k]), (k, clock, skip)
    return a


@settings(max_examples=200, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(
    # trace boundaries anywhere (sub-ms too): the ms clock rounds them up
    segs=st.lists(st.tuples(st.integers(1, 400 * 10**9), st.integers(0, 800)), min_size=0, max_size=12),
    d0=st.integers(0, 800),
    poll_ms=st.integers(1, 9000),
    # cool-downs at any ns, negative ones too, and past every bound
    cools=st.lists(st.one_of(st.integers(-(10**12), 10**12), st.sampled_from([0, 1, -1, 999_999, 1_000_001,
                                                                              2**62, -(2**62)])), min_size=2, max_size=2),
    up_msgs=st.one_of(st.integers(-5, 900), st.sampled_from([2**40, -(2**40)])),
    down_msgs=st.one_of(st.integers(-5, 900), st.sampled_from([2**40, -(2**40)])),
    up_pods=st.integers(-3, 6), down_pods=st.integers(-3, 6), max_pods=st.integers(-2, 14), min_pods=st.integers(-2, 14),
    init=st.integers(0, 14), lat_ms=st.tuples(st.integers(0, 40), st.integers(0, 40), st.integers(0, 40)),
    horizon_ns=st.integers(1, 900 * 10**9),
)
def test_ms_clock_equals_ns_clock_property(segs, d0, poll_ms, cools, up_msgs, down_msgs, up_pods, down_pods, max_pods,
                                           min_pods, init, lat_ms, horizon_ns):
    tr = sweep.Trace.from_segments([(0, d0)] + sorted(segs))
    grid = sweep.grid(poll_ns=[poll_ms * 10**6, 2**63 - 1], up_cool_ns=[cools[0]], down_cool_ns=[cools[1]],
                      up_msgs=[up_msgs], down_msgs=[down_msgs], up_pods=[up_pods], down_pods=[down_pods],
                      max_pods=[max_pods], min_pods=[min_pods])
    lat = tuple(x * 10**6 for x in lat_ms)
    if lat[0] == 0 and poll_ms == 0:
        return
    r = _both_clocks(tr, grid, init, horizon_ns, lat)
    assert r.ms_clock


def test_ms_clock_is_chosen_only_when_exact():
    tr = step_trace()
    ms_lat = (2 * 10**6, 10**6, 10**6)
    g = sweep.grid(poll_ns=[S, 5 * S], up_cool_ns=[0, 10 * S + 1])
    assert _both_clocks(tr, g, 1, 900 * S, ms_lat).ms_clock
    # a latency or a period that fires with a sub-ms part: the nanosecond clock, same results
    assert not _both_clocks(tr, g, 1, 900 * S, (2_500_000, 10**6, 10**6)).ms_clock
    assert not _both_clocks(tr, sweep.grid(poll_ns=[S + 1]), 1, 900 * S, ms_lat).ms_clock
    # ... unless that period never fires (longer than the horizon)
    assert _both_clocks(tr, sweep.grid(poll_ns=[S, 901 * S + 1]), 1, 900 * S, ms_lat).ms_clock
    # depths outside [0, 2^31 - 2], or a horizon past 2^30 ms: the nanosecond clock
    neg = sweep.Trace.from_segments([(0, 5), (60 * S, -1)])
    assert not _both_clocks(neg, g, 1, 900 * S, ms_lat).ms_clock
    big = sweep.Trace.from_segments([(0, 5), (60 * S, 2**31 - 1)])
    assert not _both_clocks(big, g, 1, 900 * S, ms_lat).ms_clock
    assert _both_clocks(sweep.Trace.from_segments([(0, 5), (60 * S, 2**31 - 2)]), g, 1, 900 * S, ms_lat).ms_clock
    # the deepest queue over a long horizon: backlog runs far past 2^53 msg-ms, still exact
    deep = sweep.Trace.from_segments([(0, 2**31 - 2), (3600 * S, 3), (7200 * S, 2**31 - 2)])
    g2 = sweep.grid(poll_ns=[60 * S], up_cool_ns=[0], down_cool_ns=[0], up_msgs=[100], down_msgs=[10], max_pods=[3])
    assert _both_clocks(deep, g2, 1, 10**8 * 10**6, ms_lat).ms_clock
    long_h = 2**30 * 10**6
    assert not sweep.run(tr, sweep.grid(poll_ns=[3600 * S]), 1, long_h, ms_lat, device="cpu").ms_clock
    with pytest.raises(ValueError, match="clock"):
        sweep.run(tr, g, 1, 900 * S, ms_lat, device="cpu", clock="fast")


def test_ms_clock_boundaries_exactly_at_cool_down_expiry():
    """Cool-downs that expire exactly on a poll, one ns before and one ns after (strict After,
    main.go:52,66), and trace boundaries one ns either side of a poll: both clocks agree."""
    polls = [k * S for k in range(1, 40)]
    segs = [(0, 0)] + [(t + off, 500 if i % 2 == 0 else 0) for i, t in enumerate(polls[::3]) for off in (-1, 1)]
    segs = sorted(set(segs))
    tr = sweep.Trace(np.array([s[0] for s in segs]), np.array([s[1] for s in segs]))
    g = sweep.grid(poll_ns=[S], up_cool_ns=[3 * S - 1, 3 * S, 3 * S + 1, 3 * S + 2 * 10**6],
                   down_cool_ns=[2 * S - 1, 2 * S, 2 * S + 1], up_msgs=[100], down_msgs=[10])
    for lat in ((0, 0, 0), (10**6, 10**6, 10**6), (0, 2 * 10**6, 0)):
        assert _both_clocks(tr, g, 1, 60 * S, lat).ms_clock


def test_steady_stretch_skip_is_chosen_for_coarse_traces():
    """skip="auto" (policy_sim.h skip_pays): on when a trace segment spans four or more of the
    grid's shortest poll intervals on the millisecond clock (five on the nanosecond one), off for
    a trace sampled at every poll (the GPU kernel is slower with the check where no stretch
    forms). Either way the results are the same, and the skip leaves the simulated poll count as
    it is."""
    rng = np.random.default_rng(3)
    coarse = sweep.Trace(np.arange(0, 3600 * S, 60 * S), rng.integers(0, 400, 60))
    fine = sweep.Trace(np.arange(0, 3600 * S, 5 * S), rng.integers(0, 400, 720))
    g = sweep.grid(poll_ns=[5 * S, 10 * S], up_cool_ns=[0, 60 * S, 300 * S], down_cool_ns=[0, 120 * S],
                   up_msgs=[100, 300], down_msgs=[10, 50])
    lat = (2 * 10**6, 10**6, 10**6)
    assert sweep.run(coarse, g, 1, 3600 * S, lat, device="cpu").skip  # 12 polls a segment
    assert not sweep.run(fine, g, 1, 3600 * S, lat, device="cpu").skip  # 1
    half = sweep.Trace(np.arange(0, 3600 * S, 25 * S), rng.integers(0, 400, 144))  # 5 - latency
    assert sweep.run(half, g, 1, 3600 * S, lat, device="cpu").skip
    assert not sweep.run(half, g, 1, 3600 * S, lat, device="cpu", clock="ns").skip
    for tr in (coarse, fine):
        r = _both_clocks(tr, g, 1, 3600 * S, lat)
        assert r.out["polls"].min() > 300  # every lane still counts every poll
    with pytest.raises(ValueError, match="skip"):
        sweep.run(coarse, g, 1, 3600 * S, lat, device="cpu", skip="maybe")
