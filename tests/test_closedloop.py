"""Closed-loop what-if sweep (csrc/sim/queue_sim.h): the native CPU path must agree exactly with
the independent Python statement of the model, and the model must behave like a queue."""
import numpy as np
import pytest

from kube_sqs_autoscaler_amd.tune import closedloop as cl
from kube_sqs_autoscaler_amd.tune import sweep

S = 1_000_000_000
LAT = (2_000_000, 1_000_000, 1_000_000)


def burst_trace():
    # quiet, a 10-minute burst of 40 msgs/s, quiet again; 1.5 msgs/s fractional rate in between
    return cl.ArrivalTrace.from_segments([(0, 0.5), (300, 40.0), (900, 1.5), (1500, 0.0)])


def small_grid():
    return sweep.grid(poll_ns=[5 * S, 7 * S], up_cool_ns=[0, 30 * S, 120 * S], down_cool_ns=[0, 60 * S],
                      up_msgs=[20, 100], down_msgs=[5], max_pods=[4, 8], min_pods=[1])


@pytest.mark.parametrize("startup_s,service", [(0, 5.0), (90, 5.0), (45, 12.5)])
def test_cpu_path_equals_python_model(nat, startup_s, service):
    tr, grid = burst_trace(), small_grid()
    model = cl.QueueModel(service_rate=service, startup_ns=startup_s * S, slo_backlog=200, init_backlog=30)
    horizon = 2400 * S
    res = cl.run(tr, grid, model, 1, horizon, LAT, seeds=3, seed0=11, device="cpu")
    for i in range(0, len(res), 5):
        for s in range(3):
            want = cl.reference_lane(tr, res.config(i), model, 1, horizon, LAT, 11 + s)
            got = {k: int(v[i, s]) for k, v in res.out.items()}
            assert got == want, (res.config(i), s)


def test_queue_physics():
    tr = burst_trace()
    horizon = 2400 * S
    base = dict(poll_ns=[5 * S], up_cool_ns=[10 * S], down_cool_ns=[30 * S], up_msgs=[50], down_msgs=[5], min_pods=[1])
    res = cl.run(tr, sweep.grid(max_pods=[1, 2, 4, 8, 16], **base), cl.QueueModel(5.0, 30 * S, 100), 1, horizon, LAT,
                 seeds=16, device="cpu")
    summ = res.summary()
    # more headroom drains the burst faster: mean backlog falls (weakly) and cost rises as max-pods grows
    assert np.all(np.diff(summ["backlog_mean"]) <= 1e-9)
    assert np.all(np.diff(summ["pod_hours_mean"]) >= -1e-9)
    assert summ["backlog_mean"][0] > 5 * summ["backlog_mean"][-1]
    # conservation: what arrived was served or is still queued (milli-message flooring: +-1 each)
    arrived, served, final = (res.out[k] for k in ("arrived", "served", "final_backlog"))
    assert np.all(np.abs(arrived - served - final) <= 2)
    # the burst really arrives: ~40 msgs/s x 600 s
    assert 20000 < arrived.mean() < 28000


def test_startup_delay_costs_backlog():
    tr, horizon = burst_trace(), 2400 * S
    grid = sweep.grid(poll_ns=[5 * S], up_cool_ns=[10 * S], down_cool_ns=[30 * S], up_msgs=[50], max_pods=[8])
    fast = cl.run(tr, grid, cl.QueueModel(5.0, 0, 100), 1, horizon, LAT, seeds=16, device="cpu").summary()
    slow = cl.run(tr, grid, cl.QueueModel(5.0, 300 * S, 100), 1, horizon, LAT, seeds=16, device="cpu").summary()
    assert slow["backlog_mean"][0] > fast["backlog_mean"][0]
    assert slow["violation_s_mean"][0] > fast["violation_s_mean"][0]


def test_common_random_numbers_and_seed_streams():
    tr, horizon, grid = burst_trace(), 1800 * S, sweep.grid(max_pods=[4, 8])
    m = cl.QueueModel(5.0, 30 * S, 100)
    a = cl.run(tr, grid, m, 1, horizon, LAT, seeds=4, seed0=7, device="cpu")
    b = cl.run(tr, grid, m, 1, horizon, LAT, seeds=4, seed0=7, device="cpu")
    c = cl.run(tr, grid, m, 1, horizon, LAT, seeds=4, seed0=8, device="cpu")
    assert all(np.array_equal(a.out[k], b.out[k]) for k in a.out)
    assert not np.array_equal(a.out["arrived"], c.out["arrived"])
    # every seed is its own arrival sequence
    assert len(set(a.out["arrived"][0].tolist())) > 1


def test_validation():
    tr, grid = burst_trace(), sweep.grid()
    with pytest.raises(ValueError, match="service rate"):
        cl.run(tr, grid, cl.QueueModel(-1.0), device="cpu")
    with pytest.raises(ValueError, match="startup"):
        cl.run(tr, grid, cl.QueueModel(1.0, startup_ns=2 * 86400 * S), device="cpu")
    with pytest.raises(ValueError, match="horizon"):
        cl.run(tr, grid, cl.QueueModel(1.0), horizon_ns=40 * 86400 * S, device="cpu")
    with pytest.raises(ValueError, match="arrival rates"):
        cl.ArrivalTrace.from_segments([(0, -1.0)])


def test_arrival_csv(tmp_path):
    p = tmp_path / "arrivals.csv"
    p.write_text("seconds,rate\n100,2\n160,10.5\n")
    tr = cl.ArrivalTrace.from_csv(str(p))
    assert tr.t_ms.tolist() == [0, 60000] and tr.rate_milli.tolist() == [2000, 10500]


def test_tune_cli_closed_loop_ranks_under_violation_bound(tmp_path, capsys):
    import json

    from kube_sqs_autoscaler_amd.tune.__main__ import main

    csv_path = tmp_path / "rate.csv"
    csv_path.write_text("seconds,msgs_per_second\n0,2\n600,30\n1200,2\n")
    argv = ["--arrivals", str(csv_path), "--horizon", "40m", "--service-rate", "5", "--startup-delay", "60s",
            "--slo-backlog", "300", "--seeds", "8", "--device", "cpu", "--max-violation", "8m",
            "--grid", "scale-up-cool-down=0s:4m:1m", "--grid", "scale-up-messages=50,200,800",
            "--grid", "max-pods=2,8", "--json", "--top", "5"]
    assert main(argv) == 0
    lines = [json.loads(x) for x in capsys.readouterr().out.splitlines()]
    info, rows = lines[0], lines[1:]
    assert info["configs"] == 5 * 3 * 2 and info["seeds"] == 8 and info["device"] == "cpu"
    assert 0 < len(rows) <= 5 and info["feasible"] >= len(rows)
    assert all(r["violation_s_p95"] <= 480 for r in rows)
    costs = [r["pod_hours_mean"] for r in rows]
    assert costs == sorted(costs)
    # two pods drain 10 msgs/s < 30 msgs/s arriving: the 10-minute burst backs up past the SLO
    assert all(r["max_pods"] == 8 for r in rows)
    assert "pod_hours_mean" in info["reference_defaults"]
    # table output and the Pareto front
    assert main(argv[:-3] + ["--pareto"]) == 0
    out = capsys.readouterr().out
    assert "configs x 8 seeds" in out and "pod_hours_mean" in out


def test_tune_cli_closed_loop_argument_errors(tmp_path):
    import pytest

    from kube_sqs_autoscaler_amd.tune.__main__ import main

    csv_path = tmp_path / "rate.csv"
    csv_path.write_text("0,1\n")
    with pytest.raises(SystemExit):
        main(["--arrivals", str(csv_path)])  # no --service-rate
    with pytest.raises(SystemExit):
        main(["--arrivals", str(csv_path), "--service-rate", "1", "--objective", "nope", "--device", "cpu"])
    with pytest.raises(SystemExit):
        main(["--arrivals", str(csv_path), "--trace", str(csv_path), "--service-rate", "1"])


@pytest.mark.parametrize("rate,service,poll_s,init", [(1e6, 1e6, 20 * 86400, 10**12), (1e6, 0.001, 3, 10**12),
                                                      (999_999.999, 1e6, 86400, 0), (0.001, 1e6, 1, 10**12)])
def test_cpu_path_equals_python_model_at_extremes(nat, rate, service, poll_s, init):
    """Bounds of the validated inputs: maximum rates, 20-day polls in a 30-day horizon (intervals
    above 2^31 ms), a 1e12-message backlog -- the saturating and wide-operand paths."""
    tr = cl.ArrivalTrace.from_segments([(0, rate), (7 * 86400, rate / 2)])
    grid = sweep.grid(poll_ns=[poll_s * S], up_cool_ns=[0], down_cool_ns=[0], up_msgs=[1, 10**15], max_pods=[2**31 - 1, 50])
    model = cl.QueueModel(service_rate=service, startup_ns=86400 * S, slo_backlog=0, init_backlog=init)
    horizon = (30 * 86400 if poll_s > 86400 else 400) * S
    res = cl.run(tr, grid, model, 1, horizon, (0, 0, 0), seeds=2, seed0=5, device="cpu")
    assert not res.fast_arith  # 2^31 - 1 pods: queue_sim.h's fast_path_ok refuses
    for i in range(len(res)):
        for s in range(2):
            want = cl.reference_lane(tr, res.config(i), model, 1, horizon, (0, 0, 0), 5 + s)
            assert {k: int(v[i, s]) for k, v in res.out.items()} == want, (res.config(i), s)


def test_cpu_path_equals_python_model_on_fine_segments(nat):
    """Segments shorter than a poll interval, boundaries on whole poll times, a zero-rate run and
    a rate held to the horizon: the register-resident rate cursor (queue_sim.h RateCursor) must
    integrate exactly what the Python model does."""
    segs = [(0.0, 3.0), (2.0, 0.0), (2.5, 7.25), (5.0, 40.0), (10.0, 0.5), (10.001, 12.0), (35.0, 0.0),
            (70.0, 0.0), (71.0, 90.0), (71.5, 1.0)]
    tr = cl.ArrivalTrace.from_segments(segs)
    grid = sweep.grid(poll_ns=[1 * S, 5 * S], up_cool_ns=[0, 3 * S], down_cool_ns=[0], up_msgs=[10, 50],
                      down_msgs=[2], max_pods=[6], min_pods=[1])
    model = cl.QueueModel(service_rate=3.0, startup_ns=2 * S, slo_backlog=50, init_backlog=5)
    horizon = 120 * S
    res = cl.run(tr, grid, model, 1, horizon, (0, 1_000_000, 1_000_000), seeds=4, seed0=3, device="cpu")
    assert res.fast_arith
    for i in range(len(res)):
        for s in range(4):
            want = cl.reference_lane(tr, res.config(i), model, 1, horizon, (0, 1_000_000, 1_000_000), 3 + s)
            got = {k: int(v[i, s]) for k, v in res.out.items()}
            assert got == want, (res.config(i), s)


@pytest.mark.parametrize("tweak,fast", [
    ({}, True),
    ({"min_pods": [-1]}, False),             # a negative replica bound: counts could go negative
    ({"max_pods": [2**31 - 2], "up_pods": [2]}, False),  # max + up wraps int32
    ({"down_pods": [-3]}, False),
])
def test_fast_arithmetic_selection_is_exact(nat, tweak, fast):
    """queue_sim.h runs FastArith (plain integer ops, 32-bit times) only when fast_path_ok proves
    that nothing can saturate or wrap; then it computes exactly what the saturating arithmetic
    (and the Python model) does."""
    tr = burst_trace()
    axes = dict(poll_ns=[5 * S], up_cool_ns=[0, 60 * S], down_cool_ns=[0, 120 * S], up_msgs=[20, 100], down_msgs=[5],
                max_pods=[4, 8], min_pods=[1])
    axes.update(tweak)
    grid = sweep.grid(**axes)
    model = cl.QueueModel(service_rate=5.0, startup_ns=45 * S, slo_backlog=100, init_backlog=15)
    auto = cl.run(tr, grid, model, 1, 2400 * S, LAT, seeds=4, seed0=2, device="cpu")
    sat = cl.run(tr, grid, model, 1, 2400 * S, LAT, seeds=4, seed0=2, device="cpu", arith="saturating")
    assert auto.fast_arith is fast and not sat.fast_arith
    assert auto.ms_clock is fast and not sat.ms_clock  # whole-ms periods and latencies
    for k in auto.out:
        assert np.array_equal(auto.out[k], sat.out[k]), k
    for i in range(len(auto)):
        want = cl.reference_lane(tr, auto.config(i), model, 1, 2400 * S, LAT, 3)
        assert {k: int(v[i, 1]) for k, v in auto.out.items()} == want
    with pytest.raises(ValueError, match="arith"):
        cl.run(tr, grid, model, device="cpu", arith="fast")


def test_fast_arithmetic_refuses_unbounded_backlogs(nat):
    """A 1e12-message initial backlog times a 30-day horizon could overflow the backlog
    integral: fast_path_ok must fall back to the saturating arithmetic."""
    tr = cl.ArrivalTrace.from_segments([(0, 1.0)])
    grid = sweep.grid(poll_ns=[3600 * S], max_pods=[4])
    big = cl.run(tr, grid, cl.QueueModel(1.0, 0, 10, init_backlog=10**12), 1, 30 * 86400 * S, LAT, seeds=1, device="cpu")
    small = cl.run(tr, grid, cl.QueueModel(1.0, 0, 10, init_backlog=10**6), 1, 30 * 86400 * S, LAT, seeds=1, device="cpu")
    assert not big.fast_arith and small.fast_arith


def test_fast_arithmetic_matches_saturating_on_random_extremes(nat):
    """Randomised inputs near the bounds fast_path_ok reasons about (rates up to 1e6 msgs/s,
    service up to 1e6, backlogs up to 1e12, horizons up to 30 days, pods up to 2^31 - 1): whenever
    the host picks FastArith it must compute exactly what the saturating arithmetic does."""
    rng = np.random.default_rng(20261017)
    picked = {True: 0, False: 0}
    for _ in range(40):
        horizon_s = int(rng.choice([600, 86400, 10 * 86400, 30 * 86400]))
        n_seg = int(rng.integers(1, 5))
        starts = sorted({0, *[int(x) for x in rng.integers(1, horizon_s, n_seg - 1)]})
        rates = [float(rng.choice([0.0, 0.001, 3.5, 1e3, 1e6])) for _ in starts]
        tr = cl.ArrivalTrace.from_segments(list(zip(starts, rates)))
        grid = sweep.grid(poll_ns=[max(horizon_s // 500, 1) * S], up_cool_ns=[0, 60 * S], down_cool_ns=[0],
                          up_msgs=[int(rng.choice([1, 100, 10**9]))], down_msgs=[0],
                          up_pods=[int(rng.choice([1, 1000, 2**30]))],
                          max_pods=[int(rng.choice([8, 10**4, 2**31 - 1]))], min_pods=[0, 1])
        model = cl.QueueModel(service_rate=float(rng.choice([0.0, 0.5, 40.0, 1e6])),
                              startup_ns=int(rng.choice([0, 60, 86400])) * S, slo_backlog=100,
                              init_backlog=int(rng.choice([0, 10**6, 10**12])))
        lat = (int(rng.integers(0, 5_000_000)), 1_500_000, 700_000)
        init = int(rng.choice([0, 3]))
        args = (tr, grid, model, init, horizon_s * S, lat)
        auto = cl.run(*args, seeds=2, seed0=9, device="cpu")
        sat = cl.run(*args, seeds=2, seed0=9, device="cpu", arith="saturating")
        for k in auto.out:
            assert np.array_equal(auto.out[k], sat.out[k]), (k, horizon_s, rates, model, auto.fast_arith)
        picked[auto.fast_arith] += 1
    assert picked[True] and picked[False]


def test_ms_decision_clock_equals_ns_clock_on_random_inputs(nat):
    """simulate_queue_ms (decisions on 32-bit millisecond clocks) against FastArith on the
    nanosecond clock and against the saturating arithmetic: cool-downs and start-up delays at any
    nanosecond (the ms clock ceils the former and floors the latter), several poll periods, rate
    traces with sub-second boundaries, and periods that never fire."""
    rng = np.random.default_rng(1017)
    for _ in range(30):
        horizon_s = int(rng.choice([300, 3600, 86400]))
        starts = sorted({0.0, *[float(x) for x in rng.uniform(0.001, horizon_s, int(rng.integers(0, 6)))]})
        tr = cl.ArrivalTrace.from_segments([(t, float(rng.choice([0.0, 0.3, 4.0, 60.0, 900.0]))) for t in starts])
        cools = [0, int(rng.integers(0, 10**12)), int(rng.integers(-10**10, 10**10)), 7 * S + 1, -1, 2**62]
        grid = sweep.grid(poll_ns=[int(rng.integers(1, 20_000)) * 10**6, int(rng.integers(1, 9)) * S, 2**62],
                          up_cool_ns=cools[:3], down_cool_ns=cools[3:], up_msgs=[int(rng.integers(-5, 300))],
                          down_msgs=[int(rng.integers(-5, 50))], up_pods=[int(rng.integers(0, 4))],
                          down_pods=[int(rng.integers(0, 4))], max_pods=[int(rng.integers(0, 30))],
                          min_pods=[int(rng.integers(0, 4))])
        model = cl.QueueModel(service_rate=float(rng.choice([0.0, 0.7, 5.0, 80.0])),
                              startup_ns=int(rng.integers(0, 200 * S)), slo_backlog=int(rng.integers(0, 500)),
                              init_backlog=int(rng.integers(0, 5000)))
        lat = tuple(int(x) * 10**6 for x in rng.integers(0, 30, 3))
        if lat[0] == 0:
            lat = (10**6,) + lat[1:]
        args = (tr, grid, model, int(rng.integers(0, 5)), horizon_s * S, lat)
        ms = cl.run(*args, seeds=3, seed0=4, device="cpu")
        ns = cl.run(*args, seeds=3, seed0=4, device="cpu", arith="fast-ns")
        sat = cl.run(*args, seeds=3, seed0=4, device="cpu", arith="saturating")
        assert ms.fast_arith and ms.ms_clock and ns.fast_arith and not ns.ms_clock
        for k in ms.out:
            assert np.array_equal(ms.out[k], ns.out[k]), (k, lat, model)
            assert np.array_equal(ms.out[k], sat.out[k]), (k, lat, model)
    # a sub-millisecond latency: the nanosecond clock
    tr = burst_trace()
    r = cl.run(tr, sweep.grid(poll_ns=[5 * S]), cl.QueueModel(5.0, 0, 100), 1, 600 * S, (1_500_000, 10**6, 10**6),
               seeds=1, device="cpu")
    assert r.fast_arith and not r.ms_clock
