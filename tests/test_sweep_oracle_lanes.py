"""The what-if kernels' shared simulation headers (csrc/sim/policy_sim.h, queue_sim.h) against
the independent Python models, lane by lane, on random and adversarial configurations. The CPU
build of those headers is checked here; tests/test_gpu.py checks the gfx950 build the same way
on the GPU box (and bit-exactness GPU == CPU on every lane)."""
import time

import numpy as np

from _lanes import ADVERSARIAL, MS, S, lanes_to_check, random_params, random_walk_trace
from kube_sqs_autoscaler_amd.tune import closedloop as cl
from kube_sqs_autoscaler_amd.tune import sweep

LAT = (2 * MS, 1 * MS, 1 * MS)


def test_open_loop_cpu_lanes_equal_oracle():
    t0 = time.perf_counter()
    params = random_params(1024, seed=7)
    for n, seed in ((400, 1), (2600, 2)):  # below and above the 2048-segment LDS limit of the GPU path
        tr = random_walk_trace(n, seed)
        horizon = min(int(tr.t_ns[-1]) + 10 * S, 1800 * S)
        c = sweep.run(tr, params, 2, horizon, LAT, device="cpu")
        lanes = lanes_to_check(params.shape[1], 256, seed)
        for i in lanes:
            o = sweep.oracle_row(tr, c.config(i), 2, horizon, LAT)
            assert {k: c.row(i)[k] for k in o} == o, (i, c.config(i))
        # the checked lanes do exercise the state machine in every direction
        for k in ("ups", "downs", "noop_ups", "noop_downs"):
            assert int(c.out[k][lanes].sum()) > 0, k
    assert time.perf_counter() - t0 < 120


def test_closed_loop_cpu_lanes_equal_reference_model():
    params = random_params(512, seed=11, min_poll_ms=2000)
    tr = cl.ArrivalTrace.from_segments([(0, 0.5), (120, 30.0), (400, 2.0), (700, 45.0), (800, 0.0)])
    model = cl.QueueModel(service_rate=4.0, startup_ns=45 * S, slo_backlog=150, init_backlog=20)
    seeds = 4
    c = cl.run(tr, params, model, 1, 1200 * S, LAT, seeds=seeds, device="cpu")
    rng = np.random.default_rng(3)
    lanes = lanes_to_check(params.shape[1], 256, 5)
    for i in lanes:
        s = int(rng.integers(0, seeds))
        want = cl.reference_lane(tr, c.config(i), model, 1, 1200 * S, LAT, 1 + s)
        assert {k: int(v[i, s]) for k, v in c.out.items()} == want, (i, c.config(i))
    assert len(lanes) == 256 and lanes[: len(ADVERSARIAL)] == list(range(len(ADVERSARIAL)))
