"""Sharded what-if sweeps (tune/distributed.py): torchrun ranks over gloo on CPU must reproduce
the single-process sweep exactly (RCCL on an MI355X node runs the same code path with cuda
tensors)."""
import json
import os
import socket
import subprocess
import sys

import pytest

import numpy as np

from kube_sqs_autoscaler_amd.tune import sweep
from kube_sqs_autoscaler_amd.tune.distributed import config_costs, shard_plan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
S = 1_000_000_000


@pytest.mark.parametrize("m,world", [(10, 3), (3, 8), (0, 2), (1000, 8), (7, 1)])
def test_shard_plan_partitions_the_grid(m, world):
    costs = np.random.default_rng(m).integers(1, 100, size=m)
    plan = shard_plan(costs, world)
    assert len(plan) == world
    assert sorted(np.concatenate(plan).tolist()) == list(range(m))
    sizes = [len(p) for p in plan]
    assert max(sizes) - min(sizes) <= 1
    for p in plan:  # each share in decreasing-cost order, ties in grid order
        assert all((costs[a], -a) >= (costs[b], -b) for a, b in zip(p, p[1:]))


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_shard_plan_balances_cost_over_poll_periods(world):
    """A lane's work is horizon / poll period: on a 1 s..10 s grid (poll outermost) equal-count
    contiguous slices put ~10x the polls on rank 0 as on the last rank; the plan keeps the
    per-rank cost sums within 10 % of each other."""
    params = sweep.grid(poll_ns=[k * S for k in range(1, 11)], up_cool_ns=[0, 30 * S, 60 * S, 120 * S],
                        up_msgs=[50, 100, 200], max_pods=[4, 8])
    horizon, lat = 3600 * S, (1_000_000, 1_000_000, 1_000_000)
    costs = config_costs(params, horizon, lat)
    assert costs.sum() == sweep.estimated_polls(params, horizon, lat)
    loads = [int(costs[p].sum()) for p in shard_plan(costs, world)]
    assert max(loads) / min(loads) <= 1.1, loads
    # what equal-count contiguous slices (the round-3 split) would have given
    bounds = np.linspace(0, len(costs), world + 1).astype(int)
    naive = [int(costs[a:b].sum()) for a, b in zip(bounds, bounds[1:])]
    assert max(naive) / min(naive) > 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args, world=None):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    if world is None:
        cmd = [sys.executable, "-m", "kube_sqs_autoscaler_amd.tune", *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "-m", "kube_sqs_autoscaler_amd.tune",
               "--distributed", *args]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    return lines[0], lines[1:]


def test_open_loop_three_ranks_equal_single_process(tmp_path):
    csv = tmp_path / "depth.csv"
    csv.write_text("seconds,depth\n" + "".join(f"{i * 5},{(i * 37) % 400}\n" for i in range(300)))
    # poll periods vary, so the cost-balanced plan interleaves the grid over the ranks and the
    # gathered rows must be scattered back into grid order
    args = ["--trace", str(csv), "--device", "cpu", "--json", "--top", "0", "--grid", "poll-period=1s,5s,10s",
            "--grid", "scale-up-cool-down=0s:2m:20s", "--grid", "scale-up-messages=50,100,200,400",
            "--grid", "max-pods=4,8,16"]  # 3 x 7 x 4 x 3 = 252 configs
    info1, rows1 = _run(args)
    info3, rows3 = _run(args, world=3)
    assert info3["ranks"] == 3 and info1["ranks"] == 1
    assert info1["configs"] == info3["configs"] == 252
    assert rows1 == rows3 and len(rows1) == 252


def test_closed_loop_two_ranks_equal_single_process(tmp_path):
    csv = tmp_path / "rate.csv"
    csv.write_text("seconds,msgs_per_second\n0,2\n600,30\n1200,2\n")
    args = ["--arrivals", str(csv), "--horizon", "40m", "--service-rate", "5", "--seeds", "6", "--device", "cpu",
            "--json", "--top", "0", "--grid", "scale-up-cool-down=0s:4m:1m", "--grid", "max-pods=2,8,9", "--grid", "poll-period=2s,7s"]
    info1, rows1 = _run(args)
    info2, rows2 = _run(args, world=2)
    assert info2["ranks"] == 2 and info1["configs"] == info2["configs"] == 30
    assert rows1 == rows2 and len(rows1) == 30


def test_group_refuses_to_start_after_the_kernels_library(monkeypatch):
    import sys

    from kube_sqs_autoscaler_amd.ops import gpu
    from kube_sqs_autoscaler_amd.tune import distributed

    monkeypatch.setattr(gpu, "_LIB", object())
    monkeypatch.delitem(sys.modules, "torch", raising=False)
    with pytest.raises(RuntimeError, match="before the first GPU sweep"):
        distributed.Group("cpu")


def test_shard_plan_imbalance_is_at_most_one_configuration():
    """Property: the snake deal keeps any two ranks' cost sums within the costliest single
    configuration, for any costs and rank count."""
    from hypothesis import given, settings
    from hypothesis import strategies as st

    @settings(max_examples=400, deadline=None)
    @given(st.lists(st.integers(1, 10**6), max_size=80), st.integers(1, 9))
    def check(costs, world):
        c = np.array(costs, dtype=np.int64)
        plan = shard_plan(c, world)
        assert sorted(np.concatenate(plan).tolist()) == list(range(len(c)))
        if len(c):
            loads = [int(c[p].sum()) for p in plan]
            assert max(loads) - min(loads) <= int(c.max())

    check()


def test_config_costs_do_not_wrap_on_huge_periods():
    """a poll period near int64's max plus the latency wrapped negative, was clamped
    to a step of 1 and costed at horizon polls; clipped to the horizon it costs what it is, at
    most one poll."""
    horizon = 24 * 3600 * 10**9
    params = np.array([[5 * 10**9, np.iinfo(np.int64).max - 10, horizon * 2, 0]], dtype=np.int64)
    costs = config_costs(params, horizon, (10**6, 10**6, 10**6))
    assert costs.tolist() == [horizon // (5 * 10**9 + 10**6), 0, 0, min(horizon // 10**6, 1 << 26)]
