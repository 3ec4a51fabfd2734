"""How evenly `tune --distributed` splits a sweep over the ranks: the shards of an 8-rank job,
each run on this GPU one after another, under the cost-balanced plan (tune/distributed.py
``shard_plan``) and under equal-count contiguous slices of the poll-sorted grid (round 3's split).
A job finishes with its slowest rank, so the number that matters is the slowest shard's kernel
time against the mean. One JSON line per (split, rank), then a summary line per split.

    python scripts/shard_balance.py [--world 8]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from kube_sqs_autoscaler_amd.tune import sweep  # noqa: E402
from kube_sqs_autoscaler_amd.tune.distributed import config_costs, shard_plan  # noqa: E402

S = 1_000_000_000


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--device", default="gpu")
    a = ap.parse_args()
    rng = np.random.default_rng(7)
    n = 24 * 3600 // 30
    t = np.arange(n, dtype=np.int64) * 30 * S
    depth = np.maximum(0, 200 + 180 * np.sin(np.arange(n) / n * 6 * np.pi) + rng.normal(0, 40, n)).astype(np.int64)
    tr = sweep.Trace(t, depth)
    # poll periods 1 s .. 10 s, outermost: a lane's work is horizon / period. On the GPU each
    # shard must be large enough to fill the chip several times over (1M lanes per shard at
    # --world 8): a shard the chip runs in one pass takes as long as its longest lane whatever
    # its total, and then no split can help.
    big = a.device == "gpu"
    grid = sweep.grid(poll_ns=[k * S for k in range(1, 11)],
                      up_cool_ns=list(range(0, 600 * S, (6 if big else 20) * S)),
                      down_cool_ns=list(range(0, 1200 * S, (30 if big else 60) * S)),
                      up_msgs=[50, 100, 150, 200, 300, 400, 600, 800, 1200, 1600] if big else [50, 100, 200, 400, 800],
                      max_pods=[4, 8, 16, 32, 64] if big else [8, 16, 32], min_pods=[1, 2, 3, 4] if big else [1])
    horizon, lat = (6 if big else 24) * 3600 * S, (2_000_000, 1_000_000, 1_000_000)
    m = grid.shape[1]
    costs = config_costs(grid, horizon, lat)
    bounds = np.linspace(0, m, a.world + 1).astype(int)
    splits = {"cost_balanced": shard_plan(costs, a.world),
              "contiguous": [np.arange(lo, hi) for lo, hi in zip(bounds, bounds[1:])]}
    sweep.run(tr, grid[:, :4096], 1, horizon, lat, a.device)  # warm-up (device buffers, code object)
    for name, plan in splits.items():
        ms = []
        for r, idx in enumerate(plan):
            t0 = time.perf_counter()
            res = sweep.run(tr, np.ascontiguousarray(grid[:, idx]), 1, horizon, lat, a.device)
            wall_ms = (time.perf_counter() - t0) * 1e3
            ms.append(res.kernel_ms if res.kernel_ms > 0 else wall_ms)  # the CPU path reports no kernel time
            print(json.dumps({"split": name, "rank": r, "configs": len(idx), "simulated_polls": int(costs[idx].sum()),
                              "kernel_ms": round(res.kernel_ms, 3), "wall_ms": round(wall_ms, 3)}), flush=True)
        loads = [int(costs[idx].sum()) for idx in plan]
        print(json.dumps({"split": name, "world": a.world, "configs": m, "device": a.device,
                          "timed": "kernel" if a.device == "gpu" else "wall",
                          "slowest_over_mean": round(max(ms) / (sum(ms) / len(ms)), 3),
                          "max_over_min": round(max(ms) / min(ms), 3),
                          "max_over_min_polls": round(max(loads) / min(loads), 3),
                          "job_ms_if_parallel": round(max(ms), 3)}), flush=True)


if __name__ == "__main__":
    main()
