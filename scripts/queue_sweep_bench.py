"""Closed-loop what-if sweep throughput: configurations x seeds over a synthetic 24 h arrival
pattern, gfx950 kernel vs the CPU path (same header, bit-identical). One JSON line per device.

``--arith saturating`` forces queue_sim.h's saturating arithmetic on the GPU, ``--arith fast-ns``
FastArith with the nanosecond decision clock (default: auto, which runs FastArith when its bounds
hold, on the millisecond decision clock when periods and latencies are whole ms -- both hold here). The CPU slice always runs the saturating
arithmetic, so the equality line checks the GPU's arithmetic against it."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from kube_sqs_autoscaler_amd.tune import closedloop as cl  # noqa: E402
from kube_sqs_autoscaler_amd.tune import sweep  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--arith", choices=("auto", "saturating", "fast-ns"), default="auto",
                help="GPU arithmetic: auto (FastArith on the ms decision clock here), fast-ns, saturating")
args = ap.parse_args()
S = 1_000_000_000
minutes = np.arange(1440)
rate = 20 + 15 * np.sin(minutes / 1440 * 2 * np.pi * 2) + (np.random.default_rng(3).random(1440) < 0.02) * 120
trace = cl.ArrivalTrace.from_segments([(60.0 * i, float(r)) for i, r in enumerate(rate)])
grid = sweep.grid(poll_ns=[5 * S], up_cool_ns=list(range(0, 600 * S, 30 * S)), down_cool_ns=list(range(0, 1800 * S, 120 * S)),
                  up_msgs=[25, 50, 100, 200, 400], down_msgs=[5, 25], max_pods=[8, 16, 32, 64], min_pods=[1, 2])
model = cl.QueueModel(service_rate=4.0, startup_ns=90 * S, slo_backlog=500)
seeds, horizon, lat = 32, 86400 * S, (2_000_000, 1_000_000, 1_000_000)
m = grid.shape[1]
results = {}
for device in ("gpu", "cpu"):
    if device == "gpu" and not sweep.gpu_available():
        continue
    sub = grid if device == "gpu" else grid[:, : max(1, m // 100)]  # CPU on a 1 % slice
    arith = args.arith if device == "gpu" else "saturating"
    cl.run(trace, sub[:, :64], model, 1, horizon, lat, seeds=seeds, device=device, arith=arith)  # warm-up
    t0 = time.perf_counter()
    r = cl.run(trace, sub, model, 1, horizon, lat, seeds=seeds, device=device, threads=16, arith=arith)
    wall = time.perf_counter() - t0
    polls = int(r.out["polls"].sum())
    results[device] = r
    summ = r.summary()
    feasible = summ["violation_s_p95"] <= 600
    best = int(np.argmin(np.where(feasible, summ["pod_hours_mean"], np.inf))) if feasible.any() else None
    print(json.dumps({"device": device, "arith": ("fast" if r.fast_arith else "saturating") + ("+ms" if r.ms_clock else ""), "configs": sub.shape[1], "seeds": seeds, "lane_polls": polls,
                      "wall_s": round(wall, 4), "kernel_ms": round(r.kernel_ms, 3),
                      "lane_polls_per_s": round(polls / wall, 1),
                      "feasible": int(feasible.sum()),
                      "best_under_10min_p95_violation": None if best is None else r.row(best)}), flush=True)
if "gpu" in results and "cpu" in results:
    g, c = results["gpu"], results["cpu"]
    k = c.params.shape[1]
    print(json.dumps({"gpu_equals_cpu_on_slice": all(np.array_equal(g.out[key][:k], c.out[key]) for key in g.out)}),
          flush=True)
