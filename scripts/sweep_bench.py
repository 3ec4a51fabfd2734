"""What-if sweep throughput: 1M configurations over a synthetic 24 h queue trace, gfx950 kernel
vs the CPU path (same simulator, bit-identical results). One JSON line per device."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from kube_sqs_autoscaler_amd.tune import sweep  # noqa: E402

S = 1_000_000_000
# KSA_BENCH_SEGMENT_S: trace resolution (5 s: 17280 segments, read from global memory; 30 s:
# 2880, staged in LDS on both clocks)
seg_s = int(os.environ.get("KSA_BENCH_SEGMENT_S", "5"))
rng = np.random.default_rng(7)
n = 24 * 3600 // seg_s  # one segment per seg_s over a day
t = np.arange(n, dtype=np.int64) * seg_s * S
base = 200 + 180 * np.sin(np.arange(n) / n * 2 * np.pi * 3)  # three daily waves
bursts = (rng.random(n) < 0.01) * rng.integers(500, 5000, n)
depth = np.maximum(0, base + rng.normal(0, 40, n) + bursts).astype(np.int64)
tr = sweep.Trace(t, depth)
grid = sweep.grid(poll_ns=[5 * S], up_cool_ns=list(range(0, 600 * S, 6 * S)), down_cool_ns=list(range(0, 1500 * S, 30 * S)),
                  up_msgs=[50, 100, 150, 200, 300, 400, 600, 800, 1200, 1600], down_msgs=[10, 50],
                  max_pods=[4, 8, 16, 32, 64], min_pods=[1, 2])
m = grid.shape[1]
horizon = 24 * 3600 * S
lat = (2_000_000, 1_000_000, 1_000_000)
results = {}
# (device, clock): the GPU on both clocks (the auto run takes the millisecond one: whole-ms periods
# and latencies), the CPU on the nanosecond clock (the exactness baseline)
for device, clock in (("gpu", "auto"), ("gpu", "ns"), ("cpu", "ns")):
    if device == "gpu" and not sweep.gpu_available():
        continue
    sub = grid if device == "gpu" else grid[:, : m // 20]  # CPU on a 5 % slice, scaled
    sweep.run(tr, sub[:, :1024], 1, horizon, lat, device, clock=clock)  # warm-up
    t0 = time.perf_counter()
    r = sweep.run(tr, sub, 1, horizon, lat, device, threads=16, clock=clock)
    wall = time.perf_counter() - t0
    polls = int(r.out["polls"].sum())
    results[device + "_" + clock] = r
    print(json.dumps({"device": device, "clock": "ms" if r.ms_clock else "ns", "configs": sub.shape[1],
                      "simulated_polls": polls, "wall_s": round(wall, 4),
                      "kernel_ms": round(r.kernel_ms, 3), "polls_per_s": round(polls / wall, 1),
                      "best_pod_ms_within_backlog_p50": int(np.min(r.out["pod_ms"][r.out["backlog"] <= np.median(r.out["backlog"])]))}),
          flush=True)
if "gpu_auto" in results:
    c = results["cpu_ns"]
    k = c.params.shape[1]
    for name in ("gpu_auto", "gpu_ns"):
        g = results[name]
        same = all(np.array_equal(g.out[key][:k], c.out[key]) for key in g.out)
        print(json.dumps({f"{name}_equals_cpu_ns_on_slice": same}), flush=True)
    a, b = results["gpu_auto"], results["gpu_ns"]
    print(json.dumps({"gpu_ms_clock_equals_gpu_ns_clock": all(np.array_equal(a.out[key], b.out[key]) for key in a.out)}),
          flush=True)
