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
by_skip = {}
# (device, clock, skip): the GPU on both clocks (the auto run takes the millisecond one: whole-ms
# periods and latencies), the CPU on the nanosecond clock (the exactness baseline). The
# steady-stretch skip as sweep.run picks it ("auto"), or -- KSA_BENCH_SKIP_AB=1 -- every run with
# it forced on and off (same results).
skips = ("on", "off") if os.environ.get("KSA_BENCH_SKIP_AB") == "1" else ("auto",)
runs = [(dev, clk, sk) for dev, clk in (("gpu", "auto"), ("gpu", "ns"), ("cpu", "ns")) for sk in skips]
for device, clock, skip in runs:
    if device == "gpu" and not sweep.gpu_available():
        continue
    sub = grid if device == "gpu" else grid[:, : m // 20]  # CPU on a 5 % slice, scaled
    # warm-up: the GPU's device buffers and code object; the CPU path's first large run (page
    # faults on fresh output arrays, thread start-up) ran up to 2x slower, so it warms at full size
    sweep.run(tr, sub[:, :1024] if device == "gpu" else sub, 1, horizon, lat, device, clock=clock, skip=skip)
    t0 = time.perf_counter()
    r = sweep.run(tr, sub, 1, horizon, lat, device, threads=min(16, os.cpu_count() or 8), clock=clock, skip=skip)
    wall = time.perf_counter() - t0
    polls = int(r.out["polls"].sum())
    results.setdefault(device + "_" + clock, r)
    by_skip[(device, clock, skip)] = r
    print(json.dumps({"device": device, "clock": "ms" if r.ms_clock else "ns", "skip": r.skip, "segment_s": seg_s,
                      "configs": sub.shape[1],
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
if len(skips) == 2:  # each run without the skip against the same run with it
    same = all(np.array_equal(r.out[key], by_skip[(d, c, "off")].out[key])
               for (d, c, sk), r in by_skip.items() if sk == "on" for key in r.out)
    print(json.dumps({"skip_off_equals_skip_on": same}), flush=True)
