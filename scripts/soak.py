"""Soak: the headline configuration (one queue, /scale, pipelined read, busy-poll) polling back to
back for --minutes against the localhost fakes, one JSON line per --window seconds: polls, p50 /
p99 / max latency of the window, errors, RSS of this process. A leak shows as RSS growth, a
slowdown as p50 drift, a stall as a window with few polls. Ends with a summary line.

    python scripts/soak.py --minutes 5 --window 10 > gpurun_out/soak.jsonl
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.bench.latency import BenchEnv  # noqa: E402


def rss_kb() -> int:
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1])
    return 0


def pct(v, p):
    return v[min(len(v) - 1, max(0, int(p / 100.0 * len(v) + 0.5) - 1))] if v else 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=5.0)
    ap.add_argument("--window", type=float, default=10.0)
    ap.add_argument("--busy-poll-us", type=int, default=25)
    a = ap.parse_args()
    env = BenchEnv(1, "scale", pipeline=True, busy_poll_ns=a.busy_poll_us * 1000)
    runner = env.runners[0]
    out = []
    try:
        env.run(2000)  # warm-up
        env.clear()
        end = time.monotonic() + a.minutes * 60
        k = 0
        while time.monotonic() < end:
            st0 = runner.stats()
            t0 = time.monotonic()
            polls = 0
            samples = []
            while time.monotonic() - t0 < a.window:
                env.run(2000)  # a batch of polls, then drain the latency ring
                samples += runner.latencies()
                env.clear()
                polls += 2000
            st1 = runner.stats()
            samples.sort()
            row = {"window": k, "t_s": round(time.monotonic() - (end - a.minutes * 60), 1), "polls": polls,
                   "polls_per_s": round(polls / (time.monotonic() - t0), 1),
                   "p50_us": round(pct(samples, 50) / 1e3, 2), "p99_us": round(pct(samples, 99) / 1e3, 2),
                   "max_us": round(samples[-1] / 1e3, 1) if samples else 0,
                   "errors": (st1["depth_errors"] - st0["depth_errors"]) + (st1["failed_ups"] - st0["failed_ups"]) +
                             (st1["failed_downs"] - st0["failed_downs"]),
                   "rss_kb": rss_kb()}
            out.append(row)
            print(json.dumps(row), flush=True)
            k += 1
    finally:
        env.close()
    if out:
        first, last = out[0], out[-1]
        print(json.dumps({"summary": True, "windows": len(out), "polls": sum(r["polls"] for r in out),
                          "errors": sum(r["errors"] for r in out),
                          "p50_us_first_last": [first["p50_us"], last["p50_us"]],
                          "p50_us_range": [min(r["p50_us"] for r in out), max(r["p50_us"] for r in out)],
                          "p99_us_max": max(r["p99_us"] for r in out),
                          "rss_kb_first_last": [first["rss_kb"], last["rss_kb"]],
                          "signature_failures": env.sqs.signature_failures()}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
