#!/usr/bin/env python3
"""Where does latency go as tracked queues are added? (VERDICT r01 weak #1 / next #4.)

For 1/2/4/8 queues in one autoscaler process and each endpoint placement -- one shared fake
pair in-process, one pair per queue in-process, one pair per queue in a separate endpoint
process -- three interleaved rounds of `measure_detailed`: p50, per-phase medians, and the
scheduler's view per thread group (CPU, run-queue wait, context switches per poll), plus
cgroup throttling and IPI counts. One JSON line per run to stdout.

Usage: python scripts/multiqueue_probe.py [--samples 2000] [--rounds 3] [--busy-poll-us 25]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.bench.latency import measure_detailed  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=2000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--busy-poll-us", type=int, nargs="+", default=[25])
    ap.add_argument("--servers", nargs="+", default=["shared", "per-queue", "process"])
    ap.add_argument("--queues", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--affinity", nargs="+", default=["none"])
    ap.add_argument("--loggers", nargs="+", default=["shared"])
    ap.add_argument("--log-level", nargs="+", default=["info"])
    a = ap.parse_args()
    env = {"cpus_visible": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
    try:
        env["cpu.max"] = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        pass
    print(json.dumps({"env": env}), flush=True)
    for rnd in range(a.rounds):
        for bp in a.busy_poll_us:
            for aff in a.affinity:
                for sv in a.servers:
                    if aff == "llc" and sv == "shared":
                        continue
                    for lg in a.loggers:
                        for lv in a.log_level:
                            for q in a.queues:
                                d = measure_detailed(q, a.samples, 200, "scale", pipeline=True,
                                                     busy_poll_ns=bp * 1000, servers=sv, affinity=aff, loggers=lg,
                                                     log_level=lv)
                                d["round"] = rnd
                                print(json.dumps(d), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
