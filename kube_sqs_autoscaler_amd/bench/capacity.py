"""Capacity benchmark: many tracked queues on a few worker threads (native Scheduler).

Production question: how many queues can one autoscaler process track at a given poll period
without polls starting late? N queues, each with its own connections and Deployment, run
through ``Scheduler(K)``. Every poll is a full signed SQS call + Deployment GET (+ write when the
fake's 200/0 cycle says so). Reports achieved polls/s against the ideal N/period, the fraction
of polls that started more than 1 ms after they were due, the worst lateness, and the worker
threads' CPU per poll and in cores.
"""
from __future__ import annotations

import time
from typing import Dict

from ..ops import native
from .latency import BenchEnv


def run_capacity(queues: int, period_s: float, threads: int, duration_s: float = 5.0,
                 prewarm_ns: int = -1) -> Dict[str, float]:
    """Steady-state numbers are taken after a warm-up of two poll periods (connections set up,
    staggered starts done). ``prewarm_ns``: each queue's --poll-prewarm (-1: the CLI default),
    which the scheduler runs as a separate event before each poll."""
    from ..config import DEFAULT_POLL_PREWARM_NS

    if prewarm_ns < 0:
        prewarm_ns = DEFAULT_POLL_PREWARM_NS
    nat = native()
    env = BenchEnv(queues)
    try:
        sched = nat.Scheduler(threads)
        runners = []
        for r in env.runners:
            cfg = nat.LoopConfig()
            cfg.poll_period_ns = int(period_s * 1e9)
            cfg.scale_up_cool_down_ns = 0
            cfg.scale_down_cool_down_ns = 0
            cfg.prefetch = True
            cfg.prewarm_ns = prewarm_ns
            rr = nat.Runner(cfg, r.sqs, r.scaler, nat.RealClock(), env.log)
            runners.append(rr)
            sched.add(rr)
        sched.start()
        time.sleep(2 * period_s)
        sched.reset_lateness()
        p0 = sum(r.stats()["polls"] for r in runners)
        c0 = sum(r.stats()["poll_cpu_ns"] for r in runners)
        t0 = time.perf_counter()
        time.sleep(duration_s)
        polls = sum(r.stats()["polls"] for r in runners) - p0
        cpu = sum(r.stats()["poll_cpu_ns"] for r in runners) - c0
        wall = time.perf_counter() - t0
        late, max_late = sched.late_polls(), sched.max_lateness_ns()
        sched.stop()
        sched.join()
        return {
            "queues": queues,
            "threads": threads,
            "poll_period_s": period_s,
            "prewarm_us": prewarm_ns / 1e3,
            "polls_per_s": round(polls / wall, 1),
            "ideal_polls_per_s": round(queues / period_s, 1),
            "late_poll_fraction": round(late / max(polls, 1), 4),
            "max_lateness_ms": round(max_late / 1e6, 3),
            # the pooled threads' CPU in the polls themselves (the warm-up events are not counted)
            "cpu_ms_per_poll": round(cpu / max(polls, 1) / 1e6, 4),
            "cpu_cores": round(cpu / 1e9 / wall, 3),
            "signature_failures": env.sqs.signature_failures(),
        }
    finally:
        env.close()


if __name__ == "__main__":
    import json
    import sys

    for q, p, k in ((256, 1.0, 4), (1024, 1.0, 8), (1024, 0.25, 8)):
        print(json.dumps(run_capacity(q, p, k)), flush=True)
    sys.exit(0)
