"""What the poll path's spinning buys at a production cadence, and what it costs in CPU.

Three spins can sit on a poll: the busy-poll window on every read (--busy-poll, 25 us), and,
within --busy-poll-budget (LoopConfig.spin_budget_ppm; 0 by default since round 5), the pre-poll
warm-up's spin to the due time (LoopConfig.prewarm_spin, near endpoints only) and the spin through
a near endpoint's answer. The arms: the CLI defaults (the window only), a 1 % budget (round 4's
defaults), the same without the warm-up's spin, and no spinning at all. All arms share one run
(queue q runs arm q % arms, starts staggered over the period, one fake SQS and one fake apiserver
process), so the box's idle-state drift does not land between them. One JSON line per arm,
period and endpoint kind: poll->patch p50/p90 and the worker's CPU per poll (the spans' thread
CPU time). (Round 5's r05c/r05d runs named the arms from the 1 % budget's side: "default" was
today's budget_1pct, "window_only" today's default; r05g's budget arms gave each queue 1 %.)

    python scripts/spin_arms.py --period-ms 1000 --polls 27 --queues 8
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.autoscaler import ONE_PERCENT_PPM  # noqa: E402
from kube_sqs_autoscaler_amd.bench.latency import measure_cadenced_arms  # noqa: E402
from kube_sqs_autoscaler_amd.config import DEFAULT_POLL_PREWARM_NS  # noqa: E402

MS = 1_000_000
BASE = dict(mode="scale", pipeline=True, busy_poll_ns=25_000, prewarm_ns=DEFAULT_POLL_PREWARM_NS)


def arms(queues: int) -> dict:
    """The arms, each queue with the budget --busy-poll-budget=1 gives a process of ``queues``
    queues (1 % of the period shared by them)."""
    ppm = ONE_PERCENT_PPM // max(queues, 1)
    return {
        "default": BASE,
        "budget_1pct": dict(BASE, spin_budget_ppm=ppm),
        "budget_1pct_no_warmup_spin": dict(BASE, spin_budget_ppm=ppm, prewarm_spin=False),
        "no_spin": dict(BASE, busy_poll_ns=0),
    }


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--period-ms", type=int, nargs="+", default=[250, 1000])
    ap.add_argument("--polls", type=int, default=27, help="polls per queue (the first two are dropped)")
    ap.add_argument("--queues", type=int, default=8, help="queues per arm")
    ap.add_argument("--sqs-latency-ms", type=float, default=0.0, help="the fake SQS answers this much later")
    ap.add_argument("--kube-latency-ms", type=float, default=0.0, help="the fake apiserver answers this much later")
    ap.add_argument("--sleeping-only", action="store_true", help="skip the endpoints that never sleep")
    a = ap.parse_args()
    lat = dict(sqs_latency_ns=int(a.sqs_latency_ms * MS), kube_latency_ns=int(a.kube_latency_ms * MS))
    for period in a.period_ms:
        for hot in (False,) if a.sleeping_only else (False, True):
            res = measure_cadenced_arms(period * MS, a.polls, a.queues, arms(a.queues), hot_endpoints=hot, **lat)
            for name, r in res.items():
                print(json.dumps({"arm": name, "period_ms": period, "hot_endpoints": hot, "queues": a.queues,
                                  "sqs_latency_ms": a.sqs_latency_ms, "kube_latency_ms": a.kube_latency_ms,
                                  **{k: r.get(k) for k in ("p50_ms", "p90_ms", "samples", "cpu_ms_per_poll",
                                                           "cpu_ms_per_poll_p50", "phase_median_us")}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
