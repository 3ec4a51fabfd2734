"""Paired A/B of the poll-path knobs at a production cadence.

The cadence rows of ``bench.py`` compare whole configurations in separate runs, so run-to-run
noise (loopback send cost, scheduler placement) lands between them. Here the arms share one run:
queue q gets arm q % 4, all
queues against the same endpoint process, starts staggered over the period. The arms (ARMS):
``--poll-prewarm=200us`` and ``--busy-poll=25us`` with ``--busy-poll-budget=1`` (round 4's
defaults), the same without the spin budget (the CLI defaults since round 5), no warm-up, and a
fixed 300 us busy-poll window. One
JSON line per arm and endpoint kind (fakes that sleep / never sleep): poll->patch p50/p90 and the
per-call phase medians (``HttpTiming``, see ``bench/latency.py``; ``--untimed`` drops them).

    python scripts/cadence_arms.py --period-ms 1000 --polls 27 --queues 16
"""
import argparse
import json
import os
import statistics
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.autoscaler import ONE_PERCENT_PPM  # noqa: E402
from kube_sqs_autoscaler_amd.bench.latency import BenchEnv, _detail_medians  # noqa: E402

MS = 1_000_000
# (prewarm ns, busy-poll ns, spin budget): --busy-poll-budget=1 (None: the process's 1 % of the
# period shared by its queues, autoscaler.loop_config), the same without the spin budget (the CLI
# defaults), no warm-up, and a 300 us fixed window
ARMS = [(200_000, 25_000, None), (200_000, 25_000, 0), (0, 25_000, 0), (200_000, 300_000, 0)]


def run(period_ms: int, polls: int, queues: int, skip: int = 2, timed: bool = True) -> None:
    for hot in (False, True):
        env = BenchEnv(queues, "scale", pipeline=True, busy_poll_ns=[a[1] for a in ARMS], servers="process",
                       poll_period_ns=period_ms * MS, stagger=True, hot_endpoints=hot,
                       prewarm_ns=[a[0] for a in ARMS],
                       spin_budget_ppm=[ONE_PERCENT_PPM // queues if a[2] is None else a[2] for a in ARMS],
                       timing=timed)
        files = [tempfile.TemporaryFile() for _ in env.runners]
        try:
            for r, f in zip(env.runners, files):
                r.set_trace_fd(f.fileno())
            env.run(polls)
            per_arm = {i: [] for i in range(len(ARMS))}
            for q, (r, f) in enumerate(zip(env.runners, files)):
                r.set_trace_fd(-1)
                f.seek(0)
                per_arm[q % len(ARMS)] += [json.loads(x) for x in f.read().decode().splitlines()][skip:]
        finally:
            for f in files:
                f.close()
            env.close()
        for i, (prewarm, busy, budget) in enumerate(ARMS):
            spans = [s for s in per_arm[i] if s["patch_latency_ns"] >= 0]
            lat = sorted(s["patch_latency_ns"] for s in spans)
            if not lat:
                continue
            print(json.dumps({"period_ms": period_ms, "hot_endpoints": hot, "timed": timed, "prewarm_us": prewarm / 1e3,
                              "busy_poll_us": busy / 1e3, "spin_budget": "1%/queues" if budget is None else budget,
                              "samples": len(lat),
                              "p50_us": round(lat[len(lat) // 2] / 1e3, 1),
                              "p90_us": round(lat[int(len(lat) * 0.9)] / 1e3, 1),
                              "depth_us": round(statistics.median(s["depth_ns"] for s in spans) / 1e3, 1),
                              "write_us": round(statistics.median(s["update_ns"] for s in spans) / 1e3, 1),
                              "calls": _detail_medians(spans)}), flush=True)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--period-ms", type=int, default=1000)
    ap.add_argument("--polls", type=int, default=27, help="polls per queue (the first two are dropped)")
    ap.add_argument("--queues", type=int, default=16, help="a multiple of 4: each arm gets queues / 4")
    ap.add_argument("--untimed", action="store_true", help="no per-call timing (the p50s without its syscalls)")
    a = ap.parse_args()
    if a.queues % len(ARMS):
        ap.error("--queues must be a multiple of 4")
    run(a.period_ms, a.polls, a.queues, timed=not a.untimed)
    return 0


if __name__ == "__main__":
    sys.exit(main())
