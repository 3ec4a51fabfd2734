"""Poll->patch latency at the reference's own poll period, 5 s (/root/reference/main.go:83).

bench.py's cadence rows stop at 1 s so that the whole bench fits the driver's budget. This runs
the same measurement (bench/latency.py ``measure_cadenced_arms``: one thread per queue, starts
staggered over the period, one fake SQS process and one fake apiserver process serving every
queue, every poll scaling) at 5 s, with many queues and few polls each, so that ~400 samples per
path take 40 s per row: the CLI defaults and the reference-equivalent path (full-Deployment
GET + PUT, sequential, no warm-up, no busy-poll) as paired arms of one run, plain and TLS. One
JSON line per path and row, with each path's worker CPU per poll.

``--presend-ab``: the arms are the CLI defaults with and without ``--poll-presend`` instead (the
evidence that decides its default: on only if it is at most 0.95x in every run).

    python scripts/cadence_5s.py --queues 64 --polls 8
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.bench.latency import measure_cadenced_arms  # noqa: E402
from kube_sqs_autoscaler_amd.config import DEFAULT_POLL_PREWARM_NS  # noqa: E402

MS = 1_000_000


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--period-ms", type=int, default=5000)
    ap.add_argument("--queues", type=int, default=64, help="per path")
    ap.add_argument("--polls", type=int, default=8, help="per queue; the first 2 of each are dropped")
    ap.add_argument("--presend-ab", action="store_true", help="arms: the defaults with and without --poll-presend")
    a = ap.parse_args()
    default = dict(mode="scale", pipeline=True, busy_poll_ns=25_000, prewarm_ns=DEFAULT_POLL_PREWARM_NS)
    if a.presend_ab:
        arms = {"default": default, "default_presend": dict(default, presend=True)}
    else:
        arms = {"default": default,
                "reference_equivalent": dict(mode="deployment", pipeline=False, busy_poll_ns=0, prewarm_ns=0)}
    for tls in (False, True):
        res = measure_cadenced_arms(a.period_ms * MS, a.polls, a.queues, arms, tls)
        for name, r in res.items():
            out = {"row": name + ("_tls" if tls else ""), "period_ms": a.period_ms, "queues": a.queues,
                   "paired_with": r.get("paired_with")}
            out.update({k: r[k] for k in ("p50_ms", "p90_ms", "p99_ms", "samples", "errors", "signature_failures",
                                          "cpu_ms_per_poll") if k in r})
            out["phase_median_us"] = r.get("phase_median_us")
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
