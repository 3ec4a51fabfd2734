"""``python -m kube_sqs_autoscaler_amd.tune``: rank autoscaler settings against a queue trace.

Example -- replay a day of recorded polls, sweep cool-downs and thresholds, keep configurations
whose queue pressure stays under a bound, and rank them by pod cost::

    python -m kube_sqs_autoscaler_amd.tune --trace spans.jsonl --horizon 24h \\
        --grid scale-up-cool-down=0s:10m:10s --grid scale-down-cool-down=30s:30m:30s \\
        --grid scale-up-messages=50,100,200,400 --grid max-pods=8 \\
        --max-backlog 5e9 --objective pod_ms --top 10

Grid keys are the autoscaler's own flag names; values use its syntax (Go durations, base-0 ints),
as comma lists or ``start:stop:step`` ranges (stop inclusive). The sweep runs on the MI355X
(``--device gpu``) or on CPU threads; both give identical numbers.

Closed loop (:mod:`.closedloop`): with ``--arrivals`` (``seconds,msgs_per_second`` CSV) instead of
``--trace`` the queue is simulated -- the candidate's replicas drain it at ``--service-rate``
msgs/s per ready pod after ``--startup-delay`` -- over ``--seeds`` random arrival sequences, and
configurations are ranked by mean pod-hours subject to the 95th-percentile time above
``--slo-backlog``::

    python -m kube_sqs_autoscaler_amd.tune --arrivals rate.csv --horizon 24h \
        --service-rate 4 --startup-delay 90s --slo-backlog 500 --max-violation 10m --seeds 64 \
        --grid scale-up-cool-down=0s:10m:30s --grid max-pods=8,16,32 --top 10
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from typing import Dict, List

import numpy as np

from ..utils.goflag import parse_duration, parse_int
from . import closedloop, distributed, sweep

FLAG_TO_FIELD = {
    "poll-period": ("poll_ns", parse_duration),
    "scale-up-cool-down": ("up_cool_ns", parse_duration),
    "scale-down-cool-down": ("down_cool_ns", parse_duration),
    "scale-up-messages": ("up_msgs", parse_int),
    "scale-down-messages": ("down_msgs", parse_int),
    "scale-up-pods": ("up_pods", parse_int),
    "scale-down-pods": ("down_pods", parse_int),
    "max-pods": ("max_pods", parse_int),
    "min-pods": ("min_pods", parse_int),
}


def parse_values(spec: str, conv) -> List[int]:
    out: List[int] = []
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        if ":" in part:
            a, b, c = (conv(x) for x in part.split(":"))
            if c <= 0:
                raise ValueError(f"range step must be positive: {part}")
            out.extend(range(a, b + 1, c))
        else:
            out.append(conv(part))
    if not out:
        raise ValueError(f"no values in {spec!r}")
    return out


def parse_grid(items: List[str]) -> Dict[str, List[int]]:
    g: Dict[str, List[int]] = {}
    for item in items:
        key, _, spec = item.partition("=")
        if key not in FLAG_TO_FIELD:
            raise ValueError(f"unknown grid key {key!r}; expected one of {sorted(FLAG_TO_FIELD)}")
        field, conv = FLAG_TO_FIELD[key]
        g[field] = parse_values(spec, conv)
    return g


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m kube_sqs_autoscaler_amd.tune", description=__doc__.splitlines()[0])
    src = ap.add_mutually_exclusive_group(required=True)
    src.add_argument("--trace", help="--trace-file span log (.jsonl) or seconds,depth CSV (open loop)")
    src.add_argument("--arrivals", help="seconds,msgs_per_second CSV: simulate the queue (closed loop)")
    ap.add_argument("--queue", default=None, help="queue URL or ns/deployment to select from a multi-queue span log")
    ap.add_argument("--horizon", default="", help="simulated time (Go duration); default: trace length + 1 poll period")
    ap.add_argument("--init-replicas", type=int, default=1)
    ap.add_argument("--latency", default="1ms,1ms,1ms",
                    help="SQS, GET, write latency (Go durations); whole milliseconds, with whole-millisecond poll "
                         "periods, let the simulators run on 32-bit millisecond clocks (faster, same results)")
    ap.add_argument("--grid", action="append", default=[], help="flag=values (repeatable)")
    ap.add_argument("--objective", default=None,
                    help="open loop: pod_ms|backlog|ups|downs (default pod_ms); closed loop: a summary column "
                         "(default pod_hours_mean)")
    ap.add_argument("--max-backlog", type=float, default=None, help="keep configs with backlog <= this")
    ap.add_argument("--top", type=int, default=10, help="rows to print (0: all)")
    ap.add_argument("--pareto", action="store_true", help="list the cost/pressure Pareto front instead of a ranking")
    ap.add_argument("--device", default="auto", choices=["auto", "gpu", "cpu"])
    ap.add_argument("--json", action="store_true", help="print JSON lines instead of a table")
    ap.add_argument("--distributed", action="store_true",
                    help="shard the grid over the ranks of a torchrun launch (one GPU each); rank 0 prints")
    cl = ap.add_argument_group("closed loop (--arrivals)")
    cl.add_argument("--service-rate", type=float, default=None, help="msgs/s one ready pod drains (required)")
    cl.add_argument("--startup-delay", default="60s", help="scale-up write -> new pods taking work (Go duration)")
    cl.add_argument("--slo-backlog", type=int, default=1000, help="backlog (msgs) above which time is a violation")
    cl.add_argument("--init-backlog", type=int, default=0, help="msgs queued at t=0")
    cl.add_argument("--max-violation", default=None, help="keep configs whose p95 time above --slo-backlog <= this")
    cl.add_argument("--seeds", type=int, default=32, help="random arrival sequences per configuration")
    cl.add_argument("--seed", type=int, default=1, help="first seed (the same seeds are used for every config)")
    a = ap.parse_args(argv)
    group = distributed.Group(a.device) if a.distributed else None
    try:
        if a.arrivals is not None:
            return _closed_loop(ap, a, group)
        return _open_loop(ap, a, group)
    finally:
        if group is not None:
            group.close()


def _open_loop(ap: argparse.ArgumentParser, a, group) -> int:
    if a.trace is None:
        ap.error("one of --trace or --arrivals is required")
    if a.objective is None:
        a.objective = "pod_ms"
    if a.objective not in ("pod_ms", "backlog", "ups", "downs"):
        ap.error(f"open-loop objective must be pod_ms, backlog, ups or downs, not {a.objective!r}")

    tr = sweep.Trace.from_spans(a.trace, a.queue) if a.trace.endswith((".jsonl", ".json")) else sweep.Trace.from_csv(a.trace)
    lat = tuple(parse_duration(x) for x in a.latency.split(","))
    if len(lat) != 3:
        ap.error("--latency needs three durations")
    values = parse_grid(a.grid)
    params = sweep.grid(**values)
    horizon = parse_duration(a.horizon) if a.horizon else int(tr.t_ns[-1]) + int(params[0].max())
    t0 = time.perf_counter()
    if group is not None:
        res = distributed.run_open_loop(group, tr, params, a.init_replicas, horizon, lat)
    else:
        res = sweep.run(tr, params, a.init_replicas, horizon, lat, a.device)
    wall = time.perf_counter() - t0
    if group is not None and group.rank != 0:
        return 0
    ok = np.ones(len(res), dtype=bool)
    if a.max_backlog is not None:
        ok &= res.out["backlog"] <= a.max_backlog
    idx = np.flatnonzero(ok)
    if a.pareto:
        front = sweep.pareto_front(res.out["pod_ms"][idx], res.out["backlog"][idx])
        order = idx[front][: a.top] if a.top > 0 else idx[front]
    else:
        order = idx[np.argsort(res.out[a.objective][idx], kind="stable")]
        order = order[: a.top] if a.top > 0 else order
    baseline = sweep.run(tr, sweep.grid(), a.init_replicas, horizon, lat, "cpu").row(0)
    summary = {"configs": len(res), "feasible": int(ok.sum()), "device": res.device, "wall_s": round(wall, 4),
               "ranks": group.world if group is not None else 1,
               "kernel_ms": round(res.kernel_ms, 3), "simulated_polls": int(res.out["polls"].sum()),
               "clock": "ms" if res.ms_clock else "ns", "steady_skip": res.skip, "horizon_ns": horizon,
               "reference_defaults": baseline}
    if a.json:
        print(json.dumps(summary))
        for i in order:
            print(json.dumps(res.row(int(i))))
        return 0
    print(f"{len(res)} configs ({int(ok.sum())} feasible) on {res.device} in {wall:.3f} s, "
          f"{summary['simulated_polls']:.3g} polls simulated")
    print(f"reference defaults: pod_ms={baseline['pod_ms']} backlog={baseline['backlog']} "
          f"ups={baseline['ups']} downs={baseline['downs']}")
    cols = ["poll_ns", "up_cool_ns", "down_cool_ns", "up_msgs", "down_msgs", "up_pods", "down_pods", "max_pods",
            "min_pods", "pod_ms", "backlog", "ups", "downs", "max_replicas"]
    print("\t".join(cols))
    for i in order:
        r = res.row(int(i))
        print("\t".join(str(r[c]) for c in cols))
    return 0


CLOSED_COLS = ["poll_ns", "up_cool_ns", "down_cool_ns", "up_msgs", "down_msgs", "up_pods", "down_pods", "max_pods",
               "min_pods", "pod_hours_mean", "backlog_mean", "violation_s_p95", "peak_backlog_p95", "ups_mean",
               "downs_mean", "max_replicas_max"]


def _closed_loop(ap: argparse.ArgumentParser, a, group) -> int:
    if a.service_rate is None:
        ap.error("--arrivals needs --service-rate")
    objective = a.objective or "pod_hours_mean"
    tr = closedloop.ArrivalTrace.from_csv(a.arrivals)
    lat = tuple(parse_duration(x) for x in a.latency.split(","))
    if len(lat) != 3:
        ap.error("--latency needs three durations")
    model = closedloop.QueueModel(a.service_rate, parse_duration(a.startup_delay), a.slo_backlog, a.init_backlog)
    params = sweep.grid(**parse_grid(a.grid))
    horizon = parse_duration(a.horizon) if a.horizon else int(tr.t_ms[-1]) * 1_000_000 + 3600 * closedloop.S
    t0 = time.perf_counter()
    if group is not None:
        res = distributed.run_closed_loop(group, tr, params, model, a.init_replicas, horizon, lat, a.seeds, a.seed)
    else:
        res = closedloop.run(tr, params, model, a.init_replicas, horizon, lat, a.seeds, a.seed, a.device)
    wall = time.perf_counter() - t0
    if group is not None and group.rank != 0:
        return 0
    summ = res.summary()
    if objective not in summ:
        ap.error(f"closed-loop objective must be one of {sorted(summ)}, not {objective!r}")
    ok = np.ones(len(res), dtype=bool)
    if a.max_violation is not None:
        ok &= summ["violation_s_p95"] <= parse_duration(a.max_violation) / 1e9
    if a.max_backlog is not None:
        ok &= summ["backlog_mean"] <= a.max_backlog
    idx = np.flatnonzero(ok)
    if a.pareto:
        front = sweep.pareto_front(summ["pod_hours_mean"][idx], summ["violation_s_p95"][idx])
        order = idx[front][: a.top] if a.top > 0 else idx[front]
    else:
        order = idx[np.argsort(summ[objective][idx], kind="stable")]
        order = order[: a.top] if a.top > 0 else order
    base = closedloop.run(tr, sweep.grid(), model, a.init_replicas, horizon, lat, a.seeds, a.seed, "cpu").row(0)
    info = {"configs": len(res), "feasible": int(ok.sum()), "seeds": a.seeds, "device": res.device,
            "ranks": group.world if group is not None else 1,
            "wall_s": round(wall, 4), "kernel_ms": round(res.kernel_ms, 3),
            "simulated_polls": int(res.out["polls"].sum()),
            "arith": ("fast" if res.fast_arith else "saturating") + ("+ms" if res.ms_clock else ""),
            "horizon_ns": horizon, "reference_defaults": base}
    if a.json:
        print(json.dumps(info))
        for i in order:
            print(json.dumps(res.row(int(i))))
        return 0
    print(f"{len(res)} configs x {a.seeds} seeds ({int(ok.sum())} feasible) on {res.device} in {wall:.3f} s, "
          f"{info['simulated_polls']:.3g} polls simulated")
    print(f"reference defaults: pod_hours={base['pod_hours_mean']:.3f} backlog={base['backlog_mean']:.1f} "
          f"violation_p95={base['violation_s_p95']:.0f}s ups={base['ups_mean']:.1f}")
    print("\t".join(CLOSED_COLS))
    for i in order:
        r = res.row(int(i))
        print("\t".join(f"{r[c]:.4g}" if isinstance(r[c], float) else str(r[c]) for c in CLOSED_COLS))
    return 0


if __name__ == "__main__":
    sys.exit(main())
