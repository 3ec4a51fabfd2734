#!/usr/bin/env python3
"""Headline benchmark: poll -> scale-patch p50 latency (ms) + decision parity.

BASELINE.json names the metric "poll->scale-patch p50 latency (ms); decision parity vs ref on
synthetic trace", reported at 1/2/4/8 concurrently tracked queues. The reference publishes no
number (BASELINE.json ``published: {}``), so ``vs_baseline`` is null.

One rank per GPU (``torch.distributed``; backend ``nccl`` = RCCL on ROCm when every rank has a
GPU of its own, ``gloo`` otherwise). Each rank is one autoscaler process tracking ``--queues``
queues (default 1) against its own localhost fake SQS + fake kube-apiserver, so the job tracks
``N x queues`` queues in total (weak scaling). The ranks share nothing while timed -- each is an
independent control-plane process, as N reference deployments would be; the collective
(``all_gather``) only pools the latency samples for the job-wide p50 afterwards. A "step" is
one control-loop iteration on every tracked queue: SigV4-signed SQS GetQueueAttributes -> Deployment GET -> replica write (the trace
alternates 200/0 messages, so every iteration scales). K timed steps are bracketed by a barrier
+ ``torch.cuda.synchronize()``; ``value`` is the p50 over every sample of every rank.

Secondary rows (single rank; fixed ``--secondary-samples`` per queue, three interleaved rounds,
median): p50 at 1/2/4/8 tracked queues with the default thread-per-queue fleet and with
``--worker-processes`` (each queue against its own fake endpoint process), the strictly
sequential and reference-equivalent paths, TLS, a regional-RTT model, per-phase medians,
wire-path decision parity and apiserver requests per poll on the Appendix C traces; and the
production-cadence rows (250 ms and 1 s poll periods, 1/2/4/8 and 16 queues, sleeping and
busy-polling endpoints, the regional-RTT model at 1 s, the default and reference-equivalent paths
as paired arms of each run, each with its worker CPU per poll: ``_cadence_rows``), run on the
first ceil(cgroup CPU quota) CPUs when the quota allows fewer cores than the CPUs visible
(``--cadence-cpus``, recorded as ``cadenced_rows_cpus``).

Launch: ``python bench.py --gpus N`` with N > 1 outside a launcher starts the N ranks itself
(child processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set,
before the parent touches torch or the GPU) and exits with the first failing rank's status;
under ``torchrun`` the launcher's WORLD_SIZE must equal ``--gpus`` (exit 2 otherwise). A node
with fewer visible GPUs than ranks exits 2, unless ``--rehearse-shared-gpus``: then the ranks
share GPUs over gloo and ``n_gpus`` is the number of GPUs actually used.

Output: rank 0 prints ONE compact JSON line on stdout, at most 4,096 bytes (``result_line``): the
headline keys and the summary rows. The full result -- every row, round and breakdown -- goes
to ``--detail-out`` (default ``gpurun_out/bench_detail.json``), which the line names.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--queues Q] [--mode scale] [--detail-out F]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "poll→scale-patch p50 latency (ms); decision parity vs ref on synthetic trace"

# The driver parses the LAST line of stdout out of an 8,000-character tail; round 5's 24.6 KB
# line lost its head there and was recorded unparsed (BENCH_r05.json). The line therefore holds
# the headline keys and the summary rows only, compact and at most LINE_LIMIT bytes; the full
# result (per-round cells, phase breakdowns, setups) goes to the --detail-out file it names.
LINE_LIMIT = 4096
# extra keys carried on the line, most important first; past LINE_LIMIT the last go first
LINE_EXTRA_KEYS = ("samples", "p90_ms", "p99_ms", "signature_failures", "tracked_queues", "ranks",
                   "collective_backend", "rehearsal_shared_gpus", "decision_parity", "skipped_sections",
                   "section_errors", "p50_ms_by_tracked_queues", "wan_cadenced_p50_ms", "cpu_ms_per_poll",
                   "cadenced_reference_over_default", "cadenced_p50_ms_by_tracked_queues")


def result_line(out: dict, detail: str | None) -> str:
    """The one stdout line of ``out`` (the full result): every top-level key, ``parallelism``
    lifted out of ``config``, and an ``extra`` of LINE_EXTRA_KEYS only -- the decision parity as
    its fraction and poll count, section errors cut to 200 characters -- plus ``detail``, the file
    holding everything. Rows are dropped from the end of LINE_EXTRA_KEYS (and named under
    ``dropped_from_line``) until the line fits LINE_LIMIT bytes."""
    full = out.get("extra", {})
    extra = {k: full[k] for k in LINE_EXTRA_KEYS if k in full}
    if isinstance(extra.get("decision_parity"), dict):
        dp = extra["decision_parity"]
        agree = total = 0
        for row in (dp.get("configs") or {}).values():
            a, b = str(row.get("agree", "0/0")).split("/")
            agree, total = agree + int(a), total + int(b)
        extra["decision_parity"] = {"fraction": dp.get("fraction"), "polls": f"{agree}/{total}"}
    if "section_errors" in extra:
        extra["section_errors"] = {k: str(v)[:200] for k, v in extra["section_errors"].items()}
    extra["detail"] = detail
    line = {k: v for k, v in out.items() if k != "extra"}
    line["parallelism"] = out.get("config", {}).get("parallelism")
    line["extra"] = extra

    def dumps() -> str:
        return json.dumps(line, separators=(",", ":"), ensure_ascii=False)

    s = dumps()
    for k in reversed(LINE_EXTRA_KEYS):
        if len(s.encode()) <= LINE_LIMIT:
            break
        if k in extra:
            del extra[k]
            extra.setdefault("dropped_from_line", []).append(k)
            s = dumps()
    if len(s.encode()) > LINE_LIMIT:  # only the headline is left: cut the free-text fields
        line["data"] = str(line.get("data", ""))[:200]
        line["config"] = {**line.get("config", {}), "model": str(line.get("config", {}).get("model", ""))[:300]}
        s = dumps()
    return s


def write_detail(out: dict, path: str) -> str | None:
    """The full result as JSON at ``path`` (written to a temporary name, then renamed); the path
    written, or None when it cannot be written (the line then says so)."""
    try:
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump(out, f, indent=1)
            f.write("\n")
        os.replace(tmp, path)
        return path
    except OSError as e:
        _progress(f"--detail-out {path}: {e}")
        return None


def _parity_summary() -> dict:
    """Decision parity of the timed configuration: the five Appendix C scenarios through the
    production wire path (SigV4 HttpSqsApi + KubeRestDeployments over HTTP to the fakes, VirtualClock),
    poll by poll against the reference-semantics oracle -- for the default (pipelined /scale, the
    timed row), strictly sequential /scale, the reference-equivalent full-Deployment GET+PUT, and
    round 1's speculative GET on every poll (for its apiserver traffic)."""
    from kube_sqs_autoscaler_amd.models import parity

    wire = parity.wire_summary()
    agree = total = 0
    for row in wire.values():
        a, b = row["agree"].split("/")
        agree, total = agree + int(a), total + int(b)
    return {"path": "wire: HttpSqsApi + KubeRestDeployments -> FakeSqsServer/FakeKubeServer, VirtualClock, zero-latency oracle",
            "fraction": agree / total if total else 1.0, "configs": wire}


def _apiserver_requests_per_poll(wire: dict) -> dict:
    """Per scenario, kube-apiserver requests per poll (GETs + writes) for each config, next to
    the reference's own count on the same trace."""
    out = {}
    for key, row in wire["configs"].items():
        for sc, r in row["scenarios"].items():
            out.setdefault(sc, {})[key] = r["apiserver_requests_per_poll"]
    for sc in out:
        r = wire["configs"]["deployment"]["scenarios"][sc]
        polls = int(r["agree"].split("/")[1])
        out[sc]["reference"] = round((r["reference_gets"] + r["writes"]) / polls, 4)
    return out


def _progress(msg: str) -> None:
    """One line per finished row on stderr (stdout carries only the result line): a run of
    several minutes shows that it is alive."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def _cadence_rows(args, pipeline: bool, bp: int, hot_p50_ms: float, deadline: float = float("inf")) -> dict:
    """Poll->patch latency at production poll periods (250 ms and 1 s; the reference's default
    is 5 s, /root/reference/main.go:83), one thread per queue, staggered over the period, against
    the ``split`` fake endpoints: one fake SQS process and one fake apiserver process serving
    every queue, as production has two services (bench/latency.py ``measure_cadenced_arms``).
    Every row runs the default path (the CLI's flags: --poll-prewarm, --busy-poll) and the
    reference-equivalent path (full-Deployment GET+PUT, sequential, no warm-up, no busy-poll) as
    paired arms of ONE run, their queues interleaved: a box's idle-state and frequency behaviour
    drifts between runs and moved single-path runs of one path by 2x
    (profiles/r04c_cadence_probe.jsonl), so paths compared in separate runs could invert by
    chance. Every row also reports each arm's worker CPU per poll (``cpu_ms_per_poll``, the
    spans' thread CPU time: warm-up, spinning and the poll). In this order, most important first:

    1. BASELINE's queue axis at 250 ms: 1, 2, 4 and 8 tracked queues per path, at least
       ``--cadence-queue-samples`` scaling polls per path, in ``--cadence-queue-rounds``
       interleaved rounds pooled per cell (``cadenced_p50_ms_by_tracked_queues``);
    2. the regional-RTT model at a cadence (``wan_cadenced_p50_ms``, ``cpu_ms_per_poll``): 1 s,
       the fakes answering SQS after 2 ms and the apiserver after 1 ms -- the structural saving
       (one apiserver round trip, overlapped) at the CPU each path spends;
    3. the queue axis again against endpoints that never sleep (``_hot_endpoints``: a loaded
       production endpoint), and timed at 1 and 8 queues (every call broken down on the client,
       HttpTiming, and on the fakes, wake-up and service time per request) -- the attribution of
       the axis's growth (``cadenced_by_tracked_queues_attribution``);
    4. ``--cadence-queues`` queues per path at 250 ms, plain and TLS, and at 1 s, plain and with
       hot endpoints; then 1 s timed.

    Rows that would start past ``deadline`` (time.monotonic) are skipped and listed."""
    import math

    from kube_sqs_autoscaler_amd.bench.latency import measure_cadenced_arms
    from kube_sqs_autoscaler_amd.config import DEFAULT_POLL_PREWARM_NS

    ms = 1_000_000
    skip = 2  # each queue's first polls (dial, first allocations) are dropped
    arms = {"default": dict(mode=args.mode, pipeline=pipeline, busy_poll_ns=bp, prewarm_ns=DEFAULT_POLL_PREWARM_NS),
            "reference_equivalent": dict(mode="deployment", pipeline=False, busy_poll_ns=0, prewarm_ns=0)}
    # plan rows: (group, period label, period ns, suffix, queues per arm, polls per queue, tls, hot, timing, wan)
    # The queue axis runs in ROUNDS interleaved rounds of 1, 2, 4, 8 queues, each cell's samples
    # pooled over its rounds: a box's idle state drifts over tens of seconds (one 1-queue cell
    # read 0.20 ms and the next run's 0.09 ms, profiles/r05e, r05g), and cells measured in one
    # stretch each put that drift between them.
    rounds = max(1, int(getattr(args, "cadence_queue_rounds", 3)))
    by_q_polls = lambda q: math.ceil(args.cadence_queue_samples / rounds / q) + skip  # noqa: E731
    plan = [("by_queues", "250ms", 250 * ms, f"/{q}", q, by_q_polls(q), False, False, False, False)
            for _ in range(rounds) for q in (1, 2, 4, 8)]
    plan.append(("wan", "1s", 1000 * ms, "_wan_sqs2ms_kube1ms", args.cadence_queues, args.cadence_polls,
                 False, False, False, True))
    plan += [("by_queues_hot", "250ms", 250 * ms, f"/{q}", q, by_q_polls(q), False, True, False, False)
             for _ in range(rounds) for q in (1, 2, 4, 8)]
    plan += [("by_queues_timed", "250ms", 250 * ms, f"/{q}", q, by_q_polls(q), False, False, True, False) for q in (1, 8)]
    for label, period, variants in (("250ms", 250 * ms, ((False, False), (True, False))),
                                    ("1s", 1000 * ms, ((False, False), (False, True)))):
        for tls, hot in variants:
            suffix = ("_tls" if tls else "") + ("_hot_endpoints" if hot else "")
            plan.append(("fleet", label, period, suffix, args.cadence_queues, args.cadence_polls, tls, hot, False, False))
    plan.append(("fleet", "1s", 1000 * ms, "_timed", args.cadence_queues, args.cadence_polls, False, False, True, False))
    skipped = []
    p50, rows, cpu = {}, {}, {}
    by_q = {"250ms": {}, "250ms_hot_endpoints": {}}
    by_q_samples, by_q_setup, attribution = {}, {}, {}
    pooled = {}  # (setup key, arm, queues) -> ([latency ns], [cpu ns], [per-round p50 ms])
    for group, label, period, suffix, queues, polls, tls, hot, timing, wan in plan:
        if time.monotonic() > deadline:
            if f"{label}/{group}{suffix}" not in skipped:
                skipped.append(f"{label}/{group}{suffix}")
            continue
        by_queue_row = group in ("by_queues", "by_queues_hot")
        res = measure_cadenced_arms(period, polls, queues, arms, tls, skip=skip, hot_endpoints=hot, timing=timing,
                                    sqs_latency_ns=2 * ms if wan else 0, kube_latency_ns=1 * ms if wan else 0,
                                    keep_samples=by_queue_row)
        for name, r in res.items():
            if by_queue_row:
                key = "250ms" + ("_hot_endpoints" if hot else "")
                lat, cpus, rounds_p50 = pooled.setdefault((key, name, queues), ([], [], []))
                lat += r.pop("latencies_ns")
                cpus += r.pop("cpu_ns")
                rounds_p50.append(r["p50_ms"])
                by_q[key].setdefault(name, {})[str(queues)] = round(_pct(lat, 50) / 1e6, 4) if lat else None
                by_q_samples.setdefault(key, {}).setdefault(name, {})[str(queues)] = len(lat)
                cpu.setdefault(f"{key}_by_tracked_queues", {}).setdefault(name, {})[str(queues)] = (
                    round(sum(cpus) / len(cpus) / 1e6, 4) if cpus else None)
                if name == "default":
                    by_q_setup.setdefault(key, {})[str(queues)] = r["setup"]
            elif group == "by_queues_timed":
                attribution.setdefault(str(queues), {})[name] = {
                    k: r.get(k) for k in ("p50_ms", "phase_median_us", "call_phase_median_us", "endpoint_median_us",
                                          "setup")}
            else:
                rows.setdefault(label, {})[name + suffix] = r
                cpu.setdefault(label + suffix, {})[name] = r.get("cpu_ms_per_poll")
                if not timing:
                    p50.setdefault(label, {})[name + suffix] = r["p50_ms"]
        _progress(f"cadence {label} {group}{suffix} ({queues} queues per path): " +
                  ", ".join(f"{name} p50 {r['p50_ms']} ms over {r['samples']}, cpu {r.get('cpu_ms_per_poll')} ms/poll"
                            for name, r in res.items()))
    if skipped:
        _progress(f"cadence rows skipped (past --extras-budget-s): {skipped}")
    wan_p50 = {k[:-len("_wan_sqs2ms_kube1ms")]: v for k, v in p50.get("1s", {}).items()
               if k.endswith("_wan_sqs2ms_kube1ms")}
    growth = {}
    for key, row in by_q.items():
        for name, v in row.items():
            if v.get("1") and v.get("8"):
                growth.setdefault(key, {})[name] = round(v["8"] / v["1"], 2)
    return {
        **({"cadenced_rows_skipped": skipped} if skipped else {}),
        "cadenced_rows": rows,
        "cadenced_samples": {k: {n: r["samples"] for n, r in v.items()} for k, v in rows.items()},
        "cadenced_by_tracked_queues_samples": by_q_samples,
        "cadenced_by_tracked_queues_setup": by_q_setup,
        "cadenced_by_tracked_queues_setup_note": (
            "q tracked queues per path, one thread each; the default and the reference-equivalent path's queues "
            "interleaved in one run (2q threads, starts staggered over the period) against one fake SQS process and "
            "one fake apiserver process (thread per connection; _hot_endpoints: one busy-polling thread each)"),
        "cadenced_by_tracked_queues_attribution": attribution,
        "cadenced_by_tracked_queues_rounds_p50_ms": {
            f"{key}/{name}/{q}": v[2] for (key, name, q), v in pooled.items()},
        "cadenced_vs_hot_loop_default_plain": {k: round(v["default"] / hot_p50_ms, 2) for k, v in p50.items()
                                               if "default" in v},
        "cadenced_reference_over_default": _ratios(p50, by_q),
        "cadenced_p50_ms": p50,
        "cadenced_by_tracked_queues_8_over_1": growth,
        "cadenced_p50_ms_by_tracked_queues": {k: v for k, v in by_q.items() if v},
        "cpu_ms_per_poll_all_rows": cpu,
        "wan_cadenced_p50_ms": wan_p50,
        "cpu_ms_per_poll": cpu.get("1s_wan_sqs2ms_kube1ms", {}),
    }


def _cadence_cpus(mode: str):
    """The CPUs the cadence rows run on (``--cadence-cpus``): ``auto`` confines this process --
    the autoscaler's threads and the endpoint processes it starts, which inherit it -- to the
    first ceil(quota) of the CPUs it may use when a cgroup CPU quota allows fewer cores than
    that (at least 4), so the rows' threads stay on a compact set of cores the quota can feed
    instead of spreading over the whole host (256 CPUs and a 16-core quota on the MI355X box:
    profiles/r05x had the 8-queue cell 1.3-1.4x the 1-queue cell in every round against
    never-sleeping endpoints). ``off``: no change; a number: that many CPUs. Returns the CPU
    list, or None when unchanged."""
    import math

    if mode == "off":
        return None
    allowed = sorted(os.sched_getaffinity(0))
    if mode == "auto":
        from kube_sqs_autoscaler_amd.ops import native

        quota, period = native().read_cpu_quota()
        if not quota:
            return None
        n = max(4, math.ceil(quota / period))
    else:
        n = max(1, int(mode))
    if n >= len(allowed):
        return None
    return allowed[:n]


def _pct(v, p: float) -> int:
    """Nearest-rank percentile of ``v`` (ns)."""
    import math

    v = sorted(v)
    return v[min(len(v), max(1, math.ceil(p / 100.0 * len(v)))) - 1]


def _ratios(p50: dict, by_q: dict) -> dict:
    """Per paired cell, reference-equivalent p50 / default p50 (> 1: the default path is faster)."""
    out = {}
    for label, row in p50.items():
        for key, v in row.items():
            if key.startswith("default"):
                ref = row.get("reference_equivalent" + key[len("default"):])
                if ref and v:
                    out.setdefault(label, {})[key[len("default"):].lstrip("_") or "plain"] = round(ref / v, 2)
    for setup, row in by_q.items():
        d, r = row.get("default", {}), row.get("reference_equivalent", {})
        for q in d:
            if r.get(q) and d[q]:
                out.setdefault(f"{setup}_by_tracked_queues", {})[q] = round(r[q] / d[q], 2)
    return out


def _pin_rank(mode: str):
    """Confines this rank (every thread it starts from here on: its worker, its fakes' servers,
    the collective's) to slice LOCAL_RANK of LOCAL_WORLD_SIZE contiguous slices of the CPUs it
    may run on, so the ranks of one node do not migrate onto each other's cores. Returns the
    CPU list, or None when not pinned (one rank, ``off``, or too few CPUs). Measured on an
    MI355X box (256 CPUs; profiles/r04n_pin_ranks.jsonl): 8 ranks pinned poll like one rank
    (p50 0.0189 ms vs 0.0189), unpinned 0.0191-0.0205 ms."""
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    if mode == "off" or (mode == "auto" and local_world <= 1):
        return None
    cpus = sorted(os.sched_getaffinity(0))
    # a rank busy-polls on one CPU while its fakes' threads answer on others: with fewer than 4
    # CPUs each (a small container) confining ranks costs more than it saves, so auto leaves them
    if len(cpus) < local_world or (mode == "auto" and len(cpus) < 4 * local_world):
        return None
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    per = len(cpus) // local_world
    mine = cpus[local_rank * per:(local_rank + 1) * per]
    os.sched_setaffinity(0, mine)
    return mine


def _pool(samples_ns, wall_s: float, device, collective: bool):
    """The job-wide view after the timed region: every rank's latency samples (sorted) and the
    slowest rank's wall time. Over the process group when ``collective`` (tensors on ``device``:
    this rank's GPU under RCCL, the CPU under gloo); ranks may hold different sample counts (a
    poll whose write failed records none), and all_gather needs equal shapes, so each pads to
    the largest count with -1 and the padding is dropped."""
    import torch
    import torch.distributed as dist

    samples = torch.tensor(sorted(samples_ns), dtype=torch.int64, device=device)
    wall_t = torch.tensor([wall_s], dtype=torch.float64, device=device)
    if collective:
        world = dist.get_world_size()
        count = torch.tensor([samples.numel()], dtype=torch.int64, device=device)
        counts = [torch.empty_like(count) for _ in range(world)]
        dist.all_gather(counts, count)
        longest = max(int(c.item()) for c in counts)
        if longest:  # (every rank empty: nothing to gather)
            padded = torch.full((longest,), -1, dtype=torch.int64, device=device)
            padded[: samples.numel()] = samples
            gathered = [torch.empty_like(padded) for _ in range(world)]
            dist.all_gather(gathered, padded)
            samples = torch.cat(gathered)
            samples = samples[samples >= 0]
        dist.all_reduce(wall_t, op=dist.ReduceOp.MAX)
    return sorted(samples.cpu().tolist()), float(wall_t.item())


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch_ranks(n: int, argv: list, script: str = __file__) -> int:
    """Runs this script as ranks 0..n-1 of one job, one child process per rank (one GPU each).
    Called before anything in this process imports torch or touches a GPU, and it never execs:
    the parent only waits. Rank 0 inherits stdout, so its JSON line is the job's; the other
    ranks' stdout goes to stderr. When a rank fails the others are stopped (they would block in
    the next collective) and the first failure's exit status is returned; a SIGTERM / SIGINT to
    the launcher stops every rank before it exits."""
    import signal
    import subprocess

    port = _free_port()

    def stop(signum, frame):  # the launcher's own SIGTERM / SIGINT: the finally below stops the ranks
        raise SystemExit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, stop)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(script), *argv], env=env,
                                      stdout=None if r == 0 else sys.stderr.fileno()))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    _progress(f"rank {procs.index(p)} exited with status {code}; stopping the other ranks")
                    for q in live:
                        q.send_signal(signal.SIGTERM)
            if live:
                time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--queues", type=int, default=1, help="tracked queues per rank")
    ap.add_argument("--mode", default="scale", choices=["scale", "deployment", "patch"])
    ap.add_argument("--no-sweep", action="store_true",
                    help="skip every secondary row: the 1/2/4/8-queue sweep, the production-cadence rows, ...")
    ap.add_argument("--no-pipeline", action="store_true", help="strictly sequential SQS -> GET -> write")
    ap.add_argument("--busy-poll-us", type=int, default=25, help="adaptive client busy-poll window (CLI default --busy-poll=25us; 0: block)")
    ap.add_argument("--servers", default="auto", choices=["auto", "shared", "per-queue", "processes"],
                    help="fake SQS/apiserver: one in-process pair for all of this rank's queues (shared), one "
                         "in-process pair per queue, or one endpoint process per queue (processes, so the "
                         "fakes' threads do not share the autoscaler's process); auto: shared for one queue, "
                         "processes for more")
    ap.add_argument("--secondary-samples", type=int, default=2000,
                    help="samples per queue for every secondary row (independent of --steps)")
    ap.add_argument("--cadence-queues", type=int, default=16,
                    help="queues (one thread each, staggered) per production-cadence row")
    ap.add_argument("--cadence-polls", type=int, default=27,
                    help="polls per queue per production-cadence fleet row (the first 2 of each queue are dropped)")
    ap.add_argument("--cadence-queue-samples", type=int, default=120,
                    help="scaling polls per cell of the 250 ms 1/2/4/8-tracked-queue rows (over all its rounds)")
    ap.add_argument("--cadence-queue-rounds", type=int, default=3,
                    help="interleaved rounds of the 1/2/4/8-queue rows; each cell pools its rounds' samples")
    ap.add_argument("--no-cadence", action="store_true", help="skip the production-cadence rows")
    ap.add_argument("--cadence-cpus", default="auto",
                    help="CPUs the production-cadence rows run on: auto (the first ceil(cgroup CPU quota) CPUs, at "
                         "least 4, when the quota is below the CPUs allowed), off, or a count")
    ap.add_argument("--pin-ranks", default="auto", choices=["auto", "on", "off"],
                    help="confine each rank of a multi-rank job to its own slice of this process's CPUs, as N "
                         "autoscaler pods with CPU limits are (auto: on when the job has more than one rank)")
    ap.add_argument("--rehearse-shared-gpus", action="store_true",
                    help="allow more ranks than visible GPUs (ranks share GPUs, samples pool over gloo): a rehearsal of an "
                         "N-GPU run on a smaller box, reported with n_gpus = the GPUs actually used")
    ap.add_argument("--extras-budget-s", type=float, default=400.0,
                    help="seconds after start past which the remaining secondary sections and cadence rows are skipped "
                         "(recorded under extra.skipped_sections); the headline line is always printed")
    ap.add_argument("--detail-out", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="file for the full result (every row and breakdown); the stdout line carries the headline "
                         "and summary rows only, at most 4096 bytes, and names this file ('' : none)")
    args = ap.parse_args(argv)
    if args.gpus < 1 or args.queues < 1:
        ap.error("--gpus and --queues must be at least 1")
    if "WORLD_SIZE" in os.environ:  # under torchrun (or a rank of _launch_ranks)
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={os.environ['WORLD_SIZE']} "
                  "ranks", file=sys.stderr)
            return 2
    elif args.gpus > 1:
        return _launch_ranks(args.gpus, argv)
    t_start = time.monotonic()
    pinned = _pin_rank(args.pin_ranks)
    # stdout carries the one result line: what libraries print on fd 1 (gloo's "[Gloo] Rank 0 is
    # connected ..." during rendezvous, RCCL/HIP notices) goes to stderr instead
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    gpus_visible = torch.cuda.device_count() if use_cuda else 0
    # One rank per GPU over RCCL. More ranks than GPUs is only a rehearsal of an N-GPU run on a
    # smaller box (--rehearse-shared-gpus): ranks share devices, which RCCL cannot, so such a job
    # pools its samples over gloo and reports the GPUs it actually used, not N.
    shared_gpus = world > 1 and gpus_visible < local_world
    if shared_gpus and not args.rehearse_shared_gpus:
        print(f"bench.py: {local_world} ranks on this node but {gpus_visible} GPU(s) visible; one rank per GPU is "
              "required (--rehearse-shared-gpus runs them anyway, reporting the GPUs actually used)", file=sys.stderr)
        return 2
    n_gpus = min(gpus_visible, local_world) * (world // max(local_world, 1)) if shared_gpus else world
    backend = "nccl" if use_cuda and not shared_gpus else "gloo"
    if use_cuda:
        torch.cuda.set_device(local_rank % max(torch.cuda.device_count(), 1))
    if world > 1 and backend == "gloo" and use_cuda and rank == 0:
        _progress(f"{local_world} ranks on {torch.cuda.device_count()} GPU(s): ranks share GPUs, samples pool over gloo")
    device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    if world > 1:
        if backend == "nccl":  # RCCL; eager init bound to this rank's GPU
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")

    def barrier_sync():
        if world > 1:
            dist.barrier()
        if use_cuda:
            torch.cuda.synchronize()

    from kube_sqs_autoscaler_amd.bench.latency import BenchEnv, measure
    from kube_sqs_autoscaler_amd.ops import native

    native()  # build/load before timing
    pipeline = not args.no_pipeline
    bp = args.busy_poll_us * 1000
    servers = args.servers if args.servers != "auto" else ("shared" if args.queues == 1 else "processes")
    env = BenchEnv(args.queues, args.mode, pipeline=pipeline, busy_poll_ns=bp, servers=servers)
    try:
        if args.warmup:
            env.run(args.warmup)
        env.clear()
        barrier_sync()
        t0 = time.perf_counter()
        env.run(args.steps)
        barrier_sync()
        wall = time.perf_counter() - t0
        res = env.collect(args.steps, wall)
        if rank == 0:
            _progress(f"timed run: {args.steps} steps in {wall:.3f} s")
    finally:
        env.close()

    all_ns, wall_max = _pool(res.samples, wall, device, collective=world > 1)

    def pct(v, p):
        import math

        k = max(1, math.ceil(p / 100.0 * len(v)))
        return v[min(k, len(v)) - 1] / 1e6

    out = None
    if rank == 0:
        p50 = pct(all_ns, 50)
        extra = {
            "p90_ms": round(pct(all_ns, 90), 4),
            "p99_ms": round(pct(all_ns, 99), 4),
            "samples": len(all_ns),
            "tracked_queues": args.queues * world,
            "scale_mode": args.mode,
            "pipeline_reads": pipeline,
            "busy_poll_us": args.busy_poll_us,
            "fake_endpoints": servers,
            "collective_backend": backend if world > 1 else None,
            "gpus_visible": gpus_visible,
            "ranks": world,
            "rehearsal_shared_gpus": shared_gpus,
            "rank0_cpus": f"{pinned[0]}-{pinned[-1]}" if pinned else None,
            "iterations_per_s": round(args.queues * world * args.steps / wall_max, 1),
            "signature_failures": res.signature_failures,
            "connections": {"sqs": res.sqs_connections, "kube": res.kube_connections},
        }
        def guarded(name, fn, budgeted=True):
            """One secondary section: its failure or the time budget costs that section only --
            the headline line is printed whatever happens here."""
            if budgeted and time.monotonic() - t_start > args.extras_budget_s:
                extra.setdefault("skipped_sections", []).append(name)
                _progress(f"{name}: skipped (past --extras-budget-s)")
                return
            try:
                fn()
            except Exception as e:  # noqa: BLE001 -- recorded, never fatal to the headline
                extra.setdefault("section_errors", {})[name] = f"{type(e).__name__}: {e}"
                _progress(f"{name} failed: {type(e).__name__}: {e}")

        def secondary():
            # Secondary rows: three interleaved rounds, median p50 per row, so one disturbed run
            # (CPU migration, a noisy neighbour) cannot invert the comparison.
            n, w = args.secondary_samples, 200
            # row: (queues, mode, pipelined, busy-poll ns, tls, servers, workers)
            rows = {}
            for q in (1, 2, 4, 8):
                # --worker-processes: one worker process per queue, one endpoint process per queue
                rows[f"q{q}"] = (q, args.mode, pipeline, bp, False, "processes", "processes")
                # the default thread-per-queue fleet against the same endpoint processes
                rows[f"q{q}_threads"] = (q, args.mode, pipeline, bp, False, "processes", "threads")
            # round 1's row: 8 threads against one shared in-process fake pair
            rows["q8_threads_shared_fakes"] = (8, args.mode, pipeline, bp, False, "shared", "threads")
            rows["sequential"] = (1, args.mode, False, 0, False, "shared", "threads")
            rows["reference"] = (1, "deployment", False, 0, False, "shared", "threads")
            # Production endpoints are HTTPS: the same two paths over keep-alive TLS 1.3
            rows["tls"] = (1, args.mode, pipeline, bp, True, "shared", "threads")
            rows["reference_tls"] = (1, "deployment", False, 0, True, "shared", "threads")
            # --sqs-protocol=json (AWS JSON 1.0, what current SDKs speak to SQS) instead of the
            # reference's Query/XML
            rows["sqs_json"] = (1, args.mode, pipeline, bp, False, "shared", "threads", {"sqs_protocol": "json"})
            p50s = {k: [] for k in rows}
            samples = {k: [] for k in rows}
            for _ in range(3):
                for k, (q, mode, pl, b, tls, sv, wk, *kw) in rows.items():
                    extra_kw = kw[0] if kw else {}
                    sm = measure(q, n, w, mode, pipeline=pl, busy_poll_ns=b, tls=tls, servers=sv, workers=wk,
                                 **extra_kw).summary()
                    p50s[k].append(sm["p50_ms"])
                    samples[k].append(sm["samples"])
                _progress(f"secondary rows, round {len(p50s['sequential'])}/3 done")
            med = {k: sorted(v)[1] for k, v in p50s.items()}
            # the CLI's default fleet (a thread per queue) is the primary row
            extra["p50_ms_by_tracked_queues"] = {str(q): med[f"q{q}_threads"] for q in (1, 2, 4, 8)}
            extra["tracked_queues_config"] = ("default fleet: one worker thread per queue in one process, each queue "
                                              "against its own fake SQS + apiserver process")
            extra["p50_ms_by_tracked_queues_worker_processes"] = {str(q): med[f"q{q}"] for q in (1, 2, 4, 8)}
            extra["p50_ms_8_queues_threads_shared_fakes"] = med["q8_threads_shared_fakes"]
            extra["sequential_scale_p50_ms"] = med["sequential"]
            extra["reference_equivalent_p50_ms"] = med["reference"]
            extra["tls_p50_ms"] = {"default": med["tls"], "reference_equivalent": med["reference_tls"]}
            extra["sqs_json_protocol_p50_ms"] = med["sqs_json"]
            extra["secondary_rows_p50_ms_all_rounds"] = p50s
            extra["secondary_rows_samples_per_round"] = samples
            # Regional-RTT model: the fakes add 2 ms (SQS) / 1 ms (apiserver) per request, so the
            # structural round-trip savings show at production scale (200 polls each).
            wan = {}
            for name, mode, pl in (("optimised", args.mode, pipeline), ("reference_equivalent", "deployment", False)):
                r = measure(1, n, 5, mode, pipeline=pl, sqs_latency_ns=2_000_000, kube_latency_ns=1_000_000)
                wan[name] = r.summary()["p50_ms"]
            extra["wan_model_sqs2ms_kube1ms_p50_ms"] = wan
            _progress(f"regional-RTT model rows: {wan}")
            extra["wan_model_samples"] = n
            from kube_sqs_autoscaler_amd.bench.latency import phase_breakdown

            extra["phase_median_us"] = {
                "default": phase_breakdown(mode=args.mode, pipeline=pipeline, busy_poll_ns=bp),
                "reference_equivalent": phase_breakdown(mode="deployment", pipeline=False),
                # the same hot loop with every call timed (HttpTiming), next to the cadence rows' breakdown
                "default_timed": phase_breakdown(mode=args.mode, pipeline=pipeline, busy_poll_ns=bp, timing=True),
            }

        def parity():
            extra["decision_parity"] = _parity_summary()
            extra["apiserver_requests_per_poll"] = _apiserver_requests_per_poll(extra["decision_parity"])

        if world == 1 and not args.no_sweep:
            guarded("secondary_rows", secondary)
        if world == 1 and not args.no_sweep and not args.no_cadence:
            def cadence():
                cpus = _cadence_cpus(args.cadence_cpus)
                before = os.sched_getaffinity(0)
                if cpus:
                    os.sched_setaffinity(0, cpus)
                    extra["cadenced_rows_cpus"] = f"{cpus[0]}-{cpus[-1]}" if cpus == list(range(cpus[0], cpus[-1] + 1)) \
                        else cpus
                try:
                    extra.update(_cadence_rows(args, pipeline, bp, p50, deadline=t_start + args.extras_budget_s))
                finally:
                    os.sched_setaffinity(0, before)

            guarded("cadence_rows", cadence)
        guarded("decision_parity", parity, budgeted=False)  # seconds; part of the metric's name
        out = {
            "metric": METRIC,
            "value": round(p50, 4),
            "unit": "ms",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max * 1000.0 / args.steps, 5),
            "higher_is_better": False,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",  # control-plane service: no tensor compute (BASELINE.json north_star)
            "data": "synthetic: every poll alternates 200 / 0 messages, served by localhost fake SQS + fake kube-apiserver (SigV4 + bearer auth verified)",
            "config": {
                "model": "kube-sqs-autoscaler control loop, scaling path: depth alternates 200/0 on every poll with "
                         "poll-period=0 and both cool-downs 0, scale-up-messages=100 / scale-down-messages=10, "
                         "min 1 / max 8, so every poll does SQS GetQueueAttributes + Deployment GET + /scale write "
                         f"({args.mode} mode{', pipelined read' if pipeline else ''})",
                "global_batch": args.queues * world,
                "seq_len": 1,
                "parallelism": f"dp{world}",
            },
            "extra": extra,
        }
        detail = write_detail(out, args.detail_out) if args.detail_out else None
        os.write(result_fd, (result_line(out, detail) + "\n").encode())
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
