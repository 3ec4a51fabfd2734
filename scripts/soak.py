"""Soak: the CLI at a production cadence against failing endpoints, then a replay of its spans.

Starts TLS fake SQS and kube-apiserver endpoints in this process and runs the real CLI
(``python -m kube_sqs_autoscaler_amd``) as a child tracking ``--queues`` queues at
``--poll-period`` with short cool-downs, so it scales up and down all the time (each queue's
depth is a square wave of its own period). While it runs, a fault schedule hits it:

* apiserver 503 with ``Retry-After: 1`` (client-go retries after the wait), plain 500s,
  409 conflicts (a concurrent write after the GET) and dropped connections;
* SQS throttles (503 ``RequestThrottled`` with ``Retry-After: 1``; the SDK retryer backs off)
  and dropped connections;
* a bearer-token rotation half-way: the token file is rewritten and the apiserver accepts only
  the new token, so the next apiserver call gets a 401 and the client re-reads the file.

Every ``--window`` seconds it prints one JSON line: the child's open fds, threads and RSS, the
poll and failure counters from its ``/metrics``, and the faults injected so far. At the end the
child is stopped with SIGTERM and every queue's ``--trace-file`` spans are replayed through
models/replay.py: each cool-down gate, no-op and clamp the loop decided must be the reference's
(/root/reference/main.go:40-78, scale/scale.go:54-107) given the inputs the spans recorded. The
summary line has the mismatch count (must be 0) and whether fds / threads / RSS stayed flat.

    python scripts/soak.py --minutes 10 --queues 8 --poll-period 1s > gpurun_out/soak.jsonl

``--worker-processes``: the CLI runs one worker process per queue (resources are then summed over
the supervisor and its workers). ``--ecs-refresh SECONDS``: the AWS credentials come from a
container-credentials endpoint (AWS_CONTAINER_CREDENTIALS_FULL_URI) whose every set lives just
long enough for the CLI's credential broker (parallel/credbroker.py) to refresh it SECONDS
after the last fetch (at most every 10 s); the queues switch to the newest when their own copy
enters its 5-minute window. The summary counts the
endpoint's fetches, which must stay at one per refresh for the whole fleet, not one per queue,
and names the session token of the last poll. ``--ecs-outage START:SECONDS``
makes the endpoint answer 500 for a while (an agent restart): the sets already fetched keep
signing -- past the queues' 5-minute window when the outage outlasts the broker's refresh lead,
until a minute before the set expires (``ksa_aws_credential_stale_signs_total``) -- so no poll may
fail for it: with an outage, the summary is ok only when no poll failed to read the depth.

``--hot``: the old back-to-back soak of one queue (no faults), p50/p99 per window.
"""
import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

AKID, SECRET, REGION = "AKIDSOAK", "soak/secret", "us-east-1"
S = 1_000_000_000
THROTTLE = ('<?xml version="1.0"?><ErrorResponse><Error><Type>Sender</Type><Code>RequestThrottled</Code>'
            '<Message>Rate exceeded</Message></Error><RequestId>soak</RequestId></ErrorResponse>')
HIGH = {"ApproximateNumberOfMessages": "400", "ApproximateNumberOfMessagesDelayed": "50",
        "ApproximateNumberOfMessagesNotVisible": "50"}
LOW = {"ApproximateNumberOfMessages": "0", "ApproximateNumberOfMessagesDelayed": "0",
       "ApproximateNumberOfMessagesNotVisible": "0"}


def proc_stats(pid: int, tree: bool = False) -> dict:
    """fds, threads and RSS of ``pid`` -- summed over it and its descendants with ``tree``, which
    adds their PSS (proportional set size: shared pages split between the processes)."""
    pids = [pid]
    if tree:
        import psutil

        pids += [c.pid for c in psutil.Process(pid).children(recursive=True)]
    out = {"fds": 0, "rss_kb": 0, "threads": 0}
    if tree:
        out["pss_kb"] = 0  # summed RSS counts the pages the workers share with the supervisor once each
    for p in pids:
        try:
            out["fds"] += len(os.listdir(f"/proc/{p}/fd"))
            if tree:
                with open(f"/proc/{p}/smaps_rollup") as f:
                    out["pss_kb"] += sum(int(line.split()[1]) for line in f if line.startswith("Pss:"))
            with open(f"/proc/{p}/status") as f:
                for line in f:
                    if line.startswith("VmRSS:"):
                        out["rss_kb"] += int(line.split()[1])
                    elif line.startswith("Threads:"):
                        out["threads"] += int(line.split()[1])
        except OSError:  # a worker that just exited
            continue
    if tree:
        out["processes"] = len(pids)
    return out


class EcsEndpoint:
    """A container-credentials endpoint: every set is new (its own session token) and lives long
    enough past the queues' 5-minute window for the broker (parallel/credbroker.py
    ``refresh_due_at``) to refresh it ``refresh_s`` after issue: twice ``refresh_s`` past the
    window (the lead is half of that), or a minute more than ``refresh_s`` when that half would be
    under the broker's one-minute minimum lead."""

    def __init__(self, refresh_s: float, outage=None):
        """``outage``: (start, end) in time.monotonic() seconds during which every fetch fails
        with a 500 (an ECS agent / Pod Identity agent restart)."""
        from datetime import datetime, timedelta, timezone
        from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

        ep = self
        # a set the broker refreshes refresh_s after issue (credbroker.refresh_due_at: half the
        # time before the queues' window, but at least a minute early)
        life_past_window = 2 * refresh_s if refresh_s >= 60 else refresh_s + 60
        self.fetches = 0
        self.failed = 0
        self.outage = outage
        self.lock = threading.Lock()

        class Handler(BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802
                if ep.outage and ep.outage[0] <= time.monotonic() < ep.outage[1]:
                    with ep.lock:
                        ep.failed += 1
                    body = b'{"code":"InternalError","message":"agent restarting"}'
                    self.send_response(500)
                    self.send_header("Content-Length", str(len(body)))
                    self.end_headers()
                    self.wfile.write(body)
                    return
                with ep.lock:
                    ep.fetches += 1
                    n = ep.fetches
                expires = datetime.now(timezone.utc) + timedelta(minutes=5, seconds=life_past_window)
                body = json.dumps({"AccessKeyId": AKID, "SecretAccessKey": SECRET, "Token": f"soak-session-{n}",
                                   "Expiration": expires.strftime("%Y-%m-%dT%H:%M:%S.%fZ")}).encode()
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):
                pass

        self.server = ThreadingHTTPServer(("127.0.0.1", 0), Handler)
        self.url = f"http://127.0.0.1:{self.server.server_address[1]}/creds"
        threading.Thread(target=self.server.serve_forever, daemon=True).start()

    def close(self) -> None:
        self.server.shutdown()
        self.server.server_close()


def scrape(port: int) -> dict:
    text = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
    tot = {}
    for line in text.splitlines():
        if line.startswith("#") or "{" not in line:
            continue
        name = line.split("{", 1)[0]
        if name.endswith("_total"):
            key = name[4:-6]
            if 'client="' in line:  # transport counters: one per client (sqs / apiserver)
                key += "_" + line.split('client="', 1)[1].split('"', 1)[0]
            tot[key] = tot.get(key, 0) + float(line.rsplit(" ", 1)[1])
    out = {k: int(v) for k, v in tot.items() if k in (
        "polls", "scale_ups", "scale_downs", "depth_errors", "failed_ups", "failed_downs", "sqs_retries",
        "sqs_throttle_retries", "apiserver_retries", "apiserver_conflicts", "apiserver_errors",
        "aws_credential_fetches", "aws_credential_stale_signs") or (
        k.startswith("http_") and k.split("_")[1] in ("connects", "presends", "presend", "reconnect", "idle"))}
    if "poll_cpu_seconds" in tot and out.get("polls"):  # the workers' CPU per poll so far (ksa_poll_cpu_seconds_total)
        out["poll_cpu_ms_per_poll"] = round(tot["poll_cpu_seconds"] * 1000 / out["polls"], 4)
    return out


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def cadenced(a) -> int:
    import yaml

    from kube_sqs_autoscaler_amd.models.oracle import Params
    from kube_sqs_autoscaler_amd.models.replay import group_spans, replay_queue
    from kube_sqs_autoscaler_amd.ops import fakes, native
    from kube_sqs_autoscaler_amd.utils.goflag import parse_duration

    nat = native()
    period = parse_duration(a.poll_period)
    up_cool, down_cool = parse_duration(a.up_cool_down), parse_duration(a.down_cool_down)
    tmp = tempfile.mkdtemp(prefix="ksa-soak-")
    tokens = ["soak-token-1", "soak-token-2"]
    fk = fakes()
    sqs = fk.FakeSqsServer()
    sqs.require_signature(AKID, SECRET, REGION)
    sqs.start("127.0.0.1", 0, True)
    kube = fk.FakeKubeServer()
    kube.require_token(tokens[0])
    kube.start("127.0.0.1", 0, True)
    token_file = os.path.join(tmp, "token")
    with open(token_file, "w") as f:
        f.write(tokens[0])
    ca = os.path.join(tmp, "sqs-ca.pem")
    with open(ca, "w") as f:
        f.write(sqs.cert_pem)
    import base64

    kc = os.path.join(tmp, "kubeconfig")
    with open(kc, "w") as f:
        yaml.safe_dump({"current-context": "s", "contexts": [{"name": "s", "context": {"cluster": "c", "user": "u"}}],
                        "clusters": [{"name": "c", "cluster": {"server": kube.url, "certificate-authority-data":
                                                               base64.b64encode(kube.cert_pem.encode()).decode()}}],
                        "users": [{"name": "u", "user": {"tokenFile": token_file}}]}, f)
    urls = [f"{sqs.url}/000000000000/soak-{q}" for q in range(a.queues)]
    for q in range(a.queues):
        kube.add_deployment("soak", f"workers-{q}", 1)
    waves = [(20 + 7 * q) * S for q in range(a.queues)]  # each queue's square-wave period

    def set_depths(t_ns: int) -> None:
        for q, url in enumerate(urls):
            sqs.set_attributes(url, HIGH if (t_ns % waves[q]) < waves[q] // 2 else LOW)

    set_depths(0)
    trace = os.path.join(tmp, "spans.jsonl")
    port = free_port()
    args = [sys.executable, "-m", "kube_sqs_autoscaler_amd", f"--poll-period={a.poll_period}",
            f"--scale-up-cool-down={a.up_cool_down}", f"--scale-down-cool-down={a.down_cool_down}", "--max-pods=8",
            f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", f"--trace-file={trace}",
            f"--metrics-addr=127.0.0.1:{port}", "--log-level=warning", "--api-timeout=10s"]
    args += [f"--queue=url={u},deployment=workers-{q},namespace=soak" for q, u in enumerate(urls)]
    if a.presend:
        args.append("--poll-presend")
    if a.worker_processes:
        args.append("--worker-processes")
    env = dict(os.environ, KUBE_CONFIG_PATH=kc, AWS_CA_BUNDLE=ca, HOME=tmp)
    ecs = None
    if a.ecs_refresh > 0:
        outage = None
        if a.ecs_outage:
            start, length = (float(x) for x in a.ecs_outage.split(":"))
            outage = (time.monotonic() + start, time.monotonic() + start + length)
        ecs = EcsEndpoint(a.ecs_refresh, outage)
        for k in ("AWS_ACCESS_KEY_ID", "AWS_SECRET_ACCESS_KEY", "AWS_SESSION_TOKEN", "AWS_PROFILE"):
            env.pop(k, None)
        env.update(AWS_CONTAINER_CREDENTIALS_FULL_URI=ecs.url, AWS_EC2_METADATA_DISABLED="true")
    else:
        env.update(AWS_ACCESS_KEY_ID=AKID, AWS_SECRET_ACCESS_KEY=SECRET)
    err = open(os.path.join(tmp, "stderr.log"), "w")
    child = subprocess.Popen(args, cwd=ROOT, env=env, stderr=err, stdout=subprocess.DEVNULL)
    injected = {"kube_503_retry_after": 0, "kube_500": 0, "kube_409": 0, "kube_drop": 0, "sqs_throttle": 0,
                "sqs_drop": 0, "token_rotations": 0}
    stop = threading.Event()
    t_start = time.monotonic()

    def driver() -> None:
        step = 0
        next_fault = t_start + a.fault_every
        rotated = False
        while not stop.wait(0.05):
            now = time.monotonic()
            set_depths(int((now - t_start) * S))
            if not rotated and now - t_start >= a.minutes * 30:
                with open(token_file + ".new", "w") as f:
                    f.write(tokens[1])
                os.replace(token_file + ".new", token_file)
                kube.require_token(tokens[1])
                injected["token_rotations"] += 1
                rotated = True
            if now >= next_fault:
                next_fault = now + a.fault_every
                kind = step % 6
                step += 1
                if kind == 0:
                    kube.inject(2, fk.InjectedFault(503, '{"kind":"Status","code":503,"message":"overloaded"}',
                                                     "application/json", retry_after="1"))
                    injected["kube_503_retry_after"] += 2
                elif kind == 1:
                    kube.inject(1, fk.InjectedFault(500, '{"kind":"Status","code":500,"message":"etcd"}',
                                                     "application/json"))
                    injected["kube_500"] += 1
                elif kind == 2:
                    kube.conflict_next(2)
                    injected["kube_409"] += 2
                elif kind == 3:
                    kube.drop_connections()
                    injected["kube_drop"] += 1
                elif kind == 4:
                    sqs.inject(2, fk.InjectedFault(503, THROTTLE, "text/xml", retry_after="1"))
                    injected["sqs_throttle"] += 2
                else:
                    sqs.drop_connections()
                    injected["sqs_drop"] += 1

    th = threading.Thread(target=driver, daemon=True)
    th.start()
    rows = []
    try:
        end = t_start + a.minutes * 60
        k = 0
        while time.monotonic() < end and child.poll() is None:
            time.sleep(min(a.window, max(0.0, end - time.monotonic())))
            if child.poll() is not None:
                break
            # resources first: the scrape's own handler thread and socket may still be alive
            # right after it returns, and would count as a thread and an fd of the process
            res = proc_stats(child.pid, tree=a.worker_processes)
            try:
                m = scrape(port)
            except OSError as e:
                m = {"scrape_error": str(e)}
            row = {"window": k, "t_s": round(time.monotonic() - t_start, 1), **res, **m, "injected": dict(injected)}
            if ecs is not None:
                row["credential_fetches"] = ecs.fetches
            rows.append(row)
            print(json.dumps(row), flush=True)
            k += 1
    finally:
        stop.set()
        th.join()
        if child.poll() is None:
            child.send_signal(signal.SIGTERM)
        rc = child.wait(timeout=60)
        err.close()
        elapsed = time.monotonic() - t_start
        tokens_seen = [v for k2, v in sqs.last_headers() if k2.lower() == "x-amz-security-token"]
        sqs.stop()
        kube.stop()
        if ecs is not None:
            ecs.close()
    with open(trace) as f:
        spans = [json.loads(line) for line in f if line.strip()]
    p = Params(poll_ns=period, up_cool_ns=up_cool, down_cool_ns=down_cool, up_msgs=100, down_msgs=10, max_pods=8,
               min_pods=1)
    replays = [replay_queue(p, ss, boundary_ns=a.boundary_us * 1000, queue=q) for q, ss in group_spans(spans).items()]
    # poll->patch latency of the polls that wrote (the CLI at its cadence, over TLS, faults included)
    lat = sorted(sp["patch_latency_ns"] for sp in spans if sp.get("patch_latency_ns", -1) >= 0)

    def pct_us(q):
        return round(lat[min(len(lat) - 1, max(0, int(q / 100.0 * len(lat) + 0.5) - 1))] / 1e3, 1) if lat else None

    steady = rows[1:] if len(rows) > 2 else rows  # the first window includes start-up allocations
    flat = {}
    for key, tol in (("fds", 2), ("threads", 0), ("rss_kb", 8 * 1024)):
        vals = [r[key] for r in steady if key in r]
        flat[key] = {"min": min(vals), "max": max(vals), "flat": max(vals) - min(vals) <= tol} if vals else None
    with open(os.path.join(tmp, "stderr.log")) as f:
        stderr_all = f.read()
    stderr_tail = stderr_all[-2000:]
    summary = {
        "summary": True, "minutes": a.minutes, "queues": a.queues, "poll_period": a.poll_period,
        "cool_downs": [a.up_cool_down, a.down_cool_down], "exit_code": rc, "windows": len(rows),
        "spans": len(spans), "injected": injected, "last_metrics": {k: v for k, v in rows[-1].items() if k not in
                                                                   ("window", "injected")} if rows else {},
        "replay": {"polls": sum(r.polls for r in replays), "judged": sum(r.checked for r in replays),
                   "boundary": sum(r.boundary for r in replays), "depth_errors": sum(r.depth_errors for r in replays),
                   "failed_calls": sum(r.failed_calls for r in replays),
                   "scale_writes": sum(r.scale_writes for r in replays),
                   "mismatches": sum(len(r.mismatches) for r in replays),
                   "first_mismatches": [m for r in replays for m in r.mismatches][:5]},
        "resources": flat,
        "poll_to_patch_us": {"samples": len(lat), "p50": pct_us(50), "p90": pct_us(90), "p99": pct_us(99)},
        "signature_failures": sqs.signature_failures(), "kube_auth_failures": kube.auth_failures(),
        "worker_processes": a.worker_processes,
        "ok": rc == 0 and all(r.ok for r in replays) and all(v and v["flat"] for v in flat.values()),
    }
    if ecs is not None:
        # one fetch at start-up, then one per refresh for the whole fleet
        most = 2 + int(elapsed / a.ecs_refresh)
        summary["credentials"] = {"refresh_s": a.ecs_refresh, "fetches": ecs.fetches, "at_most": most,
                                  "last_poll_token": tokens_seen[-1] if tokens_seen else None,
                                  "outage_s": a.ecs_outage or None, "failed_fetches": ecs.failed,
                                  "stale_signs": rows[-1].get("aws_credential_stale_signs") if rows else None,
                                  "refresh_failed_warnings": stderr_all.count("keep signing with the current set")}
        summary["ok"] = summary["ok"] and ecs.fetches <= most
        if a.ecs_outage:  # the sets still sign through the outage: no poll may fail for it
            summary["ok"] = summary["ok"] and summary["replay"]["depth_errors"] == 0
    if not summary["ok"]:
        summary["stderr_tail"] = stderr_tail
    print(json.dumps(summary), flush=True)
    return 0 if summary["ok"] else 1


def hot(a) -> int:
    from kube_sqs_autoscaler_amd.bench.latency import BenchEnv

    def pct(v, q):
        return v[min(len(v) - 1, max(0, int(q / 100.0 * len(v) + 0.5) - 1))] if v else 0

    env = BenchEnv(1, "scale", pipeline=True, busy_poll_ns=25_000)
    runner = env.runners[0]
    try:
        env.run(2000)
        env.clear()
        end = time.monotonic() + a.minutes * 60
        k = 0
        while time.monotonic() < end:
            t0, polls, samples = time.monotonic(), 0, []
            while time.monotonic() - t0 < a.window:
                env.run(2000)
                samples += runner.latencies()
                env.clear()
                polls += 2000
            samples.sort()
            print(json.dumps({"window": k, "polls": polls, "p50_us": round(pct(samples, 50) / 1e3, 2),
                              "p99_us": round(pct(samples, 99) / 1e3, 2), **proc_stats(os.getpid())}), flush=True)
            k += 1
    finally:
        env.close()
    return 0


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--minutes", type=float, default=10.0)
    ap.add_argument("--window", type=float, default=30.0, help="seconds between resource samples")
    ap.add_argument("--queues", type=int, default=8)
    ap.add_argument("--poll-period", default="1s")
    ap.add_argument("--up-cool-down", default="3s")
    ap.add_argument("--down-cool-down", default="5s")
    ap.add_argument("--fault-every", type=float, default=7.0, help="seconds between injected faults")
    ap.add_argument("--boundary-us", type=int, default=250,
                    help="cool-down comparisons this close to the edge are not judged by the replay")
    ap.add_argument("--hot", action="store_true", help="back-to-back single-queue soak without faults")
    ap.add_argument("--presend", action="store_true", help="run the CLI with --poll-presend (staged SQS requests)")
    ap.add_argument("--worker-processes", action="store_true", help="run the CLI with --worker-processes")
    ap.add_argument("--ecs-refresh", type=float, default=0.0,
                    help="seconds between credential refreshes from a container-credentials endpoint (0: static keys)")
    ap.add_argument("--ecs-outage", default="",
                    help="START:SECONDS -- the credential endpoint answers 500 for SECONDS from START s into the soak")
    a = ap.parse_args()
    return hot(a) if a.hot else cadenced(a)


if __name__ == "__main__":
    sys.exit(main())
