"""Where a poll's CPU goes: user vs kernel time of the real CLI, per poll, for both arms.

The bench's cadence rows report the worker threads' CPU per poll (``cpu_ns``, one clock read per
poll); this splits it into user and system time, which only the kernel's accounting knows (tick-
sampled, so it needs many polls). For each arm the CLI runs as a child tracking ``--queues``
bench queues (every poll scales: the fakes alternate 200 and 0 messages, cool-downs are 0) against
fake endpoints in a process of their own (``--kube-api-qps=0``: at this cadence every queue's two
apiserver calls a poll would exceed client-go's 5 per second), once for ``--short-s`` and once for ``--long-s``
seconds; the child's rusage (``os.wait4``) of the short run is subtracted from the long one, which
cancels start-up, and the difference is divided by the difference in polls (counted from the
``--trace-file`` spans, whose ``cpu_ns`` mean is reported alongside).

    python scripts/cpu_split.py --queues 8 --period-ms 100 --sqs-latency-ms 2 --kube-latency-ms 1

One JSON line per arm (the default flags, the same with ``--busy-poll=0s``, the
reference-equivalent flags): ``user_ms_per_poll``, ``sys_ms_per_poll``, ``sys_share``,
``span_cpu_ms_per_poll``.
"""
import argparse
import json
import os
import signal
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ARMS = {
    "default": [],
    "default_busy_poll_0": ["--busy-poll=0s"],  # the default path without the --busy-poll window's spin
    "reference_equivalent": ["--scale-mode=deployment", "--pipeline-reads=false", "--busy-poll=0s",
                             "--poll-prewarm=0s"],
}


def run_cli(a, arm: str, seconds: float, tmp: str) -> dict:
    import yaml

    from kube_sqs_autoscaler_amd.bench.latency import AKID, REGION, SECRET, TOKEN, deployment_name, queue_url

    srv = subprocess.Popen([sys.executable, "-m", "kube_sqs_autoscaler_amd.bench.fakeserve", "--queues", str(a.queues),
                            "--sqs-latency-ns", str(int(a.sqs_latency_ms * 1e6)),
                            "--kube-latency-ns", str(int(a.kube_latency_ms * 1e6))],
                           cwd=ROOT, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        info = json.loads(srv.stdout.readline())
        sqs, kube = info["sqs"][0]["url"], info["kube"][0]["url"]
        kc = os.path.join(tmp, "kubeconfig")
        with open(kc, "w") as f:
            yaml.safe_dump({"current-context": "b", "contexts": [{"name": "b", "context": {"cluster": "c", "user": "u"}}],
                            "clusters": [{"name": "c", "cluster": {"server": kube}}],
                            "users": [{"name": "u", "user": {"token": TOKEN}}]}, f)
        trace = os.path.join(tmp, f"spans-{arm}-{seconds:g}.jsonl")
        args = [sys.executable, "-m", "kube_sqs_autoscaler_amd", f"--aws-region={REGION}", f"--sqs-endpoint={sqs}",
                f"--poll-period={a.period_ms}ms", "--scale-up-cool-down=0s", "--scale-down-cool-down=0s",
                "--max-pods=8", f"--trace-file={trace}", "--kube-api-qps=0", *ARMS[arm]]
        args += [f"--queue=url={queue_url(sqs, q)},deployment={deployment_name(q)},namespace=bench"
                 for q in range(a.queues)]
        env = dict(os.environ, AWS_ACCESS_KEY_ID=AKID, AWS_SECRET_ACCESS_KEY=SECRET, KUBE_CONFIG_PATH=kc, HOME=tmp)
        child = subprocess.Popen(args, cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        time.sleep(seconds)
        child.send_signal(signal.SIGTERM)
        _, status, ru = os.wait4(child.pid, 0)
        child.returncode = os.waitstatus_to_exitcode(status)
        with open(trace) as f:
            spans = [json.loads(line) for line in f if line.strip()]
        return {"rc": child.returncode, "user_s": ru.ru_utime, "sys_s": ru.ru_stime, "polls": len(spans),
                "span_cpu_ns": sum(s.get("cpu_ns", 0) for s in spans),
                # a call cut short by the SIGTERM is the stop, not an error
                "errors": sum(1 for s in spans if "error" in s and "request canceled" not in s["error"])}
    finally:
        try:
            srv.stdin.write("quit\n")
            srv.stdin.flush()
        except OSError:
            pass
        srv.wait(timeout=30)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--queues", type=int, default=8)
    ap.add_argument("--period-ms", type=int, default=100)
    ap.add_argument("--short-s", type=float, default=8.0)
    ap.add_argument("--long-s", type=float, default=28.0)
    ap.add_argument("--sqs-latency-ms", type=float, default=0.0)
    ap.add_argument("--kube-latency-ms", type=float, default=0.0)
    a = ap.parse_args()
    rc = 0
    with tempfile.TemporaryDirectory(prefix="ksa-cpu-split-") as tmp:
        for arm in ARMS:
            short, long_ = run_cli(a, arm, a.short_s, tmp), run_cli(a, arm, a.long_s, tmp)
            polls = long_["polls"] - short["polls"]
            ok = short["rc"] == 0 and long_["rc"] == 0 and polls > 0 and not short["errors"] and not long_["errors"]
            rc |= 0 if ok else 1
            user = (long_["user_s"] - short["user_s"]) * 1e3 / max(polls, 1)
            sys_ = (long_["sys_s"] - short["sys_s"]) * 1e3 / max(polls, 1)
            print(json.dumps({
                "arm": arm, "queues": a.queues, "period_ms": a.period_ms,
                "endpoint_latency_ms": {"sqs": a.sqs_latency_ms, "kube": a.kube_latency_ms},
                "polls": polls, "user_ms_per_poll": round(user, 4), "sys_ms_per_poll": round(sys_, 4),
                "process_cpu_ms_per_poll": round(user + sys_, 4),
                "sys_share": round(sys_ / (user + sys_), 3) if user + sys_ > 0 else None,
                "span_cpu_ms_per_poll": round((long_["span_cpu_ns"] - short["span_cpu_ns"]) / 1e6 / max(polls, 1), 4),
                "ok": ok, "runs": {"short": short, "long": long_},
            }), flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
