"""The evidence scripts under scripts/ stay runnable: each one on tiny settings (CPU here; the
GPU sweep benches fall back to the CPU path when no GPU is visible)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240, env=None, soak=False):
    """The script's JSON lines. ``soak``: a short soak's exit status also reflects whether fds /
    threads / RSS stayed flat over its two steady windows, which an 18 s run with a fault every
    2 s can miss by a reconnect in flight at a sample; the caller checks the summary's decisions
    itself (flatness is what the 10-minute box soaks show, profiles/r05p/ and later)."""
    r = subprocess.run([sys.executable, *args], cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, **(env or {})))
    rows = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    if soak and r.returncode == 1 and rows and rows[-1].get("summary"):
        return rows
    assert r.returncode == 0, (r.stderr[-2000:], r.stdout.strip().splitlines()[-1:])
    return rows


def test_cadence_5s_script(nat):
    rows = _run(["scripts/cadence_5s.py", "--period-ms", "60", "--queues", "2", "--polls", "4"])
    assert [r["row"] for r in rows] == ["default", "reference_equivalent", "default_tls", "reference_equivalent_tls"]
    assert all(r["samples"] >= 2 and r["errors"] == 0 and r["signature_failures"] == 0 for r in rows)


def test_cadence_arms_script(nat):
    rows = _run(["scripts/cadence_arms.py", "--period-ms", "60", "--polls", "4", "--queues", "4", "--untimed"])
    assert len(rows) == 8  # 4 arms x (fakes that sleep, fakes that never sleep)
    assert {r["spin_budget"] for r in rows} == {"1%/queues", 0}


@pytest.mark.slow
def test_soak_script_short(nat):
    rows = _run(["scripts/soak.py", "--minutes", "0.3", "--window", "6", "--queues", "2", "--fault-every", "2",
                 "--presend"], timeout=200, soak=True)
    summary = rows[-1]
    assert summary["summary"] and summary["replay"]["mismatches"] == 0 and summary["exit_code"] == 0, summary
    # the per-client transport counters of /metrics reach the window rows: with --poll-presend the
    # warm-up stages the polls' SQS requests (1 s period)
    windows = [r for r in rows if "window" in r and "scrape_error" not in r]
    assert windows and windows[-1]["http_connects_sqs"] >= 2 and windows[-1]["http_presends_sqs"] > 0
    assert 0 < windows[-1]["poll_cpu_ms_per_poll"] < 50  # ksa_poll_cpu_seconds_total over the polls


@pytest.mark.slow
def test_soak_script_worker_processes_rotating_credentials(nat):
    """--worker-processes with a container-credentials endpoint whose sets the broker refreshes
    5 s after issue (at most every 10 s, credbroker.MIN_REFRESH_NS): the supervisor's broker
    fetches for the whole fleet (one fetch per refresh, not one per worker), decisions and
    signatures are unaffected, the resources are the process tree's. (The workers move to a newer
    set once their own copy enters its 5-minute window, past this short run: the box soaks show
    it, profiles/r05p/.)"""
    rows = _run(["scripts/soak.py", "--minutes", "0.3", "--window", "6", "--queues", "3", "--fault-every", "2",
                 "--worker-processes", "--ecs-refresh", "5"], timeout=200, soak=True)
    summary = rows[-1]
    assert summary["exit_code"] == 0 and summary["replay"]["mismatches"] == 0, summary
    assert summary["signature_failures"] == 0
    creds = summary["credentials"]
    assert 2 <= creds["fetches"] <= creds["at_most"], creds
    assert summary["last_metrics"]["processes"] == 4  # the supervisor and 3 workers
    # /metrics counts the broker's fetches (ksa_aws_credential_fetches_total)
    assert 1 <= summary["last_metrics"]["aws_credential_fetches"] <= creds["fetches"]


@pytest.mark.slow
def test_cpu_split_script(nat):
    rows = _run(["scripts/cpu_split.py", "--queues", "2", "--period-ms", "50", "--short-s", "2.5", "--long-s", "4"],
                timeout=200)
    assert [r["arm"] for r in rows] == ["default", "default_busy_poll_0", "reference_equivalent"]
    assert all(r["ok"] and r["polls"] > 0 and r["span_cpu_ms_per_poll"] > 0 for r in rows)


@pytest.mark.slow
def test_sweep_bench_scripts_cpu(nat):
    env = {"HIP_VISIBLE_DEVICES": "", "KSA_BENCH_SEGMENT_S": "300"}
    rows = _run(["scripts/sweep_bench.py"], env=env)
    assert any(r.get("device") == "cpu" and r["simulated_polls"] > 0 for r in rows)
    rows = _run(["scripts/queue_sweep_bench.py"], env=env)
    assert any(r.get("device") == "cpu" and r["lane_polls"] > 0 for r in rows)


@pytest.mark.slow
def test_shard_balance_script_cpu(nat):
    rows = _run(["scripts/shard_balance.py", "--device", "cpu", "--world", "2"])
    summary = {r["split"]: r for r in rows if "world" in r}
    assert summary["cost_balanced"]["max_over_min_polls"] <= 1.01
    assert summary["contiguous"]["max_over_min_polls"] > 2
