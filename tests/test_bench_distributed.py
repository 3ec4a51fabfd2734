"""bench.py contract: one JSON line; multi-rank path over torch.distributed (gloo on CPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _json_line(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _check(out, n, steps, warmup, gpus=None):
    """``n`` ranks; ``gpus``: the n_gpus reported (default n; a CPU rehearsal uses none)."""
    assert out["metric"].startswith("poll") and out["unit"] == "ms" and out["higher_is_better"] is False
    assert out["n_gpus"] == (n if gpus is None else gpus) and out["steps"] == steps and out["warmup"] == warmup
    assert out["value"] > 0 and out["ms_per_step"] > 0 and out["scaling"] == "weak"
    assert out["config"]["parallelism"] == f"dp{n}" and out["vs_baseline"] is None
    assert out["extra"]["decision_parity"]["fraction"] == 1.0
    assert out["extra"]["samples"] == steps * n and out["extra"]["signature_failures"] == 0


def test_bench_single_rank():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "200", "--warmup", "20", "--no-sweep"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    _check(_json_line(r.stdout), 1, 200, 20)


@pytest.mark.slow
def test_bench_two_ranks_gloo():
    env = dict(os.environ)
    env["CUDA_VISIBLE_DEVICES"] = ""  # CPU ranks: gloo backend
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", "--steps", "150",
                        "--warmup", "10", "--rehearse-shared-gpus"], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    out = _json_line(r.stdout)
    _check(out, 2, 150, 10, gpus=0)
    assert out["extra"]["tracked_queues"] == 2


def test_bench_launches_its_own_ranks_without_a_launcher():
    """`python bench.py --gpus 3` (what the driver runs on one node, no torchrun) starts three
    ranks itself over gloo here (RCCL on GPUs), and rank 0's line covers all three."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "3", "--steps", "50", "--warmup", "5", "--no-sweep",
                        "--rehearse-shared-gpus"], cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(r.stdout.splitlines()) == 1, r.stdout  # gloo's rendezvous chatter goes to stderr
    out = _json_line(r.stdout)
    _check(out, 3, 50, 5, gpus=0)  # a rehearsal: n_gpus is the GPUs used (none here), not 3
    assert out["extra"]["tracked_queues"] == 3 and out["config"]["global_batch"] == 3
    assert out["extra"]["ranks"] == 3 and out["extra"]["rehearsal_shared_gpus"] is True
    assert out["extra"]["collective_backend"] == "gloo"  # no GPUs here (RCCL on a GPU node)


def test_bench_refuses_more_ranks_than_gpus_without_the_rehearsal_flag():
    """`--gpus 3` on a box without 3 GPUs exits 2: n_gpus must be GPUs, not ranks sharing one."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "3", "--steps", "5", "--warmup", "1", "--no-sweep"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2 and r.stdout == ""
    assert "3 ranks on this node but 0 GPU(s) visible" in r.stderr


def test_bench_refuses_a_launcher_world_that_differs_from_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--steps", "5"], cwd=ROOT, capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr and r.stdout == ""


def test_rank_launcher_stops_the_job_when_one_rank_fails(tmp_path):
    """A failing rank ends the job with its status; a rank still waiting (in a collective, here
    a sleep) is stopped rather than left to hang the launch."""
    import time

    sys.path.insert(0, ROOT)
    import bench

    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1':\n    sys.exit(3)\n"
                      "assert os.environ['WORLD_SIZE'] == '3' and os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
                      "time.sleep(120)\n")
    t0 = time.monotonic()
    assert bench._launch_ranks(3, [], script=str(script)) == 3
    assert time.monotonic() - t0 < 30


def test_bench_prints_its_line_when_secondary_sections_run_out_of_time():
    """--extras-budget-s: sections past the budget are skipped and named; the headline line and
    the decision parity (part of the metric) are still there."""
    r = subprocess.run([sys.executable, "bench.py", "--steps", "50", "--warmup", "5", "--extras-budget-s", "0"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = _json_line(r.stdout)
    _check(out, 1, 50, 5)
    assert out["extra"]["skipped_sections"] == ["secondary_rows", "cadence_rows"]
    assert "section_errors" not in out["extra"] and "cadenced_p50_ms" not in out["extra"]


def test_cadence_rows_past_their_deadline_are_skipped_and_named():
    """The cadence section checks the budget before every row (16 rows of up to ~30 s each), so a
    slow box cannot run the whole section past --extras-budget-s."""
    import argparse

    sys.path.insert(0, ROOT)
    import bench

    args = argparse.Namespace(mode="scale", cadence_polls=3, cadence_queues=1, cadence_queue_samples=4)
    out = bench._cadence_rows(args, True, 0, 0.02, deadline=0.0)
    sk = out["cadenced_rows_skipped"]
    assert len(sk) == 16 and "250ms/fleet" in sk and "1s/wan_wan_sqs2ms_kube1ms" in sk
    assert "250ms/by_queues/8" in sk and "250ms/by_queues_hot/8" in sk and "250ms/by_queues_timed/1" in sk
    assert "1s/fleet_timed" in sk
    assert out["cadenced_p50_ms"] == {} and out["cadenced_vs_hot_loop_default_plain"] == {}
    assert out["cadenced_p50_ms_by_tracked_queues"] == {} and out["wan_cadenced_p50_ms"] == {}
    assert out["cpu_ms_per_poll"] == {}


@pytest.mark.slow
def test_cadence_rows_cover_the_queue_axis_default_and_reference(monkeypatch):
    """BASELINE's 1/2/4/8 tracked queues at a 250 ms cadence, default vs reference-equivalent
    path, each row with at least --cadence-queue-samples scaling polls (small here), against
    sleeping and hot endpoints, with the 1- and 8-queue attribution; the regional-RTT row at a
    cadence with both arms' CPU per poll."""
    import argparse

    sys.path.insert(0, ROOT)
    import bench
    from kube_sqs_autoscaler_amd.bench import latency

    calls = []
    real = latency.measure_cadenced_arms

    def fast(period, polls, queues, arms, *a, **kw):  # every row at a 20 ms cadence
        calls.append((period, polls, queues, sorted(arms)))
        return real(20_000_000, polls, queues, arms, *a, **kw)

    monkeypatch.setattr(latency, "measure_cadenced_arms", fast)
    args = argparse.Namespace(mode="scale", cadence_polls=3, cadence_queues=2, cadence_queue_samples=8)
    import time

    out = bench._cadence_rows(args, True, 25_000, 0.02, deadline=time.monotonic() + 120)
    for setup in ("250ms", "250ms_hot_endpoints"):
        by_q = out["cadenced_p50_ms_by_tracked_queues"][setup]
        assert set(by_q) == {"default", "reference_equivalent"}
        for name in by_q:
            assert set(by_q[name]) == {"1", "2", "4", "8"} and all(v > 0 for v in by_q[name].values())
            assert all(n >= 8 for n in out["cadenced_by_tracked_queues_samples"][setup][name].values())
        assert set(out["cadenced_by_tracked_queues_8_over_1"][setup]) == {"default", "reference_equivalent"}
        for q, st in out["cadenced_by_tracked_queues_setup"][setup].items():
            assert st["cpus_available"] >= 1 and st["autoscaler_threads"] >= 2 * int(q)
            assert len(st["endpoint_threads"]) == 2
            assert (st["endpoint_cpu_us_per_request"] is None) if "hot" in setup else len(st["endpoint_cpu_us_per_request"]) == 2
    # both paths in one run; three interleaved rounds of 1/2/4/8 queues, pooled per cell
    assert calls[0] == (250_000_000, 5, 1, ["default", "reference_equivalent"])
    assert [c[2] for c in calls[:12]] == [1, 2, 4, 8] * 3
    rounds = out["cadenced_by_tracked_queues_rounds_p50_ms"]
    assert len(rounds["250ms/default/1"]) == 3 and len(rounds["250ms_hot_endpoints/reference_equivalent/8"]) == 3
    att = out["cadenced_by_tracked_queues_attribution"]
    assert set(att) == {"1", "8"} and "endpoint_median_us" in att["8"]["default"]
    assert "call_phase_median_us" in att["1"]["reference_equivalent"]
    assert "cadenced_rows_skipped" not in out and set(out["cadenced_p50_ms"]) == {"250ms", "1s"}
    assert set(out["cadenced_p50_ms"]["250ms"]) == {"default", "reference_equivalent", "default_tls",
                                                   "reference_equivalent_tls"}
    r = out["cadenced_rows"]["1s"]["default_timed"]
    assert r["paired_with"] == ["reference_equivalent"] and r["queues_in_run"] == 4 and "call_phase_median_us" in r
    assert set(out["wan_cadenced_p50_ms"]) == {"default", "reference_equivalent"}
    assert all(v > 2.0 for v in out["wan_cadenced_p50_ms"].values())  # a 2 ms SQS answer at least
    assert set(out["cpu_ms_per_poll"]) == {"default", "reference_equivalent"}
    assert all(v > 0 for v in out["cpu_ms_per_poll"].values())
    assert list(out)[-2:] == ["wan_cadenced_p50_ms", "cpu_ms_per_poll"]
    ratios = out["cadenced_reference_over_default"]
    assert set(ratios["250ms"]) == {"plain", "tls"}
    assert set(ratios["1s"]) == {"plain", "hot_endpoints", "wan_sqs2ms_kube1ms"}
    assert set(ratios["250ms_by_tracked_queues"]) == {"1", "2", "4", "8"}


def test_rank_launcher_stops_its_ranks_when_it_is_terminated(tmp_path):
    """A SIGTERM to `bench.py --gpus N` (a driver time limit) must not leave its ranks running."""
    import signal
    import time

    script = tmp_path / "rank.py"
    pids = tmp_path / "pids"
    pids.mkdir()
    # written under a temporary name and renamed, so the test never reads a half-written file
    script.write_text("import os, time\n"
                      f"f = os.path.join({str(pids)!r}, os.environ['RANK'])\n"
                      "open(f + '.tmp', 'w').write(str(os.getpid()))\n"
                      "os.replace(f + '.tmp', f)\n"
                      "time.sleep(120)\n")
    launcher = tmp_path / "launch.py"
    launcher.write_text(f"import sys; sys.path.insert(0, {ROOT!r}); import bench\n"
                        f"sys.exit(bench._launch_ranks(2, [], script={str(script)!r}))\n")
    p = subprocess.Popen([sys.executable, str(launcher)])
    deadline = time.monotonic() + 30
    while len(list(pids.glob("[0-9]"))) < 2 and time.monotonic() < deadline:
        time.sleep(0.05)
    ranks = [int(f.read_text()) for f in pids.glob("[0-9]")]
    assert len(ranks) == 2
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) == 128 + signal.SIGTERM
    for pid in ranks:
        deadline = time.monotonic() + 10
        while time.monotonic() < deadline:
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                break
            time.sleep(0.05)
        else:
            raise AssertionError(f"rank pid {pid} still running")


def test_rank_pinning_slices_the_cpus(monkeypatch):
    """--pin-ranks: rank r of a node's N ranks gets slice r of N contiguous slices of the CPUs it
    may use; auto leaves ranks unpinned with fewer than 4 CPUs each, and one rank always."""
    sys.path.insert(0, ROOT)
    import bench

    got = {}
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(64)))
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: got.setdefault("cpus", list(cpus)))
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert bench._pin_rank("auto") == list(range(24, 32)) == got["cpus"]
    assert bench._pin_rank("off") is None
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(16)))
    assert bench._pin_rank("auto") is None  # 2 CPUs per rank: left unpinned
    assert bench._pin_rank("on") == [6, 7]
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    assert bench._pin_rank("auto") is None
