"""--worker-processes: one worker process per tracked queue (parallel/procfleet.py)."""
import os
import signal
import subprocess
import sys
import time

import pytest
import yaml

from kube_sqs_autoscaler_amd.parallel.procfleet import ProcessFleet

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AKID, SECRET, REGION, TOKEN = "AKIDPF", "pf/secret", "us-east-1", "pf-token"


@pytest.fixture
def servers(nat, tmp_path):
    sqs = nat.FakeSqsServer()
    sqs.require_signature(AKID, SECRET, REGION)
    sqs.start()
    kube = nat.FakeKubeServer()
    kube.require_token(TOKEN)
    kube.start()
    kc = tmp_path / "kubeconfig"
    kc.write_text(yaml.safe_dump({
        "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
        "users": [{"name": "u", "user": {"token": TOKEN}}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
    env = {"AWS_ACCESS_KEY_ID": AKID, "AWS_SECRET_ACCESS_KEY": SECRET, "KUBE_CONFIG_PATH": str(kc)}
    yield sqs, kube, env
    sqs.stop()
    kube.stop()


def _specs(sqs, kube, depths):
    specs = []
    for i, depth in enumerate(depths):
        url = f"{sqs.url}/123/q{i}"
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": depth})
        kube.add_deployment("gpu", f"w{i}", 4)
        specs += ["--queue", f"url={url},deployment=w{i},namespace=gpu,attribute-names=ApproximateNumberOfMessages"]
    return specs


def test_cli_worker_processes_scale_each_queue(servers, capfd):
    from kube_sqs_autoscaler_amd.cli import main

    sqs, kube, env = servers
    specs = _specs(sqs, kube, ["500", "0", "50"])
    rc = main([f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-up-cool-down=0s",
               "--scale-down-cool-down=0s", "--max-pods=6", "--worker-processes", *specs], environ=env, max_iterations=5)
    assert rc == 0
    assert [kube.replicas("gpu", f"w{i}") for i in range(3)] == [6, 1, 4]
    err = capfd.readouterr().err
    assert 'msg="Scale up successful. Replicas: 6" deployment=gpu/w0' in err
    assert sqs.signature_failures() == 0


def test_fleet_mirrors_stats_latencies_and_max_override(nat, servers):
    """The supervisor sees each worker's counters and latencies through its shared slot, and a
    max-pods override written there (the GPU-capacity cap) is applied by the worker."""
    from kube_sqs_autoscaler_amd import autoscaler
    from kube_sqs_autoscaler_amd.config import parse_args
    from kube_sqs_autoscaler_amd.utils.log import make_logger

    sqs, kube, env = servers
    specs = _specs(sqs, kube, ["500", "500"])
    cfg = parse_args([f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=1ms",
                      "--scale-up-cool-down=0s", "--max-pods=20", "--kube-api-qps=0", *specs], env)
    rest = autoscaler.load_rest_config(cfg, env)
    log = make_logger("error", "text")
    clock = nat.RealClock()
    builds = [lambda t=t: autoscaler.new_runner(t, cfg, rest, log, clock, environ=env) for t in cfg.targets]
    fleet = ProcessFleet(builds, cfg.targets)
    try:
        fleet.workers[1].runner.scaler.max = 5  # the cap, before the first poll
        fleet.start(8)
        assert fleet.wait(30)
        assert fleet.exit_codes() == [0, 0]
        st = fleet.stats()
        assert [s["polls"] for s in st] == [8, 8] and [s["scale_ups"] for s in st] == [8, 1]
        assert kube.replicas("gpu", "w0") == 12 and kube.replicas("gpu", "w1") == 5
        assert len(fleet.workers[0].runner.latencies()) == 8 and st[0]["latency_samples"] == 8
        assert all(s["poll_cpu_ns"] > 0 for s in st)  # each worker process's poll CPU, through its slot
        assert all(v > 0 for v in fleet.workers[0].runner.latencies())
        assert st[0]["latency_sum_ns"] == sum(fleet.workers[0].runner.latencies())
    finally:
        fleet.close()


def test_sigterm_stops_worker_processes(servers, tmp_path):
    sqs, kube, env = servers
    specs = _specs(sqs, kube, ["0", "0"])
    e = dict(os.environ)
    e.update(env)
    p = subprocess.Popen([sys.executable, "-m", "kube_sqs_autoscaler_amd", f"--aws-region={REGION}",
                          f"--sqs-endpoint={sqs.url}", "--poll-period=20ms", "--worker-processes", *specs],
                         cwd=ROOT, env=e, stderr=subprocess.PIPE, text=True)
    try:
        deadline = time.time() + 60
        while time.time() < deadline and sqs.requests() < 4:
            time.sleep(0.05)
        assert sqs.requests() >= 4
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=20) == 0
        err = p.stderr.read()
        assert "Stopped kube-sqs-autoscaler" in err
    finally:
        if p.poll() is None:
            p.kill()
    n = sqs.requests()
    time.sleep(0.2)
    assert sqs.requests() == n  # no orphaned worker keeps polling


def test_flag_conflict():
    from kube_sqs_autoscaler_amd.config import parse_args
    from kube_sqs_autoscaler_amd.utils.goflag import FlagError

    with pytest.raises(FlagError):
        parse_args(["--worker-processes", "--worker-threads=2"], {})


def test_metrics_and_health_over_worker_processes(nat, servers):
    """/metrics and /healthz of a --worker-processes fleet come from the workers' shared slots."""
    import urllib.request

    from kube_sqs_autoscaler_amd import autoscaler
    from kube_sqs_autoscaler_amd.config import parse_args
    from kube_sqs_autoscaler_amd.metrics import Health, MetricsServer
    from kube_sqs_autoscaler_amd.utils.log import make_logger

    sqs, kube, env = servers
    specs = _specs(sqs, kube, ["500", "0"])
    cfg = parse_args([f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=5ms",
                      "--scale-up-cool-down=0s", "--scale-down-cool-down=0s", "--max-pods=7", *specs], env)
    rest = autoscaler.load_rest_config(cfg, env)
    log = make_logger("error", "text")
    builds = [lambda t=t: autoscaler.new_runner(t, cfg, rest, log, nat.RealClock(), environ=env) for t in cfg.targets]
    fleet = ProcessFleet(builds, cfg.targets)
    health = Health(fleet, [Health.budget_ns(t.poll_period_ns, cfg.api_timeout_ns) for t in cfg.targets])
    m = MetricsServer(fleet, "127.0.0.1:0", health)
    m.start()
    try:
        fleet.start()
        deadline = time.time() + 30
        while time.time() < deadline and kube.replicas("gpu", "w0") < 7:
            time.sleep(0.01)
        base = f"http://127.0.0.1:{m.port}"
        assert urllib.request.urlopen(base + "/healthz").read() == b"ok"
        while time.time() < deadline and not all(s["polls"] > 0 for s in fleet.stats()):
            time.sleep(0.01)
        assert urllib.request.urlopen(base + "/readyz").read() == b"ok"
        text = urllib.request.urlopen(base + "/metrics").read().decode()
        assert 'ksa_scale_ups_total{deployment="gpu/w0"' in text
        assert 'ksa_replicas{deployment="gpu/w0",queue="' in text and "} 7.0" in text
        assert 'ksa_poll_to_patch_seconds_count{deployment="gpu/w0"' in text
        assert 'ksa_poll_to_patch_latency_seconds_bucket{deployment="gpu/w0",le="+Inf"' in text
    finally:
        fleet.stop()
        fleet.join()
        m.stop()
        fleet.close()
    assert kube.replicas("gpu", "w0") == 7 and kube.replicas("gpu", "w1") == 1


def test_a_dead_worker_process_brings_the_fleet_down(servers):
    """A worker process killed on its own (the OOM killer, a crash) must not leave its queue
    unpolled while the others carry on: the supervisor stops the rest and exits non-zero, so the
    pod restarts -- what a crashing thread does to the single-process fleet."""
    sqs, kube, env = servers
    specs = _specs(sqs, kube, ["0", "0", "0"])
    e = dict(os.environ)
    e.update(env)
    p = subprocess.Popen([sys.executable, "-m", "kube_sqs_autoscaler_amd", f"--aws-region={REGION}",
                          f"--sqs-endpoint={sqs.url}", "--poll-period=20ms", "--worker-processes", *specs],
                         cwd=ROOT, env=e, stderr=subprocess.PIPE, text=True)
    try:
        deadline = time.time() + 60
        while time.time() < deadline and sqs.requests() < 6:
            time.sleep(0.05)
        with open(f"/proc/{p.pid}/task/{p.pid}/children") as f:
            kids = [int(x) for x in f.read().split()]
        assert len(kids) == 3
        os.kill(kids[1], signal.SIGKILL)
        assert p.wait(timeout=20) == 1
        err = p.stderr.read()
        assert "worker process(es) [1] died" in err and "-9" in err
    finally:
        if p.poll() is None:
            p.kill()
    n = sqs.requests()
    time.sleep(0.2)
    assert sqs.requests() == n  # the surviving workers were stopped too


@pytest.mark.parametrize("fleet_kind", ["threads", "processes"])
def test_readyz_reports_the_last_error_for_both_fleets(nat, servers, fleet_kind):
    """--readiness-failure-window with persistent failures: /readyz's 503 reason carries the
    worker's last poll error whether the queue runs on a thread (Runner.last_error) or in a
    worker process (the error text crosses the shared slot's seqlock), and the text is the same."""
    import urllib.error
    import urllib.request

    from kube_sqs_autoscaler_amd import autoscaler
    from kube_sqs_autoscaler_amd.config import parse_args
    from kube_sqs_autoscaler_amd.metrics import Health, MetricsServer
    from kube_sqs_autoscaler_amd.parallel.fleet import Fleet
    from kube_sqs_autoscaler_amd.utils.log import make_logger

    sqs, kube, env = servers
    specs = _specs(sqs, kube, ["500"])
    sqs.inject(1_000_000, nat.InjectedFault(403, "<ErrorResponse><Error><Type>Sender</Type><Code>AccessDenied</Code>"
                                                 "<Message>not authorized</Message></Error></ErrorResponse>", "text/xml"))
    cfg = parse_args([f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=5ms", *specs], env)
    rest = autoscaler.load_rest_config(cfg, env)
    log = make_logger("fatal", "text")
    build = lambda t: autoscaler.new_runner(t, cfg, rest, log, nat.RealClock(), environ=env)  # noqa: E731
    if fleet_kind == "processes":
        fleet = ProcessFleet([lambda t=t: build(t) for t in cfg.targets], cfg.targets)
    else:
        fleet = Fleet([build(t) for t in cfg.targets])
    health = Health(fleet, [Health.budget_ns(t.poll_period_ns, cfg.api_timeout_ns) for t in cfg.targets],
                    failure_window_ns=100_000_000)
    m = MetricsServer(fleet, "127.0.0.1:0", health)
    m.start()

    def readyz():
        try:
            r = urllib.request.urlopen(f"http://127.0.0.1:{m.port}/readyz")
            return r.status, r.read().decode()
        except urllib.error.HTTPError as e:
            return e.code, e.read().decode()

    try:
        fleet.start()
        deadline = time.time() + 20
        while "every poll failed" not in readyz()[1]:
            assert time.time() < deadline, readyz()
            time.sleep(0.02)
        code, why = readyz()
        assert code == 503
        assert "; last error: Failed to get messages in SQS: AccessDenied: not authorized" in why, why
        err = fleet.workers[0].runner.last_error()
        assert err.startswith("Failed to get messages in SQS: AccessDenied: not authorized") and err in why
    finally:
        fleet.stop()
        fleet.join()
        m.stop()
        if fleet_kind == "processes":
            fleet.close()


def test_shared_error_slot_truncates_on_a_character_boundary(nat):
    """The worker-process error slot keeps at most 511 bytes and never splits a UTF-8 character."""
    import mmap

    buf = mmap.mmap(-1, nat.shared_worker_state_size())
    import ctypes

    addr = ctypes.addressof(ctypes.c_char.from_buffer(buf))
    nat.init_shared_worker_state(addr)
    assert nat.read_shared_worker_error(addr) == ""
    nat.write_shared_worker_error(addr, "short error")
    assert nat.read_shared_worker_error(addr) == "short error"
    text = "x" * 510 + "é" + "tail"  # the 2-byte character straddles byte 511
    nat.write_shared_worker_error(addr, text)
    assert nat.read_shared_worker_error(addr) == "x" * 510
    nat.write_shared_worker_error(addr, "later")  # a shorter text replaces a longer one
    assert nat.read_shared_worker_error(addr) == "later"
    del addr


def test_stuck_worker_is_killed_after_the_stop_deadline(nat):
    """A worker that a stop cannot end (here: stuck building its clients, deaf to SIGTERM) is
    SIGKILLed KILL_AFTER_S after the stop, so the supervisor's exit never waits on it."""
    from types import SimpleNamespace

    def stuck():
        while True:
            time.sleep(0.05)

    fleet = ProcessFleet([stuck], [SimpleNamespace(name="d", queue_url="q", min_pods=1, max_pods=8)])
    fleet.KILL_AFTER_S = 0.5
    try:
        time.sleep(0.2)
        t0 = time.monotonic()
        fleet.stop()
        fleet.join()
        assert time.monotonic() - t0 < 5.0
        assert fleet.exit_codes() == [-signal.SIGKILL]
    finally:
        fleet.close()
