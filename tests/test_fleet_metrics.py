"""Multi-queue fleet isolation + Prometheus/health endpoints."""
import urllib.request

import pytest

from kube_sqs_autoscaler_amd.bench.latency import BenchEnv
from kube_sqs_autoscaler_amd.metrics import MetricsServer
from kube_sqs_autoscaler_amd.parallel.fleet import Fleet


class W:
    def __init__(self, runner, target):
        self.runner, self.target = runner, target


def test_fleet_runs_queues_independently(nat):
    env = BenchEnv(4)
    try:
        fleet = Fleet([W(r, t) for r, t in zip(env.runners, env.targets)])
        fleet.start(25)
        assert fleet.wait(30)
        fleet.join()
        stats = fleet.stats()
        assert [s["polls"] for s in stats] == [25] * 4
        # 200/0 alternation: 13 ups, 12 downs each, every one a write
        assert all(s["scale_ups"] == 13 and s["scale_downs"] == 12 for s in stats)
        assert env.sqs.signature_failures() == 0
        assert env.sqs.connections() == 4 and env.kube.connections() == 4  # one per worker
    finally:
        env.close()


def test_fleet_stop_interrupts_sleep(nat):
    env = BenchEnv(2)
    try:
        for r in env.runners:
            pass
        cfg = nat.LoopConfig()
        cfg.poll_period_ns = 3600 * nat.SECOND
        fleet = Fleet([W(nat.Runner(cfg, r.sqs, r.scaler, nat.RealClock(), env.log), t)
                       for r, t in zip(env.runners, env.targets)])
        fleet.start()
        assert not fleet.wait(0.2)
        fleet.stop()
        assert fleet.wait(5)
        fleet.join()
        assert all(s["polls"] == 0 for s in fleet.stats())
    finally:
        env.close()


def test_metrics_endpoints(nat):
    env = BenchEnv(2)
    try:
        fleet = Fleet([W(r, t) for r, t in zip(env.runners, env.targets)])
        m = MetricsServer(fleet, "127.0.0.1:0")
        m.start()
        try:
            base = f"http://127.0.0.1:{m.port}"
            with pytest.raises(urllib.error.HTTPError) as e:
                urllib.request.urlopen(base + "/readyz")
            assert e.value.code == 503
            fleet.start(10)
            fleet.join()
            body = urllib.request.urlopen(base + "/metrics").read().decode()
            assert 'ksa_polls_total{deployment="bench/gpu-worker-0"' in body
            assert "ksa_scale_ups_total" in body and "ksa_poll_to_patch_seconds_count" in body
            assert 'ksa_replicas{deployment="bench/gpu-worker-1"' in body
            assert urllib.request.urlopen(base + "/readyz").read() == b"ok"
            assert urllib.request.urlopen(base + "/healthz").status == 200
        finally:
            m.stop()
    finally:
        env.close()
