"""--gpu-aware-max=cluster: cap max-pods at allocatable amd.com/gpu (MI355X specialisation)."""
import pytest
import yaml

from kube_sqs_autoscaler_amd.kube.config import RestConfig
from kube_sqs_autoscaler_amd.kube.gpus import ClusterGpuCapacity, MaxPodsCapper

TOKEN = "gpu-token"


@pytest.fixture
def kube(nat):
    k = nat.FakeKubeServer()
    k.require_token(TOKEN)
    k.start()
    k.add_node("mi355x-a", {"gpu": "mi355x", "pool": "a"}, "amd.com/gpu", 8)
    k.add_node("mi355x-b", {"gpu": "mi355x", "pool": "b"}, "amd.com/gpu", 8)
    k.add_node("mi355x-cordoned", {"gpu": "mi355x", "pool": "b"}, "amd.com/gpu", 8, True)
    k.add_node("cpu-1", {"pool": "cpu"}, "amd.com/gpu", 0)
    yield k
    k.stop()


def test_allocatable_sum_and_selector(kube):
    rc = RestConfig(host=kube.url, bearer_token=TOKEN)
    assert ClusterGpuCapacity(rc).allocatable_gpus() == 16  # cordoned node excluded
    assert ClusterGpuCapacity(rc, node_selector="gpu=mi355x,pool=a").allocatable_gpus() == 8
    assert ClusterGpuCapacity(rc, node_selector="gpu=mi355x", gpus_per_pod=4).pod_capacity() == 4
    assert ClusterGpuCapacity(rc, resource="nvidia.com/gpu").allocatable_gpus() == 0


def test_capper_applies_min_and_keeps_last_good(nat):
    fake = nat.FakeDeployments("ns")
    fake.add("w", 1)
    s1 = nat.PodAutoScaler(fake, "w", "ns", 8, 1, 1, 1, nat.Logger(), nat.RealClock())
    s2 = nat.PodAutoScaler(fake, "w", "ns", 32, 1, 1, 1, nat.Logger(), nat.RealClock())
    caps = [16, RuntimeError("apiserver down"), 4]

    def capacity():
        c = caps.pop(0)
        if isinstance(c, Exception):
            raise c
        return c

    m = MaxPodsCapper([s1, s2], [8, 32], capacity)
    assert m.refresh() == 16 and (s1.max, s2.max) == (8, 16)
    assert m.refresh() == 16 and (s1.max, s2.max) == (8, 16)  # failure keeps the last cap
    assert m.refresh() == 4 and (s1.max, s2.max) == (4, 4)


def test_cli_cluster_cap(nat, kube, tmp_path, capfd):
    from kube_sqs_autoscaler_amd.cli import main

    sqs = nat.FakeSqsServer()
    sqs.start()
    try:
        url = sqs.url + "/1/q"
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": "1000"})
        kube.add_deployment("ml", "w", 1)
        kc = tmp_path / "kc"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": TOKEN}}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = {"AWS_ACCESS_KEY_ID": "a", "AWS_SECRET_ACCESS_KEY": "b", "KUBE_CONFIG_PATH": str(kc)}
        rc = main([f"--sqs-queue-url={url}", "--kubernetes-deployment=w", "--kubernetes-namespace=ml", "--aws-region=us-east-1",
                   f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-up-cool-down=0s", "--scale-up-pods=3",
                   "--max-pods=100", "--attribute-names=ApproximateNumberOfMessages", "--gpu-aware-max=cluster",
                   "--gpu-node-selector=gpu=mi355x,pool=a", "--gpus-per-pod=2"], environ=env, max_iterations=5)
        assert rc == 0
        assert kube.replicas("ml", "w") == 4  # 8 GPUs on pool a / 2 per pod
        assert "GPU capacity: 4 pods" in capfd.readouterr().err
    finally:
        sqs.stop()


def test_capper_floors_at_min_pods_and_ignores_zero_capacity(nat):
    """a capacity of 0 (no GPU visible to a `local` probe, every GPU node cordoned)
    must not freeze scale-up at 0; a capacity below --min-pods never caps below it."""
    fake = nat.FakeDeployments("ns")
    fake.add("w", 1)
    s = nat.PodAutoScaler(fake, "w", "ns", 8, 3, 1, 1, nat.Logger(), nat.RealClock())
    caps = [0, 2, 5, 0]
    logs = []
    m = MaxPodsCapper([s], [8], lambda: caps.pop(0), log=lambda lvl, msg: logs.append((lvl, msg)))
    assert m.refresh() == 0 and s.max == 8  # unknown capacity: the configured max stays
    assert logs[-1][0] == "warning" and "keeping the configured max-pods [8]" in logs[-1][1]
    assert m.refresh() == 2 and s.max == 3  # floored at min-pods (3)
    assert m.refresh() == 5 and s.max == 5
    assert m.refresh() == 0 and s.max == 8


def test_local_cap_with_no_gpu_still_scales_to_max(nat, tmp_path, capfd, monkeypatch):
    """--gpu-aware-max=local on a pod that sees no GPU: a warning, and scale-up still reaches the
    configured --max-pods."""
    from kube_sqs_autoscaler_amd.cli import main
    from kube_sqs_autoscaler_amd.ops import gpu

    monkeypatch.setattr(gpu, "healthy_gpu_count", lambda: 0)
    sqs, kube = nat.FakeSqsServer(), nat.FakeKubeServer()
    sqs.start()
    kube.require_token(TOKEN)
    kube.start()
    try:
        url = sqs.url + "/1/q"
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": "1000"})
        kube.add_deployment("ml", "w", 1)
        kc = tmp_path / "kc"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": TOKEN}}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = {"AWS_ACCESS_KEY_ID": "a", "AWS_SECRET_ACCESS_KEY": "b", "KUBE_CONFIG_PATH": str(kc)}
        rc = main([f"--sqs-queue-url={url}", "--kubernetes-deployment=w", "--kubernetes-namespace=ml", "--aws-region=us-east-1",
                   f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-up-cool-down=0s", "--max-pods=6",
                   "--attribute-names=ApproximateNumberOfMessages", "--gpu-aware-max=local"], environ=env, max_iterations=8)
        assert rc == 0 and kube.replicas("ml", "w") == 6
        err = capfd.readouterr().err
        assert "level=warning" in err and "keeping the configured max-pods [6]" in err
    finally:
        sqs.stop()
        kube.stop()
