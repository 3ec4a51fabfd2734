"""The reference's pod runs with 100m CPU and 200 Mi memory (request = limit,
/root/reference/README.md:60-66). This build must fit the same pod: the whole process (and,
with --worker-processes, every worker process, counted by proportional set size so shared
pages count once) stays far below 200 Mi, and polling at a 200 ms period costs well under
100m of CPU."""
import os
import subprocess
import sys
import time

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIMIT_KB = 200 * 1024


def _pss_kb(pid):
    with open(f"/proc/{pid}/smaps_rollup") as f:
        return sum(int(l.split()[1]) for l in f if l.startswith("Pss:"))


def _cpu_ticks(pids):
    total = 0
    for pid in pids:
        with open(f"/proc/{pid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        total += int(fields[11]) + int(fields[12])  # utime + stime
    return total


@pytest.fixture
def endpoints(nat, tmp_path):
    sqs = nat.FakeSqsServer()
    sqs.start()
    kube = nat.FakeKubeServer()
    kube.start()
    kc = tmp_path / "kubeconfig"
    kc.write_text(yaml.safe_dump({
        "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
        "users": [{"name": "u", "user": {"token": "t"}}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
    env = dict(os.environ, AWS_ACCESS_KEY_ID="AKIDRES", AWS_SECRET_ACCESS_KEY="s", KUBE_CONFIG_PATH=str(kc))
    yield sqs, kube, env
    sqs.stop()
    kube.stop()


@pytest.mark.parametrize("queues,procs", [(1, False), (8, False), (8, True)], ids=["1q", "8q-threads", "8q-processes"])
def test_fits_the_reference_pod_resources(endpoints, queues, procs):
    sqs, kube, env = endpoints
    specs = []
    for i in range(queues):
        url = f"{sqs.url}/1/q{i}"
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": "0"})
        kube.add_deployment("default", f"w{i}", 1)
        specs += ["--queue", f"url={url},deployment=w{i},attribute-names=ApproximateNumberOfMessages"]
    args = [sys.executable, "-m", "kube_sqs_autoscaler_amd", "--aws-region=us-east-1", f"--sqs-endpoint={sqs.url}",
            "--poll-period=200ms", "--metrics-addr=127.0.0.1:0", *specs]
    if procs:
        args.append("--worker-processes")
    p = subprocess.Popen(args, cwd=ROOT, env=env, stderr=subprocess.DEVNULL)
    try:
        deadline = time.time() + 60
        while sqs.requests() < 2 * queues and p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        assert p.poll() is None
        with open(f"/proc/{p.pid}/task/{p.pid}/children") as f:
            pids = [p.pid] + [int(x) for x in f.read().split()]
        assert len(pids) == (1 + queues if procs else 1)
        before, t0, r0 = _cpu_ticks(pids), time.monotonic(), sqs.requests()
        time.sleep(5.0)  # long enough that per-process tick rounding (8 processes) stays small
        ticks, wall, polls = _cpu_ticks(pids) - before, time.monotonic() - t0, sqs.requests() - r0
        pss = sum(_pss_kb(x) for x in pids)
        hz = os.sysconf("SC_CLK_TCK")
        assert polls >= queues * 15  # it was polling all along (200 ms period)
        assert pss < LIMIT_KB / 2, pss
        assert ticks / hz / wall < 0.05, (ticks, wall)  # < 50m of the reference's 100m
    finally:
        p.terminate()
        p.wait(timeout=30)
