"""The autoscaler must fit the reference's pod budget: 200Mi memory, 100m CPU (README.md:60-66)."""
import os
import subprocess
import sys
import time

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rss_and_cpu_within_reference_pod_limits(nat, tmp_path):
    sqs, kube = nat.FakeSqsServer(), nat.FakeKubeServer()
    sqs.start()
    kube.start()
    try:
        kc = tmp_path / "kc"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": "x"}}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = dict(os.environ, AWS_ACCESS_KEY_ID="a", AWS_SECRET_ACCESS_KEY="b", KUBE_CONFIG_PATH=str(kc))
        args = [sys.executable, "-m", "kube_sqs_autoscaler_amd", "--aws-region=us-east-1", f"--sqs-endpoint={sqs.url}",
                "--poll-period=500ms", "--log-level=error"]
        for i in range(32):
            url = f"{sqs.url}/1/q{i}"
            sqs.set_attributes(url, {"ApproximateNumberOfMessages": "0", "ApproximateNumberOfMessagesDelayed": "0",
                                     "ApproximateNumberOfMessagesNotVisible": "0"})
            kube.add_deployment("ml", f"w{i}", 1)
            args += ["--queue", f"url={url},deployment=w{i},namespace=ml"]
        p = subprocess.Popen(args, cwd=ROOT, env=env, stderr=subprocess.DEVNULL)
        try:
            time.sleep(3)
            stat = lambda: open(f"/proc/{p.pid}/stat").read().split()
            t0, s0 = time.time(), stat()
            time.sleep(3)
            t1, s1 = time.time(), stat()
            cpu = (int(s1[13]) + int(s1[14]) - int(s0[13]) - int(s0[14])) / os.sysconf("SC_CLK_TCK") / (t1 - t0)
            rss_kb = int([l for l in open(f"/proc/{p.pid}/status") if l.startswith("VmHWM")][0].split()[1])
            assert p.poll() is None
            assert rss_kb < 200 * 1024, rss_kb  # 200Mi
            assert cpu < 0.1, cpu  # 100m, with 32 queues polled twice a second
        finally:
            p.terminate()
            p.wait(timeout=20)
        assert sqs.requests() > 32  # every queue really polled
    finally:
        sqs.stop()
        kube.stop()
