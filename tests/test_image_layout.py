"""The slim image's file system, assembled the way the Dockerfile's `base` + `slim` stages do
(Dockerfile: the package under /app, the launcher at /kube-sqs-autoscaler, PYTHONPATH=/app,
KSA_NO_AUTOBUILD=1, libksa_gpu.so and host tools removed), run with nothing importable but the
standard library, PyYAML and prometheus_client (the image's only runtime Python packages,
python3-yaml and python3-prometheus-client). The reference's manifest command
(`/kube-sqs-autoscaler --flags...`, /root/reference/README.md:37-39) must scale a Deployment
and stop cleanly on SIGTERM. No image is built here (no container runtime in CI's CPU tier);
this checks what the image would contain."""
import os
import shutil
import signal
import subprocess
import sys
import time

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AKID, SECRET, REGION, TOKEN = "AKIDIMAGE", "image/secret", "us-east-1", "image-token"


@pytest.fixture
def image_root(nat, tmp_path):
    import prometheus_client

    app = tmp_path / "app"
    shutil.copytree(os.path.join(ROOT, "kube_sqs_autoscaler_amd"), app / "kube_sqs_autoscaler_amd",
                    ignore=shutil.ignore_patterns("__pycache__", "libksa_gpu.so", "*.bin"))
    deps = tmp_path / "dist-packages"
    deps.mkdir()
    for mod in (yaml, prometheus_client):
        d = os.path.dirname(mod.__file__)
        os.symlink(d, deps / os.path.basename(d))
    launcher = tmp_path / "kube-sqs-autoscaler"
    shutil.copy(os.path.join(ROOT, "deploy", "bin", "kube-sqs-autoscaler"), launcher)
    return tmp_path, launcher, f"{app}:{deps}"


def test_slim_image_layout_scales_with_only_its_runtime_packages(nat, image_root):
    tmp, launcher, pythonpath = image_root
    sqs = nat.FakeSqsServer()
    sqs.require_signature(AKID, SECRET, REGION)
    sqs.start()
    kube = nat.FakeKubeServer()
    kube.require_token(TOKEN)
    kube.start()
    kc = tmp / "kubeconfig"
    kc.write_text(yaml.safe_dump({
        "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
        "users": [{"name": "u", "user": {"token": TOKEN}}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
    url = sqs.url + "/123/jobs"
    sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500", "ApproximateNumberOfMessagesDelayed": "0",
                             "ApproximateNumberOfMessagesNotVisible": "0"})
    kube.add_deployment("gpu", "workers", 1)
    env = {"PATH": os.environ.get("PATH", "/usr/bin:/bin"), "PYTHONPATH": pythonpath, "KSA_NO_AUTOBUILD": "1",
           "AWS_ACCESS_KEY_ID": AKID, "AWS_SECRET_ACCESS_KEY": SECRET, "KUBE_CONFIG_PATH": str(kc),
           "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    # -S: no site-packages, so only the image's packages (PYTHONPATH) can be imported
    err_path = tmp / "stderr.log"  # a file, not a pipe: nobody drains a pipe while it runs
    with open(err_path, "w") as err_file:
        p = subprocess.Popen([sys.executable, "-S", str(launcher), f"--sqs-queue-url={url}",
                              "--kubernetes-deployment=workers", "--kubernetes-namespace=gpu", f"--aws-region={REGION}",
                              f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-up-cool-down=0s",
                              "--scale-down-cool-down=0s"],
                             cwd=str(tmp), env=env, stderr=err_file, text=True)
    try:
        deadline = time.time() + 60
        while kube.replicas("gpu", "workers") < 8 and p.poll() is None and time.time() < deadline:
            time.sleep(0.01)
        p.send_signal(signal.SIGTERM)
        rc = p.wait(timeout=30)
        err = err_path.read_text()
        assert rc == 0, err[-2000:]
        assert kube.replicas("gpu", "workers") == 8
        assert 'msg="Starting kube-sqs-autoscaler"' in err and 'msg="Found 500 messages in the queue"' in err
        assert "Stopped kube-sqs-autoscaler" in err
        assert sqs.signature_failures() == 0
    finally:
        if p.poll() is None:
            p.kill()
        sqs.stop()
        kube.stop()
