"""Process entry point (reference main.go:82-116): flags -> clients -> "Starting" -> Run."""
import os
import subprocess
import sys

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AKID, SECRET, REGION, TOKEN = "AKIDCLI", "cli/secret", "us-east-1", "cli-token"


def run_cli(*args, env=None, timeout=60):
    e = dict(os.environ)
    e.pop("KUBE_CONFIG_PATH", None)
    e.update(env or {})
    return subprocess.run([sys.executable, "-m", "kube_sqs_autoscaler_amd", *args], cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=timeout)


def test_help_exits_zero():
    r = run_cli("-h")
    assert r.returncode == 0 and r.stderr.startswith("Usage of kube-sqs-autoscaler:\n  -api-timeout duration")
    assert "(default 8)" in r.stderr


def test_bad_flag_exits_two():
    r = run_cli("--poll-period=five")
    assert r.returncode == 2
    assert r.stderr.startswith('invalid value "five" for flag -poll-period: parse error\nUsage of')
    r = run_cli("--no-such-flag")
    assert r.returncode == 2 and r.stderr.startswith("flag provided but not defined: -no-such-flag")


def test_no_kube_config_panics_like_reference():
    r = run_cli("--sqs-queue-url=x", env={"KUBERNETES_SERVICE_HOST": ""})
    # after client-go's two klog warnings (tests/test_klog.py)
    assert r.returncode == 2 and r.stderr.splitlines()[2] == "panic: Failed to configure incluster or local config"


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


def test_main_in_process_scales_over_the_wire(servers, capfd):
    from kube_sqs_autoscaler_amd.cli import main

    sqs, kube, env = servers
    url = sqs.url + "/123/jobs"
    sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500", "ApproximateNumberOfMessagesDelayed": "0",
                             "ApproximateNumberOfMessagesNotVisible": "0"})
    kube.add_deployment("gpu", "workers", 1)
    rc = main([f"--sqs-queue-url={url}", "--kubernetes-deployment=workers", "--kubernetes-namespace=gpu",
               f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-up-cool-down=0s",
               "--scale-down-cool-down=0s"], environ=env, max_iterations=10)
    assert rc == 0
    assert kube.replicas("gpu", "workers") == 8  # the 8 x MI355X default cap
    err = capfd.readouterr().err
    assert 'level=info msg="Starting kube-sqs-autoscaler"' in err
    assert 'msg="Found 500 messages in the queue"' in err
    assert 'msg="More than max pods running. No scale up. Replicas: 8"' in err
    assert sqs.signature_failures() == 0


def test_main_multi_queue(servers, capfd):
    from kube_sqs_autoscaler_amd.cli import main

    sqs, kube, env = servers
    specs = []
    for i, depth in enumerate(["500", "0", "50"]):
        url = f"{sqs.url}/123/q{i}"
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": depth})
        kube.add_deployment("gpu", f"w{i}", 4)
        specs += ["--queue", f"url={url},deployment=w{i},namespace=gpu,attribute-names=ApproximateNumberOfMessages"]
    rc = main([f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-up-cool-down=0s",
               "--scale-down-cool-down=0s", "--max-pods=6", *specs], environ=env, max_iterations=5)
    assert rc == 0
    assert [kube.replicas("gpu", f"w{i}") for i in range(3)] == [6, 1, 4]
    err = capfd.readouterr().err
    assert "deployment=gpu/w0" in err and 'queue="' in err


def test_deployment_mode_full_object_put(servers):
    from kube_sqs_autoscaler_amd.cli import main

    sqs, kube, env = servers
    url = sqs.url + "/123/jobs"
    sqs.set_attributes(url, {"ApproximateNumberOfMessages": "0"})
    kube.add_deployment("default", "workers", 3)
    rc = main([f"--sqs-queue-url={url}", "--kubernetes-deployment=workers", f"--aws-region={REGION}",
               f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-down-cool-down=0s", "--scale-mode=deployment",
               "--attribute-names=ApproximateNumberOfMessages", "--log-level=error"], environ=env, max_iterations=1)
    assert rc == 0 and kube.replicas("default", "workers") == 2
    assert kube.last_method() == "PUT" and kube.last_path().endswith("/deployments/workers")


REFERENCE_ROLE = ["deployments:get", "deployments:update"]  # all /root/reference/scale/scale.go:55,72 needs


@pytest.mark.parametrize("rules", [REFERENCE_ROLE, REFERENCE_ROLE + ["deployments/scale:get"]],
                         ids=["reference-role", "scale-read-only"])
def test_default_flags_scale_under_a_reference_role(servers, capfd, rules):
    """A cluster whose Role was written for the reference (get/update on deployments only) is
    scaled with default flags: the first /scale request is refused (403), the worker warns once
    and continues with the reference's full-Deployment GET+PUT."""
    from kube_sqs_autoscaler_amd.cli import main

    sqs, kube, env = servers
    kube.set_rbac(rules)
    url = sqs.url + "/123/jobs"
    sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500", "ApproximateNumberOfMessagesDelayed": "0",
                             "ApproximateNumberOfMessagesNotVisible": "0"})
    kube.add_deployment("gpu", "workers", 1)
    rc = main([f"--sqs-queue-url={url}", "--kubernetes-deployment=workers", "--kubernetes-namespace=gpu",
               f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-up-cool-down=0s",
               "--scale-down-cool-down=0s"], environ=env, max_iterations=10)
    assert rc == 0
    assert kube.replicas("gpu", "workers") == 8
    err = capfd.readouterr().err
    assert err.count("level=warning") >= 1 and err.count("deployments/scale subresource is not usable") == 1
    assert "Failed scaling" not in err
    assert 1 <= kube.forbidden() <= 2  # the refused /scale GET (or PUT) -- once, then never again
    assert kube.last_path().endswith("/deployments/workers")  # no /scale request after the switch


def test_sigterm_graceful_shutdown(servers):
    sqs, kube, env = servers
    url = sqs.url + "/123/jobs"
    sqs.set_attributes(url, {"ApproximateNumberOfMessages": "0"})
    kube.add_deployment("default", "w", 1)
    e = dict(os.environ)
    e.update(env)
    p = subprocess.Popen([sys.executable, "-m", "kube_sqs_autoscaler_amd", f"--sqs-queue-url={url}", "--kubernetes-deployment=w",
                          f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=1h"],
                         cwd=ROOT, env=e, stderr=subprocess.PIPE, text=True)
    try:
        import time

        deadline = time.time() + 60
        buf = ""
        while "Starting kube-sqs-autoscaler" not in buf and time.time() < deadline:
            buf += p.stderr.readline()
        p.terminate()
        rc = p.wait(timeout=20)  # interrupts the 1 h poll sleep
        assert rc == 0
        assert "Stopped kube-sqs-autoscaler" in buf + p.stderr.read()
    finally:
        if p.poll() is None:
            p.kill()


def test_trace_file_spans(servers, tmp_path):
    import json

    from kube_sqs_autoscaler_amd.cli import main

    sqs, kube, env = servers
    url = sqs.url + "/123/jobs"
    sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500"})
    kube.add_deployment("gpu", "workers", 1)
    trace = tmp_path / "trace.jsonl"
    rc = main([f"--sqs-queue-url={url}", "--kubernetes-deployment=workers", "--kubernetes-namespace=gpu",
               f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-up-cool-down=0s",
               "--attribute-names=ApproximateNumberOfMessages", f"--trace-file={trace}", "--log-level=error"],
              environ=env, max_iterations=3)
    assert rc == 0
    spans = [json.loads(l) for l in trace.read_text().splitlines()]
    assert [s["poll"] for s in spans] == [1, 2, 3]
    assert spans[0]["depth"] == 500 and spans[0]["up"] == "scaled" and spans[0]["replicas_after"] == 2
    assert spans[0]["deployment"] == "gpu/workers" and spans[0]["queue"] == url and spans[0]["prefetched"] is True
    assert spans[0]["patch_latency_ns"] > 0 and spans[0]["depth_ns"] > 0


def test_dry_run_shadow_mode(servers, capfd):
    from kube_sqs_autoscaler_amd.cli import main

    sqs, kube, env = servers
    url = sqs.url + "/123/jobs"
    sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500"})
    kube.add_deployment("gpu", "workers", 2)
    writes = kube.writes()
    rc = main([f"--sqs-queue-url={url}", "--kubernetes-deployment=workers", "--kubernetes-namespace=gpu",
               f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-up-cool-down=0s",
               "--attribute-names=ApproximateNumberOfMessages", "--dry-run"], environ=env, max_iterations=3)
    assert rc == 0 and kube.writes() == writes and kube.replicas("gpu", "workers") == 2
    err = capfd.readouterr().err
    assert err.count('msg="Dry run: would scale up. Replicas: 2 -> 3"') == 3


def test_queue_spec_region(servers):
    from kube_sqs_autoscaler_amd.cli import main

    sqs, kube, env = servers
    # the fake verifies signatures for REGION only: a queue signed for another region fails,
    # the one with region=REGION works although --aws-region is wrong
    sqs.set_attributes(sqs.url + "/1/a", {"ApproximateNumberOfMessages": "500"})
    kube.add_deployment("gpu", "a", 1)
    rc = main(["--aws-region=eu-central-1", f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-up-cool-down=0s",
               "--attribute-names=ApproximateNumberOfMessages",
               "--queue", f"url={sqs.url}/1/a,deployment=a,namespace=gpu,region={REGION}"], environ=env, max_iterations=2)
    assert rc == 0 and kube.replicas("gpu", "a") == 3 and sqs.signature_failures() == 0


def test_main_end_to_end_over_tls(nat, tmp_path, capfd):
    """Both endpoints on TLS: kubeconfig CA data for the apiserver, AWS_CA_BUNDLE for SQS."""
    import base64

    from kube_sqs_autoscaler_amd.cli import main

    sqs, kube = nat.FakeSqsServer(), nat.FakeKubeServer()
    sqs.require_signature(AKID, SECRET, REGION)
    sqs.start("127.0.0.1", 0, True)
    kube.require_token(TOKEN)
    kube.start("127.0.0.1", 0, True)
    try:
        bundle = tmp_path / "aws-ca.pem"
        bundle.write_text(sqs.cert_pem)
        kc = tmp_path / "kc"
        kc.write_text(yaml.safe_dump({
            "current-context": "t",
            "clusters": [{"name": "c", "cluster": {"server": kube.url,
                                                   "certificate-authority-data": base64.b64encode(kube.cert_pem.encode()).decode()}}],
            "users": [{"name": "u", "user": {"token": TOKEN}}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = {"AWS_ACCESS_KEY_ID": AKID, "AWS_SECRET_ACCESS_KEY": SECRET, "KUBE_CONFIG_PATH": str(kc),
               "AWS_CA_BUNDLE": str(bundle)}
        url = sqs.url + "/123/jobs"
        assert url.startswith("https://") and kube.url.startswith("https://")
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": "500"})
        kube.add_deployment("gpu", "workers", 1)
        rc = main([f"--sqs-queue-url={url}", "--kubernetes-deployment=workers", "--kubernetes-namespace=gpu",
                   f"--aws-region={REGION}", f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-up-cool-down=0s",
                   "--attribute-names=ApproximateNumberOfMessages"], environ=env, max_iterations=3)
        assert rc == 0 and kube.replicas("gpu", "workers") == 4
        assert "level=error" not in capfd.readouterr().err
    finally:
        sqs.stop()
        kube.stop()


def test_reference_command_path_launcher():
    """The image installs deploy/bin/kube-sqs-autoscaler at /kube-sqs-autoscaler, so the
    reference's `command: [/kube-sqs-autoscaler, ...]` manifests run unchanged; like a Go
    binary, usage names the program by its argv[0]."""
    exe = os.path.join(ROOT, "deploy", "bin", "kube-sqs-autoscaler")
    assert os.access(exe, os.X_OK)
    e = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([exe, "-h"], env=e, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stderr.startswith(f"Usage of {exe}:\n  -api-timeout duration")
    r = subprocess.run([exe, "--max-pods=x"], env=e, capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and r.stderr.startswith('invalid value "x" for flag -max-pods: parse error')
