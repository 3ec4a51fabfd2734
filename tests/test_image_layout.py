"""The slim image's file system, assembled the way the Dockerfile's `base` + `slim` stages do
(Dockerfile: the package under /app, the launcher at /kube-sqs-autoscaler, PYTHONPATH=/app,
KSA_NO_AUTOBUILD=1, libksa_gpu.so and host tools removed), run with nothing importable but the
standard library and PyYAML (the image's only runtime Python package, Ubuntu 22.04's
python3-yaml 5.4.1; the metrics endpoint writes the Prometheus text format itself). The
reference's manifest command (`/kube-sqs-autoscaler --flags...`, /root/reference/README.md:37-39)
must scale a Deployment, serve /metrics and /readyz, and stop cleanly on SIGTERM. No image is
built here (no container runtime in CI's CPU tier); this checks what the image would contain,
and which modules the process actually loaded."""
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


@pytest.fixture(scope="module")
def image_native(tmp_path_factory):
    """_ksa_native as the image builders make it (`ops.build --image`: -DKSA_HTTP_TIMING=0),
    built outside the tree (objects cached under build/obj-image)."""
    from kube_sqs_autoscaler_amd.ops import build

    out = tmp_path_factory.mktemp("image-native") / build.NATIVE_SO.name
    return build.build_image_runtime(verbose=False, out=out)


@pytest.fixture
def image_root(nat, image_native, tmp_path):
    """The slim image's /app: the package without the GPU probe, the test doubles
    (_ksa_fakes) or the in-tree dev build of the runtime, plus the image build of _ksa_native."""
    app = tmp_path / "app"
    shutil.copytree(os.path.join(ROOT, "kube_sqs_autoscaler_amd"), app / "kube_sqs_autoscaler_amd",
                    ignore=shutil.ignore_patterns("__pycache__", "libksa_gpu.so", "*.bin", "_ksa_fakes*", "_ksa_native*"))
    shutil.copy(image_native, app / "kube_sqs_autoscaler_amd" / "ops" / image_native.name)
    deps = tmp_path / "dist-packages"
    deps.mkdir()
    d = os.path.dirname(yaml.__file__)
    os.symlink(d, deps / os.path.basename(d))
    launcher = tmp_path / "kube-sqs-autoscaler"
    shutil.copy(os.path.join(ROOT, "deploy", "bin", "kube-sqs-autoscaler"), launcher)
    return tmp_path, launcher, f"{app}:{deps}"


def test_image_runtime_carries_no_test_doubles_or_timing(image_native, image_root):
    """What the image ships: no _ksa_fakes in the package; its _ksa_native links none of the
    fakes (servers, in-memory API fakes) and has the HTTP timing diagnostics compiled out. The
    in-tree dev build has no fakes either (they live in _ksa_fakes)."""
    tmp, _, pythonpath = image_root
    files = [f for _, _, fs in os.walk(tmp / "app") for f in fs]
    assert not any(f.startswith("_ksa_fakes") for f in files)
    syms = subprocess.run(["nm", "-C", str(image_native)], capture_output=True, text=True, check=True).stdout
    for banned in ("FakeSqsServer", "FakeKubeServer", "FakeDeployments", "MockSqsApi", "TraceSqsApi",
                   "HttpServer", "generate_self_signed", "enable_rx_timestamps"):
        assert banned not in syms, banned
    code = ("from kube_sqs_autoscaler_amd.ops import native; n = native(); assert n.__file__.startswith(%r); "
            "print(n.HTTP_TIMING, sorted(a for a in dir(n) if a.startswith(('Fake', 'Mock', 'Trace', 'Injected'))))" % str(tmp))
    r = subprocess.run([sys.executable, "-S", "-c", code], env={"PYTHONPATH": pythonpath, "KSA_NO_AUTOBUILD": "1"},
                       capture_output=True, text=True, timeout=60, cwd=str(tmp))  # cwd: not the tree's copy
    assert r.returncode == 0 and r.stdout.split() == ["False", "[]"], r.stdout + r.stderr
    code = ("from kube_sqs_autoscaler_amd.ops import NativeUnavailable, fakes\n"
            "try:\n    fakes()\nexcept NativeUnavailable as e:\n    print('refused:', e)\n")
    r = subprocess.run([sys.executable, "-S", "-c", code], env={"PYTHONPATH": pythonpath, "KSA_NO_AUTOBUILD": "1"},
                       capture_output=True, text=True, timeout=60, cwd=str(tmp))
    assert r.returncode == 0 and r.stdout.startswith("refused: cannot import the native fakes (test builds only)"), \
        r.stdout + r.stderr
    from kube_sqs_autoscaler_amd.ops import native

    assert native().HTTP_TIMING is True
    assert not [a for a in dir(native()) if a.startswith(("Fake", "Mock", "Trace", "Injected"))]


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
    import socket

    with socket.socket() as sk:  # a free port for --metrics-addr
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    # -S: no site-packages, so only the image's packages (PYTHONPATH) can be imported
    err_path = tmp / "stderr.log"  # a file, not a pipe: nobody drains a pipe while it runs
    modules_path = tmp / "modules.txt"
    # the launcher runs under a wrapper that records every module loaded when the process exits
    wrapper = tmp / "run.py"
    wrapper.write_text("import atexit, runpy, sys\n"
                       f"atexit.register(lambda: open({str(modules_path)!r}, 'w').write('\\n'.join(sorted(sys.modules))))\n"
                       f"sys.argv = [{str(launcher)!r}] + sys.argv[1:]\n"
                       f"runpy.run_path({str(launcher)!r}, run_name='__main__')\n")
    with open(err_path, "w") as err_file:
        p = subprocess.Popen([sys.executable, "-S", str(wrapper), f"--sqs-queue-url={url}",
                              "--kubernetes-deployment=workers", "--kubernetes-namespace=gpu", f"--aws-region={REGION}",
                              f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-up-cool-down=0s",
                              "--scale-down-cool-down=0s", f"--metrics-addr=127.0.0.1:{port}"],
                             cwd=str(tmp), env=env, stderr=err_file, text=True)
    try:
        deadline = time.time() + 60
        while kube.replicas("gpu", "workers") < 8 and p.poll() is None and time.time() < deadline:
            time.sleep(0.01)
        import urllib.request

        metrics = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=10).read().decode()
        assert 'ksa_polls_total{deployment="gpu/workers"' in metrics and "# TYPE ksa_poll_to_patch_latency_seconds histogram" in metrics
        assert urllib.request.urlopen(f"http://127.0.0.1:{port}/readyz", timeout=10).read() == b"ok"
        p.send_signal(signal.SIGTERM)
        rc = p.wait(timeout=30)
        err = err_path.read_text()
        assert rc == 0, err[-2000:]
        assert kube.replicas("gpu", "workers") == 8
        assert 'msg="Starting kube-sqs-autoscaler"' in err and 'msg="Found 500 messages in the queue"' in err
        assert "Stopped kube-sqs-autoscaler" in err
        assert sqs.signature_failures() == 0
        # nothing outside the standard library, PyYAML and the package itself was imported
        import sysconfig

        stdlib = sysconfig.get_paths()["stdlib"]
        loaded = modules_path.read_text().split()
        outside = []
        for name in loaded:
            top = name.split(".")[0]
            if top in ("kube_sqs_autoscaler_amd", "yaml", "_yaml", "__main__") or top in sys.builtin_module_names:
                continue
            if top == "cython_runtime" or top.startswith("_cython_"):  # PyYAML's compiled _yaml module
                continue
            spec_file = getattr(sys.modules.get(top), "__file__", None) or ""
            if top in sys.stdlib_module_names or spec_file.startswith(stdlib):
                continue
            outside.append(name)
        assert not outside, outside
        assert "prometheus_client" not in loaded and "torch" not in loaded
        assert "kube_sqs_autoscaler_amd.ops._ksa_fakes" not in loaded
    finally:
        if p.poll() is None:
            p.kill()
        sqs.stop()
        kube.stop()


def test_package_uses_only_pyyaml_api_present_in_ubuntu_2204():
    """The image ships Ubuntu 22.04's python3-yaml 5.4.1, not this container's PyYAML 6: the
    package may only use what 5.4.1 has too -- safe_load / safe_dump and the error base class
    (no yaml.load without a Loader, which 6 made mandatory; nothing added in 6)."""
    import re

    allowed = {"safe_load", "safe_dump", "YAMLError"}
    used = set()
    pkg = os.path.join(ROOT, "kube_sqs_autoscaler_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith(".py"):
                with open(os.path.join(dirpath, fn)) as f:
                    used |= set(re.findall(r"\byaml\.(\w+)", f.read()))
    assert used and used <= allowed, used - allowed


def test_an_in_tree_image_build_is_replaced_by_the_release_module(monkeypatch, tmp_path):
    """`ops.build --image` writes the timing-less module over the in-tree one. Its
    stamp makes native_up_to_date() false, so the next native() rebuilds the release module; the
    stamp goes with that rebuild."""
    from kube_sqs_autoscaler_amd.ops import build

    stamp = tmp_path / "stamp"
    monkeypatch.setattr(build, "IMAGE_STAMP", stamp)
    assert build.native_up_to_date()
    stamp.write_text("-DKSA_HTTP_TIMING=0\n")
    assert not build.native_up_to_date()
    build.build_native(verbose=False)  # objects are current: a relink
    assert not stamp.exists() and build.native_up_to_date()


def test_fakes_refuse_an_image_build_of_the_runtime_in_a_dev_tree(monkeypatch, nat):
    """A dev tree whose loaded _ksa_native is the image build (no HTTP timing) gets a clear error
    from fakes() instead of attribution rows that come out empty."""
    import kube_sqs_autoscaler_amd.ops as ops

    monkeypatch.setattr(ops, "_fakes", None)
    monkeypatch.setattr(ops.native(), "HTTP_TIMING", False)
    with pytest.raises(ops.NativeUnavailable, match="image build"):
        ops.fakes()
