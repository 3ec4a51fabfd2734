"""client-go's start-up warnings as klog lines (clientcmd.BuildConfigFromFlags("", ""),
/root/reference/scale/scale.go:33; klog v2.2.0 text format, utils/klog.py)."""
import io
import os
import re
import subprocess
import sys
from datetime import datetime

import pytest

from kube_sqs_autoscaler_amd.kube.config import KubeConfigError, build_config_from_flags
from kube_sqs_autoscaler_amd.utils.klog import Klog, format_line

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NEITHER = "Neither --kubeconfig nor --master was specified.  Using the inClusterConfig.  This might not work."
KLOG = re.compile(r"^W(\d{4}) (\d\d:\d\d:\d\d\.\d{6}) +(\d+) client_config\.go:(\d+)\] (.*)$")


def test_header_layout():
    t = datetime(2026, 1, 7, 5, 4, 3, 123)
    assert format_line("W", "client_config.go", 608, "x", now=t, pid=42) == \
        "W0107 05:04:03.000123      42 client_config.go:608] x\n"
    assert format_line("E", "f.go", 1, "y\n", now=t, pid=1234567) == "E0107 05:04:03.000123 1234567 f.go:1] y\n"


def test_in_cluster_success_warns_once(tmp_path):
    (tmp_path / "token").write_text("tok\n")
    out = io.StringIO()
    rc = build_config_from_flags("", {"KUBERNETES_SERVICE_HOST": "10.0.0.1", "KUBERNETES_SERVICE_PORT": "443"},
                                 sa_dir=str(tmp_path), klog=Klog(out))
    assert rc.host == "https://10.0.0.1:443"
    lines = out.getvalue().splitlines()
    assert len(lines) == 1
    m = KLOG.match(lines[0])
    assert m and m.group(4) == "608" and m.group(5) == NEITHER and int(m.group(3)) == os.getpid()


def test_explicit_path_logs_nothing(tmp_path):
    out = io.StringIO()
    with pytest.raises(KubeConfigError):
        build_config_from_flags(str(tmp_path / "missing"), {}, klog=Klog(out))
    assert out.getvalue() == ""


def test_cli_prints_both_klog_lines_then_panics(tmp_path):
    e = dict(os.environ)
    e.pop("KUBE_CONFIG_PATH", None)
    e.update({"KUBERNETES_SERVICE_HOST": "", "HOME": str(tmp_path)})
    r = subprocess.run([sys.executable, "-m", "kube_sqs_autoscaler_amd"], cwd=ROOT, env=e, capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 2
    lines = r.stderr.splitlines()
    m1, m2 = KLOG.match(lines[0]), KLOG.match(lines[1])
    assert m1 and m1.group(4) == "608" and m1.group(5) == NEITHER
    assert m2 and m2.group(4) == "613" and m2.group(5) == (
        "error creating inClusterConfig, falling back to default config: unable to load in-cluster configuration, "
        "KUBERNETES_SERVICE_HOST and KUBERNETES_SERVICE_PORT must be defined")
    assert lines[2] == "panic: Failed to configure incluster or local config"
    assert "level=warning" not in r.stderr  # not logrus lines
