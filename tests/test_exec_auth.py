"""client-go exec credential plugins (kubeconfig ``users[].user.exec``).

The reference builds its client with ``clientcmd.BuildConfigFromFlags`` on ``KUBE_CONFIG_PATH``
(/root/reference/scale/scale.go:32-38, client-go v0.19.4 per go.mod:17), whose transport runs a
user's exec plugin (``aws eks get-token`` on EKS) and caches the ExecCredential until it
expires or a 401 comes back. Parity unpinned: client-go is not importable here, so these tests
pin the documented ExecCredential contract with a scripted plugin.
"""
import json
import os
import stat
import sys
import textwrap

import pytest
import yaml

from kube_sqs_autoscaler_amd import autoscaler
from kube_sqs_autoscaler_amd.kube.config import KubeConfigError, load_kubeconfig

V1B1 = "client.authentication.k8s.io/v1beta1"
V1A1 = "client.authentication.k8s.io/v1alpha1"
S = 1_000_000_000


def plugin(tmp_path, body, name="plugin.py"):
    """An executable Python credential plugin; it appends one line per run to runs.log."""
    p = tmp_path / name
    p.write_text(f"#!{sys.executable}\n" + textwrap.dedent("""
        import json, os, sys
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "runs.log"), "a") as f:
            f.write(json.dumps({"argv": sys.argv[1:], "info": os.environ.get("KUBERNETES_EXEC_INFO"),
                                "env": os.environ.get("PLUGIN_ENV")}) + "\\n")
    """) + textwrap.dedent(body))
    p.chmod(p.stat().st_mode | stat.S_IXUSR)
    return str(p)


def runs(tmp_path):
    f = tmp_path / "runs.log"
    return [json.loads(l) for l in f.read_text().splitlines()] if f.exists() else []


def cred_body(api=V1B1, token="tok", expiry=None, extra=""):
    st = {"token": token}
    if expiry:
        st["expirationTimestamp"] = expiry
    return f"print(json.dumps({{'kind': 'ExecCredential', 'apiVersion': {api!r}, 'status': {st!r}}}))\n" + extra


def exec_cfg(nat, command, api=V1B1, args=(), env=(), hint="", timeout_ns=0):
    c = nat.ExecConfig()
    c.command, c.args, c.env, c.api_version, c.install_hint, c.timeout_ns = command, list(args), list(env), api, hint, timeout_ns
    return c


@pytest.mark.parametrize("s,want", [
    ("1970-01-01T00:00:00Z", 0),
    ("2024-02-29T12:00:00Z", 1709208000 * S),
    ("2024-02-29T12:00:00.5Z", 1709208000 * S + S // 2),
    ("2024-02-29T14:30:00+02:30", 1709208000 * S),
    ("2024-02-29T07:00:00-05:00", 1709208000 * S),
    ("2000-01-01T00:00:00.123456789Z", 946684800 * S + 123456789),
])
def test_parse_rfc3339(nat, s, want):
    assert nat.parse_rfc3339(s) == want


@pytest.mark.parametrize("s", ["", "2023-02-29T00:00:00Z", "2024-13-01T00:00:00Z", "2024-01-01 00:00:00Z",
                               "2024-01-01T00:00:00", "2024-01-01T24:00:00Z", "2024-01-01T00:00:00.Z",
                               "2024-01-01T00:00:00+0100"])
def test_parse_rfc3339_rejects(nat, s):
    assert nat.parse_rfc3339(s) is None


def test_v1beta1_token_args_env(nat, tmp_path):
    cmd = plugin(tmp_path, cred_body(token="abc"))
    c = nat.run_exec_plugin(exec_cfg(nat, cmd, args=["eks", "get-token"], env=[("PLUGIN_ENV", "from-kubeconfig")]))
    assert c.token == "abc" and not c.has_expiry and c.cert_pem == ""
    r = runs(tmp_path)[0]
    assert r["argv"] == ["eks", "get-token"] and r["env"] == "from-kubeconfig"
    assert r["info"] is None  # client-go sends KUBERNETES_EXEC_INFO to v1alpha1 plugins only


def test_kubeconfig_env_overrides_process_env(nat, tmp_path, monkeypatch):
    monkeypatch.setenv("PLUGIN_ENV", "from-process")
    cmd = plugin(tmp_path, cred_body())
    nat.run_exec_plugin(exec_cfg(nat, cmd))
    nat.run_exec_plugin(exec_cfg(nat, cmd, env=[("PLUGIN_ENV", "override")]))
    assert [r["env"] for r in runs(tmp_path)] == ["from-process", "override"]


def test_v1alpha1_exec_info_and_401_response(nat, tmp_path):
    cmd = plugin(tmp_path, cred_body(api=V1A1))
    nat.run_exec_plugin(exec_cfg(nat, cmd, api=V1A1))
    nat.run_exec_plugin(exec_cfg(nat, cmd, api=V1A1), 401)
    infos = [json.loads(r["info"]) for r in runs(tmp_path)]
    assert infos[0] == {"kind": "ExecCredential", "apiVersion": V1A1, "spec": {}}
    assert infos[1]["spec"] == {"response": {"code": 401}}


def test_client_certificate_and_expiry(nat, tmp_path):
    body = ("print(json.dumps({'kind': 'ExecCredential', 'apiVersion': %r, 'status': {'clientCertificateData': 'CERT',"
            " 'clientKeyData': 'KEY', 'expirationTimestamp': '2030-01-01T00:00:00Z'}}))\n" % V1B1)
    c = nat.run_exec_plugin(exec_cfg(nat, plugin(tmp_path, body)))
    assert (c.token, c.cert_pem, c.key_pem, c.has_expiry) == ("", "CERT", "KEY", True)
    assert c.expiry_unix_ns == nat.parse_rfc3339("2030-01-01T00:00:00Z")


@pytest.mark.parametrize("body,msg", [
    (cred_body(api=V1A1), "plugin is configured to use API version client.authentication.k8s.io/v1beta1, plugin returned version client.authentication.k8s.io/v1alpha1"),
    ("print(json.dumps({'kind': 'ExecCredential', 'apiVersion': %r}))\n" % V1B1, "didn't return a status field"),
    ("print(json.dumps({'kind': 'ExecCredential', 'apiVersion': %r, 'status': {}}))\n" % V1B1, "didn't return a token or cert/key pair"),
    ("print(json.dumps({'kind': 'ExecCredential', 'apiVersion': %r, 'status': {'clientCertificateData': 'C'}}))\n" % V1B1,
     "returned only certificate or key, not both"),
    ("print('not json')\n", "decoding stdout"),
    ("print(json.dumps({'apiVersion': %r, 'status': {'token': 't'}}))\n" % V1B1, "Object 'Kind' is missing"),
    (cred_body(expiry="tomorrow"), "bad expirationTimestamp"),
    ("sys.exit(3)\n", "failed with exit code 3"),
])
def test_plugin_errors(nat, tmp_path, body, msg):
    with pytest.raises(nat.NativeError, match=msg.replace("(", r"\(").replace(")", r"\)")):
        nat.run_exec_plugin(exec_cfg(nat, plugin(tmp_path, body)))


def test_not_found_shows_install_hint(nat):
    with pytest.raises(nat.NativeError) as e:
        nat.run_exec_plugin(exec_cfg(nat, "ksa-no-such-plugin", hint="install it with: brew install thing"))
    assert "exec: executable ksa-no-such-plugin not found" in str(e.value)
    assert "install it with: brew install thing" in str(e.value)


def test_invalid_api_version(nat):
    with pytest.raises(nat.NativeError, match='exec plugin: invalid apiVersion "v9"'):
        nat.validate_exec_config(exec_cfg(nat, "x", api="v9"))


def test_timeout_kills_a_hung_plugin(nat, tmp_path):
    cmd = plugin(tmp_path, "import time; time.sleep(30)\n")
    with pytest.raises(nat.NativeError, match="timed out after 300ms"):
        nat.run_exec_plugin(exec_cfg(nat, cmd, timeout_ns=300_000_000))


def test_provider_caches_until_expiry(nat, tmp_path):
    clock = nat.VirtualClock(0, nat.parse_rfc3339("2030-01-01T00:00:00Z") - 10 * S)
    cmd = plugin(tmp_path, cred_body(token="t1", expiry="2030-01-01T00:00:00Z"))
    p = nat.ExecTokenProvider(exec_cfg(nat, cmd), clock)
    assert p.token() == "t1" and p.token() == "t1" and p.runs == 1
    clock.advance(10 * S)  # exactly at expiry: not yet After
    assert p.token() == "t1" and p.runs == 1
    clock.advance(1)
    assert p.token() == "t1" and p.runs == 2  # expired -> plugin runs again


def test_provider_without_expiry_refreshes_only_on_401(nat, tmp_path):
    cmd = plugin(tmp_path, cred_body(token="t1"))
    p = nat.ExecTokenProvider(exec_cfg(nat, cmd), nat.RealClock())
    assert p.token() == "t1" and p.token() == "t1" and p.runs == 1
    p.invalidate("some-other-token")  # a 401 on a token we no longer hold
    assert p.token() == "t1" and p.runs == 1
    p.invalidate("t1")
    assert p.token() == "t1" and p.runs == 2


def test_provider_error_is_wrapped(nat, tmp_path):
    p = nat.ExecTokenProvider(exec_cfg(nat, plugin(tmp_path, "sys.exit(1)\n")), nat.RealClock())
    with pytest.raises(nat.NativeError, match="getting credentials: exec: executable .* failed with exit code 1"):
        p.token()


def write_kc(tmp_path, user, server="https://api:6443"):
    kc = tmp_path / "kubeconfig"
    kc.write_text(yaml.safe_dump({
        "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": server}}],
        "users": [{"name": "u", "user": user}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
    return str(kc)


def test_kubeconfig_exec_stanza(tmp_path):
    rc = load_kubeconfig(write_kc(tmp_path, {"exec": {
        "apiVersion": V1B1, "command": "aws", "args": ["eks", "get-token", "--cluster-name", "gpu"],
        "env": [{"name": "AWS_PROFILE", "value": "ml"}], "installHint": "install the AWS CLI"}}))
    e = rc.exec_plugin
    assert (e.command, e.args, e.env, e.install_hint) == ("aws", ["eks", "get-token", "--cluster-name", "gpu"],
                                                           [("AWS_PROFILE", "ml")], "install the AWS CLI")


def test_kubeconfig_exec_relative_command(tmp_path):
    rc = load_kubeconfig(write_kc(tmp_path, {"exec": {"apiVersion": V1B1, "command": "./bin/plugin"}}))
    assert rc.exec_plugin.command == os.path.join(str(tmp_path), "./bin/plugin")


@pytest.mark.parametrize("user,msg", [
    ({"exec": {"apiVersion": "v1", "command": "x"}}, 'invalid apiVersion "v1"'),
    ({"exec": {"apiVersion": V1B1}}, "command must be specified"),
    ({"exec": {"apiVersion": V1B1, "command": "x"}, "auth-provider": {"name": "gcp"}},
     "authProvider cannot be provided in combination with an exec plugin"),
])
def test_kubeconfig_exec_errors(tmp_path, user, msg):
    with pytest.raises(KubeConfigError, match=msg):
        load_kubeconfig(write_kc(tmp_path, user))


def test_auth_provider_fails_at_client_construction(tmp_path):
    rc = load_kubeconfig(write_kc(tmp_path, {"auth-provider": {"name": "gcp", "config": {}}}))
    with pytest.raises(autoscaler.KubeClientError, match='no Auth Provider found for name "gcp"'):
        autoscaler.prepare_kube_auth(rc)


def test_exec_over_the_wire_with_rotation(nat, tmp_path):
    """The actuator authenticates with the plugin's token; when the apiserver starts rejecting
    it (401), the next request re-runs the plugin and succeeds with the rotated token."""
    (tmp_path / "current").write_text("tok-1")
    body = ("tok = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'current')).read()\n"
            "print(json.dumps({'kind': 'ExecCredential', 'apiVersion': %r, 'status': {'token': tok}}))\n" % V1B1)
    cmd = plugin(tmp_path, body)
    kube = nat.FakeKubeServer()
    kube.require_token("tok-1")
    kube.start()
    try:
        kube.add_deployment("ml", "workers", 3)
        rc = load_kubeconfig(write_kc(tmp_path, {"exec": {"apiVersion": V1B1, "command": cmd}}, kube.url))
        assert autoscaler.prepare_kube_auth(rc) is None
        apis = [autoscaler.new_deployment_api(rc, "ml", "scale", 5 * S) for _ in range(4)]
        for a in apis:
            assert a.get("workers").replicas == 3
        assert len(runs(tmp_path)) == 1  # one authenticator shared by every client of the config
        (tmp_path / "current").write_text("tok-2")
        kube.require_token("tok-2")
        with pytest.raises(nat.NativeError, match="Unauthorized"):
            apis[0].get("workers")
        assert apis[1].get("workers").replicas == 3  # refreshed after the 401
        assert len(runs(tmp_path)) == 2
    finally:
        kube.stop()


def test_cli_auth_provider_panics_like_reference(tmp_path, capfd):
    from kube_sqs_autoscaler_amd.cli import main

    kc = write_kc(tmp_path, {"auth-provider": {"name": "oidc"}})
    rc = main(["--sqs-queue-url=https://q", "--kubernetes-deployment=d", "--aws-region=us-east-1"],
              environ={"KUBE_CONFIG_PATH": kc, "AWS_ACCESS_KEY_ID": "a", "AWS_SECRET_ACCESS_KEY": "b"}, max_iterations=0)
    assert rc == 2
    assert "panic: Failed to configure client" in capfd.readouterr().err
