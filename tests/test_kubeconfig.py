"""Kube client configuration (clientcmd.BuildConfigFromFlags("", KUBE_CONFIG_PATH), scale/scale.go:32-40)."""
import base64

import pytest
import yaml

from kube_sqs_autoscaler_amd.kube.config import (
    KubeConfigError, build_config_from_flags, in_cluster_config, load_kubeconfig)


def write_kubeconfig(path, cluster, user, ctx_name="c1"):
    doc = {"apiVersion": "v1", "kind": "Config", "current-context": ctx_name,
           "clusters": [{"name": "k", "cluster": cluster}, {"name": "other", "cluster": {"server": "https://x"}}],
           "users": [{"name": "u", "user": user}],
           "contexts": [{"name": "c1", "context": {"cluster": "k", "user": "u", "namespace": "ignored"}}]}
    path.write_text(yaml.safe_dump(doc))
    return str(path)


def test_in_cluster(tmp_path):
    (tmp_path / "token").write_text("sa-token\n")
    (tmp_path / "ca.crt").write_text("CA PEM")
    rc = in_cluster_config({"KUBERNETES_SERVICE_HOST": "10.0.0.1", "KUBERNETES_SERVICE_PORT": "443"}, str(tmp_path))
    assert rc.host == "https://10.0.0.1:443" and rc.bearer_token == "sa-token" and rc.ca_pem == "CA PEM"
    assert rc.bearer_token_file.endswith("token")  # re-read for bound-token rotation
    rc6 = in_cluster_config({"KUBERNETES_SERVICE_HOST": "fd00::1", "KUBERNETES_SERVICE_PORT": "6443"}, str(tmp_path))
    assert rc6.host == "https://[fd00::1]:6443"


def test_in_cluster_missing_env():
    with pytest.raises(KubeConfigError, match="KUBERNETES_SERVICE_HOST and KUBERNETES_SERVICE_PORT must be defined"):
        in_cluster_config({}, "/nonexistent")


def test_empty_path_without_cluster_fails_like_reference():
    with pytest.raises(KubeConfigError, match="no configuration has been provided"):
        build_config_from_flags("", {}, "/nonexistent")


def test_kubeconfig_token_and_ca_data(tmp_path):
    p = write_kubeconfig(tmp_path / "kc", {"server": "https://api:6443", "certificate-authority-data": base64.b64encode(b"CA").decode(),
                                          "tls-server-name": "kubernetes"}, {"token": "t0"})
    rc = build_config_from_flags(p, {})
    assert (rc.host, rc.bearer_token, rc.ca_pem, rc.server_name) == ("https://api:6443", "t0", "CA", "kubernetes")


def test_kubeconfig_files_relative_to_kubeconfig(tmp_path):
    (tmp_path / "ca.pem").write_text("CAF")
    (tmp_path / "c.pem").write_text("CERT")
    (tmp_path / "k.pem").write_text("KEY")
    (tmp_path / "tok").write_text("ftok\n")
    p = write_kubeconfig(tmp_path / "kc", {"server": "https://api", "certificate-authority": "ca.pem"},
                         {"client-certificate": "c.pem", "client-key": "k.pem", "tokenFile": "tok"})
    rc = load_kubeconfig(p)
    assert (rc.ca_pem, rc.cert_pem, rc.key_pem, rc.bearer_token) == ("CAF", "CERT", "KEY", "ftok")


def test_kubeconfig_insecure_and_basic(tmp_path):
    p = write_kubeconfig(tmp_path / "kc", {"server": "https://api", "insecure-skip-tls-verify": True},
                         {"username": "admin", "password": "pw"})
    rc = load_kubeconfig(p)
    assert rc.insecure and (rc.username, rc.password) == ("admin", "pw")


@pytest.mark.parametrize("cluster,user,match", [
    ({"server": "https://a"}, {"exec": {"command": "aws"}}, "invalid apiVersion"),
    ({}, {"token": "t"}, "no server"),
    ({"server": "https://a"}, {"client-certificate-data": base64.b64encode(b"C").decode()}, "together"),
])
def test_kubeconfig_errors(tmp_path, cluster, user, match):
    p = write_kubeconfig(tmp_path / "kc", cluster, user)
    with pytest.raises(KubeConfigError, match=match):
        load_kubeconfig(p)


def test_kubeconfig_missing_file_and_context(tmp_path):
    with pytest.raises(KubeConfigError):
        load_kubeconfig(str(tmp_path / "none"))
    p = write_kubeconfig(tmp_path / "kc", {"server": "https://a"}, {"token": "t"}, ctx_name="nope")
    with pytest.raises(KubeConfigError, match='context "nope" not found'):
        load_kubeconfig(p)


def test_file_token_provider_rotation(tmp_path, nat):
    f = tmp_path / "token"
    f.write_text("one")
    clock = nat.VirtualClock(0)
    tp = nat.FileTokenProvider(str(f), clock, 60 * nat.SECOND)
    assert tp.token() == "one"
    f.write_text("two")
    assert tp.token() == "one"  # cached within the refresh window
    clock.advance(61 * nat.SECOND)
    assert tp.token() == "two"
    f.unlink()
    clock.advance(61 * nat.SECOND)
    assert tp.token() == "two"  # keeps the last good token if the file vanishes


def test_401_rereads_rotated_token_file(tmp_path, nat):
    """A projected token rotated early is picked up on the next request after the apiserver
    rejects the old one, not only after the periodic re-read (virtual clock: never advances)."""
    from kube_sqs_autoscaler_amd.autoscaler import new_deployment_api
    from kube_sqs_autoscaler_amd.kube.config import RestConfig
    from kube_sqs_autoscaler_amd.utils.log import capture_logger

    f = tmp_path / "token"
    f.write_text("old")
    k = nat.FakeKubeServer()
    k.require_token("new")
    k.start()
    try:
        k.add_deployment("ml", "worker", 1)
        clock = nat.VirtualClock(0)
        api = new_deployment_api(RestConfig(host=k.url, bearer_token_file=str(f)), "ml", "scale", clock=clock)
        p = nat.PodAutoScaler(api, "worker", "ml", 5, 1, 1, 1, capture_logger([]), clock)
        with pytest.raises(nat.NativeError, match="Unauthorized"):
            p.scale_up()  # "old" is read, cached and rejected ...
        f.write_text("new")  # ... the kubelet rotates the file ...
        p.scale_up()  # ... and the 401 made the provider re-read it (the clock never moved)
        assert k.replicas("ml", "worker") == 2
    finally:
        k.stop()


def test_invalidate_only_drops_the_rejected_token(tmp_path, nat):
    f = tmp_path / "token"
    f.write_text("one")
    clock = nat.VirtualClock(0)
    tp = nat.FileTokenProvider(str(f), clock, 60 * nat.SECOND)
    assert tp.token() == "one"
    f.write_text("two")
    tp.invalidate("stale-from-another-request")
    assert tp.token() == "one"  # a different token was rejected: keep the cache
    tp.invalidate("one")
    assert tp.token() == "two"
