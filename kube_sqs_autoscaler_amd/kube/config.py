"""Kubernetes client configuration: in-cluster service account or a kubeconfig file.

Mirrors ``clientcmd.BuildConfigFromFlags("", os.Getenv("KUBE_CONFIG_PATH"))``
(/root/reference/scale/scale.go:32-33, client-go v0.19.4, go.mod:17):

* path empty -> in-cluster config (``KUBERNETES_SERVICE_HOST``/``_PORT``, the projected SA
  token and CA under ``/var/run/secrets/kubernetes.io/serviceaccount``); if that fails, the
  empty explicit-path loading rules yield "no configuration has been provided";
* path set -> that kubeconfig only (``KUBECONFIG`` is *not* consulted, matching the
  reference's ``ExplicitPath`` loading rules): current-context -> cluster + user.

Supported kubeconfig auth: bearer ``token`` / ``tokenFile``, client certificates (file or
``-data``), basic auth, and ``exec`` credential plugins (``client.authentication.k8s.io``
v1alpha1/v1beta1, e.g. ``aws eks get-token``; run natively by ``ExecTokenProvider``,
``csrc/core/exec_auth.cc``); TLS via ``certificate-authority[-data]``,
``insecure-skip-tls-verify``, ``tls-server-name``. The reference turns any failure here into
``panic("Failed to configure incluster or local config")`` (scale.go:35); the CLI keeps that
text and exits non-zero. An ``auth-provider`` user loads here but, as in the reference (which
imports no ``client-go/plugin/pkg/client/auth`` provider), fails when the client is built:
``panic("Failed to configure client")`` (scale.go:40).
"""
from __future__ import annotations

import base64
import os
from dataclasses import dataclass, field
from typing import Mapping, Optional

import yaml

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class KubeConfigError(RuntimeError):
    pass


@dataclass
class RestConfig:
    host: str
    bearer_token: str = ""
    bearer_token_file: str = ""
    username: str = ""
    password: str = ""
    ca_pem: str = ""
    ca_file: str = ""
    cert_pem: str = ""
    key_pem: str = ""
    insecure: bool = False
    server_name: str = ""
    proxy_url: str = ""  # kubeconfig cluster proxy-url (client-go v0.19); "" = environment
    exec_plugin: Optional["ExecPlugin"] = None
    auth_provider: str = ""  # kubeconfig auth-provider name (unsupported, like the reference)
    source: str = ""
    # shared per-config state (the exec authenticator), like client-go's authenticator cache
    shared: dict = field(default_factory=dict, repr=False, compare=False)


EXEC_API_VERSIONS = ("client.authentication.k8s.io/v1alpha1", "client.authentication.k8s.io/v1beta1")


@dataclass
class ExecPlugin:
    """A kubeconfig ``users[].user.exec`` stanza (client-go v0.19 ``api.ExecConfig``)."""

    command: str
    args: list = field(default_factory=list)
    env: list = field(default_factory=list)  # [(name, value)], applied over the process env
    api_version: str = ""
    install_hint: str = ""


def _exec_plugin(spec: dict, base_dir: str) -> ExecPlugin:
    if not isinstance(spec, dict):
        raise KubeConfigError("invalid configuration: exec must be a mapping")
    cmd = str(spec.get("command") or "")
    # clientcmd resolves a command with a path separator relative to the kubeconfig file;
    # a bare name is looked up on PATH at run time.
    if "/" in cmd and not os.path.isabs(cmd):
        cmd = os.path.join(base_dir, cmd)
    env = []
    for e in spec.get("env") or []:
        if not isinstance(e, dict) or "name" not in e:
            raise KubeConfigError("invalid configuration: exec env entries need a name")
        env.append((str(e["name"]), str(e.get("value", ""))))
    p = ExecPlugin(command=cmd, args=[str(a) for a in spec.get("args") or []], env=env,
                   api_version=str(spec.get("apiVersion") or ""), install_hint=str(spec.get("installHint") or ""))
    if p.api_version not in EXEC_API_VERSIONS:
        raise KubeConfigError(f'exec plugin: invalid apiVersion "{p.api_version}"')
    if not p.command:
        raise KubeConfigError("invalid configuration: exec plugin command must be specified")
    return p


def in_cluster_config(environ: Optional[Mapping[str, str]] = None, sa_dir: str = SA_DIR) -> RestConfig:
    env = os.environ if environ is None else environ
    host, port = env.get("KUBERNETES_SERVICE_HOST", ""), env.get("KUBERNETES_SERVICE_PORT", "")
    if not host or not port:
        raise KubeConfigError(
            "unable to load in-cluster configuration, KUBERNETES_SERVICE_HOST and KUBERNETES_SERVICE_PORT must be defined")
    token_file = os.path.join(sa_dir, "token")
    try:
        with open(token_file) as f:
            token = f.read().strip()
    except OSError as e:
        raise KubeConfigError(f"open {token_file}: {e.strerror.lower() if e.strerror else e}")
    ca_file = os.path.join(sa_dir, "ca.crt")
    ca_pem = ""
    if os.path.exists(ca_file):
        with open(ca_file) as f:
            ca_pem = f.read()
    h = f"[{host}]" if ":" in host and not host.startswith("[") else host
    return RestConfig(host=f"https://{h}:{port}", bearer_token=token, bearer_token_file=token_file,
                      ca_pem=ca_pem, ca_file=ca_file if ca_pem else "", source="in-cluster")


def _b64(s: str) -> str:
    return base64.b64decode(s).decode()


def _read_rel(base_dir: str, path: str) -> str:
    p = path if os.path.isabs(path) else os.path.join(base_dir, path)
    with open(p) as f:
        return f.read()


def load_kubeconfig(path: str, context: str = "") -> RestConfig:
    try:
        with open(path) as f:
            doc = yaml.safe_load(f) or {}
    except OSError as e:
        raise KubeConfigError(f"stat {path}: no such file or directory" if not os.path.exists(path) else str(e))
    except yaml.YAMLError as e:
        raise KubeConfigError(f"error loading config file \"{path}\": {e}")
    base = os.path.dirname(os.path.abspath(path))

    def by_name(kind: str, name: str) -> dict:
        for item in doc.get(kind) or []:
            if item.get("name") == name:
                return item.get(kind[:-1]) or {}
        raise KubeConfigError(f'invalid configuration: {kind[:-1]} "{name}" not found')

    ctx_name = context or doc.get("current-context") or ""
    if not ctx_name:
        raise KubeConfigError("invalid configuration: no configuration has been provided, try setting KUBERNETES_MASTER environment variable")
    ctx = by_name("contexts", ctx_name)
    cluster = by_name("clusters", ctx.get("cluster", ""))
    user = by_name("users", ctx.get("user", "")) if ctx.get("user") else {}
    server = cluster.get("server", "")
    if not server:
        raise KubeConfigError("invalid configuration: no server found for cluster")
    rc = RestConfig(host=server, source=f"kubeconfig:{path}")
    rc.insecure = bool(cluster.get("insecure-skip-tls-verify", False))
    rc.server_name = cluster.get("tls-server-name", "")
    rc.proxy_url = cluster.get("proxy-url", "") or ""
    try:
        if cluster.get("certificate-authority-data"):
            rc.ca_pem = _b64(cluster["certificate-authority-data"])
        elif cluster.get("certificate-authority"):
            rc.ca_pem = _read_rel(base, cluster["certificate-authority"])
        if user.get("client-certificate-data"):
            rc.cert_pem = _b64(user["client-certificate-data"])
        elif user.get("client-certificate"):
            rc.cert_pem = _read_rel(base, user["client-certificate"])
        if user.get("client-key-data"):
            rc.key_pem = _b64(user["client-key-data"])
        elif user.get("client-key"):
            rc.key_pem = _read_rel(base, user["client-key"])
        if user.get("token"):
            rc.bearer_token = user["token"]
        elif user.get("tokenFile"):
            tf = user["tokenFile"]
            rc.bearer_token_file = tf if os.path.isabs(tf) else os.path.join(base, tf)
            rc.bearer_token = _read_rel(base, tf).strip()
    except OSError as e:
        raise KubeConfigError(f"unable to read referenced file: {e}")
    except (ValueError, TypeError) as e:
        raise KubeConfigError(f"illegal base64 data in kubeconfig: {e}")
    rc.username = user.get("username", "")
    rc.password = user.get("password", "")
    if user.get("exec"):
        rc.exec_plugin = _exec_plugin(user["exec"], base)
    if user.get("auth-provider"):
        if rc.exec_plugin is not None:
            raise KubeConfigError("invalid configuration: authProvider cannot be provided in combination with an exec plugin")
        rc.auth_provider = str((user["auth-provider"] or {}).get("name", ""))
    if bool(rc.cert_pem) != bool(rc.key_pem):
        raise KubeConfigError("invalid configuration: client-cert and client-key must be specified together")
    return rc


def build_config_from_flags(kube_config_path: str, environ: Optional[Mapping[str, str]] = None,
                            sa_dir: str = SA_DIR, klog=None) -> RestConfig:
    """clientcmd.BuildConfigFromFlags("", kube_config_path).

    Without a path client-go warns through klog before trying the in-cluster config, and again
    when that fails and it falls back to the default loading rules, which -- with no explicit
    path -- find nothing ("no configuration has been provided"). ``klog``: a utils/klog.Klog
    for those two lines (None: not written)."""
    from ..utils import klog as k

    if not kube_config_path:
        if klog is not None:
            klog.warning("Neither --kubeconfig nor --master was specified.  Using the inClusterConfig.  This might not work.",
                         k.CLIENT_CONFIG_GO, k.NEITHER_LINE)
        try:
            return in_cluster_config(environ, sa_dir)
        except KubeConfigError as e:
            if klog is not None:
                klog.warning(f"error creating inClusterConfig, falling back to default config: {e}",
                             k.CLIENT_CONFIG_GO, k.FALLBACK_LINE)
            raise KubeConfigError(
                "invalid configuration: no configuration has been provided, try setting KUBERNETES_MASTER environment variable")
    return load_kubeconfig(kube_config_path)
