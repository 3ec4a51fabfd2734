"""Component factories: configuration -> native control-loop objects.

These are the constructors of the reference, rebuilt over the native runtime:

* :func:`new_pod_autoscaler` -- ``scale.NewPodAutoScaler`` (/root/reference/scale/scale.go:31-52):
  kube config from ``KUBE_CONFIG_PATH`` (in-cluster when empty), a REST client scoped to the
  namespace, and the clamp parameters.
* :func:`new_sqs_client` -- ``kubesqs.NewSqsClient`` (/root/reference/sqs/sqs.go:35-43): a
  SigV4-signing SQS client for ``region`` over a persistent HTTPS connection, plus the
  attribute list to sum.
* :func:`new_runner` -- the state ``Run`` keeps (/root/reference/main.go:35-38): one
  independent loop per tracked queue, with its own clients and timers.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Mapping, Optional

from .config import Config, TargetConfig
from .kube.config import RestConfig, build_config_from_flags
from .ops import native
from .sqs.credentials import make_chain_provider
from .sqs.session import custom_ca_bundle
from .utils import proxy
from .utils.goflag import SECOND

ONE_PERCENT_PPM = 10_000  # LoopConfig.spin_budget_ppm for 1 % of the poll period
DEFAULT_SPIN_BUDGET_PPM = 0  # --busy-poll-budget's default (0 %): the --busy-poll window only


def spin_budget_ppm(budget_pct: float, queues: int = 1) -> int:
    """LoopConfig.spin_budget_ppm of one of ``queues`` queues sharing ``--busy-poll-budget``."""
    return int(round(budget_pct * ONE_PERCENT_PPM)) // max(queues, 1)

_SCALE_MODES = {"deployment": "Deployment", "scale": "Scale", "patch": "Patch"}


def scale_mode(name: str):
    return getattr(native().ScaleMode, _SCALE_MODES[name])


def tls_options(rc: RestConfig):
    nat = native()
    t = nat.TlsOptions()
    t.insecure_skip_verify = rc.insecure
    t.ca_pem = rc.ca_pem
    t.cert_pem = rc.cert_pem
    t.key_pem = rc.key_pem
    t.server_name = rc.server_name
    return t


def kube_proxy(rc: RestConfig, environ: Optional[Mapping[str, str]] = None) -> str:
    """client-go: the kubeconfig ``proxy-url``, else ``http.ProxyFromEnvironment``."""
    return proxy.select(rc.host, environ, rc.proxy_url)


class KubeClientError(RuntimeError):
    """``kubernetes.NewForConfig`` failed (the reference panics "Failed to configure client",
    /root/reference/scale/scale.go:38-40)."""


def exec_config(rc: RestConfig, timeout_ns: int = 0):
    nat = native()
    e = nat.ExecConfig()
    p = rc.exec_plugin
    e.command, e.args, e.env = p.command, list(p.args), list(p.env)
    e.api_version, e.install_hint, e.timeout_ns = p.api_version, p.install_hint, timeout_ns
    return e


def token_provider(rc: RestConfig, clock=None, timeout_ns: int = 0):
    """The bearer-token source for ``rc`` (None: no bearer auth).

    A static ``token`` wins over everything (client-go skips the exec plugin when the config
    already carries a token); a ``tokenFile`` / in-cluster SA token is re-read every 60 s; an
    ``exec`` plugin is run natively and its credential cached until it expires or a 401 comes
    back. The exec provider is shared by every client built from ``rc``, so N tracked queues
    run the plugin once, not N times.
    """
    nat = native()
    if rc.bearer_token_file:
        return nat.FileTokenProvider(rc.bearer_token_file, clock or nat.RealClock(), 60 * SECOND)
    if rc.bearer_token:
        return nat.StaticTokenProvider(rc.bearer_token)
    if rc.exec_plugin is not None:
        p = rc.shared.get("exec")
        if p is None:
            p = rc.shared["exec"] = nat.ExecTokenProvider(exec_config(rc, timeout_ns), clock or nat.RealClock())
        return p
    return None


def prepare_kube_auth(rc: RestConfig, clock=None, timeout_ns: int = 0) -> Optional[str]:
    """Client construction checks (``kubernetes.NewForConfig``, scale.go:38).

    Raises :class:`KubeClientError` for an ``auth-provider`` user (the reference links no
    auth-provider plugins). For an ``exec`` plugin that hands out client certificates, runs it
    once so the certificate is in the TLS config before the first connection; a plugin failure
    here is returned as a warning and retried on the first request, where client-go would run
    it.
    """
    if rc.auth_provider and not rc.bearer_token and not rc.bearer_token_file:
        raise KubeClientError(f'no Auth Provider found for name "{rc.auth_provider}"')
    if rc.exec_plugin is None or rc.bearer_token or rc.bearer_token_file or rc.cert_pem:
        return None
    p = token_provider(rc, clock, timeout_ns)
    try:
        cred = p.credential()
    except native().NativeError as e:
        return f"exec credential plugin: {e}"
    if cred.cert_pem:
        rc.cert_pem, rc.key_pem = cred.cert_pem, cred.key_pem
    return None


def auth_headers(rc: RestConfig) -> list:
    """Authorization header for ad-hoc apiserver calls (Leases, Nodes), from the same sources
    as the actuator's requests."""
    p = token_provider(rc)
    if p is not None:
        t = p.token()
        return [("Authorization", f"Bearer {t}")] if t else []
    if rc.username:
        import base64

        return [("Authorization", "Basic " + base64.b64encode(f"{rc.username}:{rc.password}".encode()).decode())]
    return []


def note_status(rc: RestConfig, headers: list, status: int) -> None:
    """A 401 on a bearer token drops it from the cache so the next call fetches a fresh one."""
    if status != 401:
        return
    p = token_provider(rc)
    for k, v in headers:
        if p is not None and k == "Authorization" and v.startswith("Bearer "):
            p.invalidate(v[7:])


def new_http_client(rc: RestConfig, timeout_ns: int, environ: Optional[Mapping[str, str]] = None):
    """A native keep-alive client to the apiserver (leader election, node listing)."""
    c = native().HttpClient(rc.host, tls_options(rc), timeout_ns)
    c.set_proxy(kube_proxy(rc, environ))
    return c


def new_deployment_api(rc: RestConfig, namespace: str, mode: str = "scale", timeout_ns: int = 30 * SECOND, clock=None,
                       busy_poll_ns: int = 0, environ: Optional[Mapping[str, str]] = None, qps: float = 0.0,
                       burst: int = 0, logger=None, rbac_fallback: bool = True):
    """The ``DeploymentInterface`` seam over REST (/root/reference/scale/scale.go:44).

    ``qps``/``burst``: the client-side throttle of this client (client-go's clientset default is
    5/10, which the CLI passes; 0 leaves it unthrottled). ``rbac_fallback``: in ``scale``/``patch``
    mode, switch to the reference's whole-Deployment GET+PUT when the apiserver refuses the
    ``/scale`` subresource (a Role written for the reference), warning once on ``logger``."""
    nat = native()
    o = nat.KubeOptions()
    o.server = rc.host
    o.proxy = kube_proxy(rc, environ)
    o.namespace = namespace
    o.mode = scale_mode(mode)
    o.tls = tls_options(rc)
    o.timeout_ns = timeout_ns
    o.busy_poll_ns = busy_poll_ns
    if clock is not None:
        o.clock = clock  # throttle waits and Retry-After sleeps
    if qps > 0:
        o.qps, o.burst = float(qps), int(burst)
        o.clock = clock or nat.RealClock()
    tp = token_provider(rc, clock, timeout_ns)
    if tp is not None:
        o.token = tp
    o.basic_user = rc.username
    o.basic_password = rc.password
    o.rbac_fallback = rbac_fallback
    if logger is not None:
        o.log = logger
    return nat.KubeRestDeployments(o)


def new_pod_autoscaler(target: TargetConfig, api, logger, clock):
    nat = native()
    return nat.PodAutoScaler(api, target.deployment, target.namespace, target.max_pods, target.min_pods,
                             target.scale_up_pods, target.scale_down_pods, logger, clock)


def new_sqs_api(region: str, clock, endpoint: str = "", protocol: str = "query", timeout_ns: int = 30 * SECOND,
                credentials=None, environ: Optional[Mapping[str, str]] = None, tls=None, busy_poll_ns: int = 0,
                retry_delays_ns: Optional[tuple] = None):
    """``retry_delays_ns``: (min, min for throttles) back-off bases; default aws-sdk-go v1's
    DefaultRetryer (30 ms / 500 ms). Tests shorten them."""
    nat = native()
    o = nat.SqsHttpOptions()
    if retry_delays_ns is not None:
        o.min_retry_delay_ns, o.min_throttle_delay_ns = retry_delays_ns
    o.region = region
    o.endpoint = endpoint
    o.protocol = nat.SqsProtocol.Json if protocol == "json" else nat.SqsProtocol.Query
    o.timeout_ns = timeout_ns
    o.busy_poll_ns = busy_poll_ns
    env = os.environ if environ is None else environ
    # aws-sdk-go's default client: http.ProxyFromEnvironment on the resolved endpoint
    o.proxy = proxy.select(endpoint or nat.HttpSqsApi.endpoint_for_region(region), env)
    if tls is not None:
        o.tls = tls
    elif custom_ca_bundle(env):  # aws-sdk-go v1 session: custom CA bundle for AWS endpoints
        t = nat.TlsOptions()
        t.ca_file = custom_ca_bundle(env)
        o.tls = t
    creds = credentials if credentials is not None else make_chain_provider(environ=environ, region=region)
    return nat.HttpSqsApi(o, creds, clock)


def shared_sqs_credentials(cache: dict, region: str, clock, environ: Optional[Mapping[str, str]] = None):
    """The process's credential source for SQS clients of ``region`` (the STS region of a web
    identity / assume-role chain follows it): one ``SharedCredentialsProvider`` per distinct
    chain configuration, kept in ``cache``, so N tracked queues make one credential fetch per
    expiry instead of N -- as the reference's one session per process (sqs/sqs.go:36). Each
    client still keeps its own copy and refreshes it in its pre-poll warm-up, off the poll."""
    p = cache.get(region)
    if p is None:
        p = cache[region] = native().SharedCredentialsProvider(make_chain_provider(environ=environ, region=region),
                                                               clock)
    return p


def new_sqs_client(target: TargetConfig, api):
    return native().SqsClient(api, target.queue_url, list(target.attribute_names))


def loop_config(target: TargetConfig, pipeline_reads: bool = False, prewarm_ns: int = 0, queues: int = 1,
                presend: bool = False, spin_budget_pct: float = 0.0):
    c = native().LoopConfig()
    c.presend = presend
    # the process's queues share --busy-poll-budget of their poll period (runner.h)
    c.spin_budget_ppm = spin_budget_ppm(spin_budget_pct, queues)
    c.prefetch = pipeline_reads
    c.prewarm_ns = prewarm_ns
    c.poll_period_ns = target.poll_period_ns
    c.scale_down_cool_down_ns = target.scale_down_cool_down_ns
    c.scale_up_cool_down_ns = target.scale_up_cool_down_ns
    c.scale_up_messages = target.scale_up_messages
    c.scale_down_messages = target.scale_down_messages
    return c


@dataclass
class Worker:
    target: TargetConfig
    runner: object
    sqs_api: object
    kube_api: object
    logger: object


def new_runner(target: TargetConfig, cfg: Config, rest: RestConfig, base_logger, clock,
               credentials=None, environ: Optional[Mapping[str, str]] = None, tag_queue: bool = False,
               credentials_cache: Optional[dict] = None) -> Worker:
    """``credentials_cache``: share one credential source per region between the process's
    workers (:func:`shared_sqs_credentials`); None with no ``credentials``: a chain of its own."""
    nat = native()
    log = base_logger
    if tag_queue:
        log = base_logger.with_fields([("deployment", target.name), ("queue", target.queue_url)])
    kube_api = new_deployment_api(rest, target.namespace, cfg.scale_mode, cfg.api_timeout_ns, clock,
                                  busy_poll_ns=cfg.busy_poll_ns, environ=environ, qps=cfg.kube_api_qps,
                                  burst=cfg.kube_api_burst, logger=log)
    scaler = new_pod_autoscaler(target, kube_api, log, clock)
    scaler.dry_run = cfg.dry_run
    region = target.region or cfg.aws_region
    if credentials is None and credentials_cache is not None:
        credentials = shared_sqs_credentials(credentials_cache, region, clock, environ)
    sqs_api = new_sqs_api(region, clock, cfg.sqs_endpoint, cfg.sqs_protocol, cfg.api_timeout_ns,
                          credentials, environ, busy_poll_ns=cfg.busy_poll_ns)
    sqs = new_sqs_client(target, sqs_api)
    runner = nat.Runner(loop_config(target, cfg.pipeline_reads, cfg.poll_prewarm_ns, len(cfg.targets), cfg.poll_presend,
                                    cfg.busy_poll_budget_pct), sqs, scaler, clock, log)
    return Worker(target, runner, sqs_api, kube_api, log)


def load_rest_config(cfg: Config, environ: Optional[Mapping[str, str]] = None, klog=None) -> RestConfig:
    return build_config_from_flags(cfg.kube_config_path, environ, klog=klog)
