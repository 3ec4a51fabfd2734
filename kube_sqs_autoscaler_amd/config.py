"""CLI surface and configuration model.

Reference parity (C1/C2 in SURVEY.md §2.1):

* the 14 flags of /root/reference/main.go:83-97 with the same names, types, help texts and
  defaults -- except ``--max-pods``, which defaults to 8 (one GPU-worker pod per MI355X on an
  8-GPU node; BASELINE.json north_star);
* the attribute-name rule of /root/reference/main.go:103-110: only when ``--attribute-names``
  differs *as a string* from the default is it split on ``,`` and each piece ``TrimSpace``d;
  empty pieces are kept (the reference then panics at /root/reference/sqs/sqs.go:58, this build
  reports an error for that poll instead);
* ``KUBE_CONFIG_PATH`` selects a kubeconfig file, empty means in-cluster
  (/root/reference/scale/scale.go:32-33).

Extensions (all off or reference-equivalent by default):

* ``--queue`` (repeatable): track several queue -> Deployment pairs from one process, one
  independent worker each (BASELINE.json: 1/2/4/8 tracked queues). Each spec is
  ``url=<sqs-url>,deployment=<name>[,namespace=..][,region=..][,<flag>=<value>...]`` where
  ``<flag>`` is any per-target flag below (``attribute-names`` uses ``|`` between names).
* ``--dry-run``: shadow mode next to a running autoscaler -- same polls and decisions, logged
  as ``Dry run: would scale ...``, no writes.
* ``--scale-mode``: ``scale`` (autoscaling/v1 ``/scale`` subresource, default), ``deployment``
  (full-object GET+PUT exactly like the reference), ``patch`` (merge patch with a
  resourceVersion precondition).
* ``--pipeline-reads`` (default on): overlap the Deployment GET with the SQS poll; the write's
  resourceVersion precondition validates the early read and a conflict re-reads once, so the
  decisions are the reference's (``models/oracle.py`` ``prefetch``). The early GET is only sent
  when the previous depth and the cool-downs say a scale call will follow (runner.h
  ``action_likely``), so an idle queue reads the apiserver no more often than the reference.
* ``--worker-processes``: one worker process per tracked queue (parallel/procfleet.py) instead
  of one thread per queue.
* ``--busy-poll-budget`` (default 0): the share of the poll period a queue may spend spinning
  beyond the ``--busy-poll`` window (runner.h ``LoopConfig::spin_budget_ppm``); off because paired
  runs showed no latency gain beyond noise for about 1.5x the CPU per poll (profiles/r05c, r05d).
* ``--poll-presend`` (default off): stage the SQS request during the warm-up (runner.h
  ``LoopConfig::presend``); off because paired A/Bs showed no end-to-end win beyond noise.
* ``--poll-prewarm`` (default 200us): the pre-poll warm-up (runner.h ``LoopConfig::prewarm``):
  the signed SQS request, the bearer token and both connections are ready, and the core awake,
  when the poll is due. The pipelined GET never dials inside the SQS call, so this is also what
  connects the apiserver client before the first pipelined poll.
* ``--sqs-endpoint`` / ``--sqs-protocol``, ``--api-timeout``, ``--log-level`` /
  ``--log-format``, ``--metrics-addr`` (+ ``--readiness-failure-window``), ``--trace-file``,
  ``--gpu-aware-max``.
* ``--leader-elect`` (+ lease name/namespace/identity/timings): Lease-based leader election so
  several replicas can run (the reference must run exactly one, README.md:27).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional

from .utils.goflag import SECOND, FlagError, FlagSet, parse_duration, parse_int

DEFAULT_ATTRIBUTE_NAMES = (
    "ApproximateNumberOfMessages,ApproximateNumberOfMessagesDelayed,ApproximateNumberOfMessagesNotVisible"
)  # /root/reference/main.go:28

REFERENCE_MAX_PODS = 5  # /root/reference/main.go:90
DEFAULT_POLL_PREWARM_NS = 200_000  # --poll-prewarm (runner.h LoopConfig::prewarm)
MI355X_MAX_PODS = 8  # one GPU-worker pod per MI355X of an 8-GPU node

SCALE_MODES = ("scale", "deployment", "patch")
SQS_PROTOCOLS = ("query", "json")


@dataclass
class TargetConfig:
    """One tracked queue and the Deployment it drives (the whole reference process)."""

    queue_url: str = ""
    deployment: str = ""
    namespace: str = "default"
    attribute_names: List[str] = field(default_factory=lambda: DEFAULT_ATTRIBUTE_NAMES.split(","))
    poll_period_ns: int = 5 * SECOND
    scale_down_cool_down_ns: int = 30 * SECOND
    scale_up_cool_down_ns: int = 10 * SECOND
    scale_up_messages: int = 100
    scale_down_messages: int = 10
    scale_up_pods: int = 1
    scale_down_pods: int = 1
    max_pods: int = MI355X_MAX_PODS
    min_pods: int = 1
    region: str = ""  # per-queue AWS region (--queue region=...); "" = --aws-region

    @property
    def name(self) -> str:
        return f"{self.namespace}/{self.deployment}"


@dataclass
class Config:
    targets: List[TargetConfig] = field(default_factory=list)
    aws_region: str = ""
    scale_mode: str = "scale"
    sqs_endpoint: str = ""
    sqs_protocol: str = "query"
    api_timeout_ns: int = 30 * SECOND
    log_level: str = "info"
    log_format: str = "text"
    metrics_addr: str = ""
    gpu_aware_max: str = ""
    gpu_resource: str = "amd.com/gpu"
    gpu_node_selector: str = ""
    gpus_per_pod: int = 1
    gpu_refresh_period_ns: int = 60 * SECOND
    kube_config_path: str = ""
    pipeline_reads: bool = True
    dry_run: bool = False
    worker_threads: int = 0
    worker_processes: bool = False
    busy_poll_ns: int = 25_000
    busy_poll_budget_pct: float = 0.0
    poll_prewarm_ns: int = DEFAULT_POLL_PREWARM_NS
    poll_presend: bool = False
    kube_api_qps: float = 5.0
    kube_api_burst: int = 10
    trace_file: str = ""
    leader_elect: bool = False
    leader_elect_lease_name: str = "kube-sqs-autoscaler"
    leader_elect_namespace: str = ""
    leader_elect_identity: str = ""
    leader_elect_lease_duration_ns: int = 15 * SECOND
    leader_elect_renew_deadline_ns: int = 10 * SECOND
    leader_elect_retry_period_ns: int = 2 * SECOND
    readiness_failure_window_ns: int = 300 * SECOND


# Go's unicode.IsSpace set, which strings.TrimSpace strips: ASCII \t \n \v \f \r and space,
# U+0085 (NEL), U+00A0 (NBSP) and the other White_Space code points. Python's str.strip()
# also strips U+001C..U+001F (and nothing Go keeps would survive it), so it is not used.
GO_SPACE = ("\t\n\v\f\r \u0085\u00a0\u1680\u2000\u2001\u2002\u2003\u2004\u2005\u2006\u2007"
            "\u2008\u2009\u200a\u2028\u2029\u202f\u205f\u3000")


def go_trim_space(s: str) -> str:
    """strings.TrimSpace."""
    return s.strip(GO_SPACE)


def parse_attribute_names(value: str) -> List[str]:
    """/root/reference/main.go:103-110 (string inequality with the default, then split+trim)."""
    if value == DEFAULT_ATTRIBUTE_NAMES:
        return DEFAULT_ATTRIBUTE_NAMES.split(",")
    return [go_trim_space(piece) for piece in value.split(",")]


def new_flag_set(program: str = "kube-sqs-autoscaler") -> FlagSet:
    fs = FlagSet(program=program)
    # /root/reference/main.go:83-97, verbatim help texts
    fs.duration("poll-period", 5 * SECOND, "The interval in seconds for checking if scaling is required")
    fs.duration("scale-down-cool-down", 30 * SECOND, "The cool down period for scaling down")
    fs.duration("scale-up-cool-down", 10 * SECOND, "The cool down period for scaling up")
    fs.int("scale-up-messages", 100, "Number of sqs messages queued up required for scaling up")
    fs.int("scale-down-messages", 10, "Number of messages required to scaling down")
    fs.int("scale-up-pods", 1, "Number of Pod in scaling up")
    fs.int("scale-down-pods", 1, "Number of Pod in scaling down")
    fs.int("max-pods", MI355X_MAX_PODS, "Max pods that kube-sqs-autoscaler can scale")
    fs.int("min-pods", 1, "Min pods that kube-sqs-autoscaler can scale")
    fs.string("aws-region", "", "Your AWS region")
    fs.string(
        "attribute-names",
        DEFAULT_ATTRIBUTE_NAMES,
        "A comma-separated list of queue attribute names to query in calculating the number of messages",
    )
    fs.string("sqs-queue-url", "", "The sqs queue url")
    fs.string("kubernetes-deployment", "", "Kubernetes Deployment to scale. This field is required")
    fs.string("kubernetes-namespace", "default", "The namespace your deployment is running in")
    # ---- extensions ----
    fs.strings(
        "queue",
        "Additional queue to track (repeatable): url=<sqs-url>,deployment=<name>[,namespace=<ns>][,<flag>=<value>...]",
    )
    fs.string("scale-mode", "scale", "How replicas are written: scale (/scale subresource), deployment (GET+PUT of the whole Deployment, like the reference) or patch")
    fs.string("sqs-endpoint", "", "Override the SQS endpoint URL (VPC endpoint, local fake); empty uses the regional endpoint")
    fs.string("sqs-protocol", "query", "SQS wire protocol: query (AWS Query/XML) or json (AWS JSON 1.0)")
    fs.duration("api-timeout", 30 * SECOND, "Per-request timeout for SQS and Kubernetes API calls")
    fs.int("worker-threads", 0, "Threads polling the tracked queues; 0 = one per queue (use fewer for hundreds of queues)")
    fs.bool("worker-processes", False, "Run every tracked queue in a worker process of its own, like one reference process per queue (no per-poll cost shared between queues)")
    fs.bool("dry-run", False, "Shadow mode: poll and decide as usual, log the scaling that would happen, never write")
    fs.bool("pipeline-reads", True, "Send the Deployment GET together with the SQS poll so the two round trips overlap, on polls likely to scale (decisions unchanged; -pipeline-reads=false for strictly sequential calls)")
    fs.float64("kube-api-qps", 5.0, "Client-side limit on kube-apiserver requests per second for each tracked queue, as client-go's default rest client (0 disables)")
    fs.int("kube-api-burst", 10, "Requests allowed in a burst above -kube-api-qps (client-go default)")
    fs.duration("busy-poll", 25_000, "Spin up to this long for an API response before sleeping, only while the peer answers within 4x this (0s disables)")
    fs.float64("busy-poll-budget", 0.0, "Percent of -poll-period the process's queues may spend spinning beyond -busy-poll, split over the queues: to the due time after -poll-prewarm and through a near endpoint's answer (never for an answer slower than 200us; at most a tenth of a cgroup CPU quota); 0 disables")
    fs.duration("poll-prewarm", DEFAULT_POLL_PREWARM_NS, "Before each poll, wake this long early to sign the SQS request, read the token and check (or dial, within 100ms) both connections, then start the poll on time (with -busy-poll-budget, spinning the end of the lead when SQS answers within 200us); decisions are unchanged (0s disables)")
    fs.bool("poll-presend", False, "With -poll-prewarm under 50ms: also hand all but the last bytes of the SQS request to the kernel during the warm-up, corked, so the poll's own write runs warm (nothing reaches the wire early)")
    fs.string("log-level", "info", "Log level: panic, fatal, error, warning, info, debug or trace")
    fs.string("log-format", "text", "Log format: text (logrus TextFormatter) or json")
    fs.string("trace-file", "", "Append one JSON span per poll (depth, decisions, per-call latencies) to this file; empty disables")
    fs.string("metrics-addr", "", "Serve Prometheus metrics and /healthz on host:port (disabled when empty)")
    fs.duration("readiness-failure-window", 300 * SECOND, "/readyz fails while every poll of a tracked queue has failed (to read the queue depth or to write the Deployment) for this long; 0s disables")
    fs.bool("leader-elect", False, "Run several replicas safely: only the holder of a coordination.k8s.io Lease scales")
    fs.string("leader-elect-lease-name", "kube-sqs-autoscaler", "Name of the leader-election Lease")
    fs.string("leader-elect-namespace", "", "Namespace of the leader-election Lease (default: --kubernetes-namespace)")
    fs.string("leader-elect-identity", "", "Holder identity in the Lease (default: $POD_NAME or hostname_pid)")
    fs.duration("leader-elect-lease-duration", 15 * SECOND, "How long a lease is valid without renewal")
    fs.duration("leader-elect-renew-deadline", 10 * SECOND, "How long the leader retries renewing before giving up leadership")
    fs.duration("leader-elect-retry-period", 2 * SECOND, "Interval between lease acquire/renew attempts")
    fs.string("gpu-aware-max", "", "Cap max-pods at GPU capacity: local (GPUs on this node passing the HBM probe) or cluster (allocatable --gpu-resource on selected nodes); empty disables")
    fs.string("gpu-resource", "amd.com/gpu", "Extended resource name of the GPUs (AMD GPU device plugin)")
    fs.string("gpu-node-selector", "", "Label selector of the GPU nodes counted by --gpu-aware-max=cluster")
    fs.int("gpus-per-pod", 1, "GPUs each worker pod requests")
    fs.duration("gpu-refresh-period", 60 * SECOND, "How often --gpu-aware-max=cluster re-reads node capacity")
    return fs


# per-target keys accepted inside --queue specs
_TARGET_INT_KEYS = {
    "scale-up-messages": "scale_up_messages",
    "scale-down-messages": "scale_down_messages",
    "scale-up-pods": "scale_up_pods",
    "scale-down-pods": "scale_down_pods",
    "max-pods": "max_pods",
    "min-pods": "min_pods",
}
_TARGET_DURATION_KEYS = {
    "poll-period": "poll_period_ns",
    "scale-down-cool-down": "scale_down_cool_down_ns",
    "scale-up-cool-down": "scale_up_cool_down_ns",
}


def parse_queue_spec(spec: str, base: TargetConfig) -> TargetConfig:
    """Parses one ``--queue`` value on top of the top-level flags."""
    t = replace(base, attribute_names=list(base.attribute_names))
    seen_url = False
    for item in spec.split(","):
        if not go_trim_space(item):
            continue
        if "=" not in item:
            raise FlagError(f'invalid value "{spec}" for flag -queue: expected key=value, got "{item}"')
        k, v = item.split("=", 1)
        k = go_trim_space(k)
        v = go_trim_space(v)
        try:
            if k in ("url", "sqs-queue-url"):
                t.queue_url = v
                seen_url = True
            elif k in ("deployment", "kubernetes-deployment"):
                t.deployment = v
            elif k in ("namespace", "kubernetes-namespace"):
                t.namespace = v
            elif k in ("region", "aws-region"):
                t.region = v
            elif k == "attribute-names":
                t.attribute_names = parse_attribute_names(v.replace("|", ","))
            elif k in _TARGET_INT_KEYS:
                setattr(t, _TARGET_INT_KEYS[k], parse_int(v))
            elif k in _TARGET_DURATION_KEYS:
                setattr(t, _TARGET_DURATION_KEYS[k], parse_duration(v))
            else:
                raise FlagError(f'invalid value "{spec}" for flag -queue: unknown key "{k}"')
        except ValueError:
            raise FlagError(f'invalid value "{spec}" for flag -queue: parse error')
    if not seen_url:
        raise FlagError(f'invalid value "{spec}" for flag -queue: missing url=')
    return t


def config_from_flags(fs: FlagSet, environ: Optional[Dict[str, str]] = None) -> Config:
    env = os.environ if environ is None else environ
    base = TargetConfig(
        queue_url=fs["sqs-queue-url"],
        deployment=fs["kubernetes-deployment"],
        namespace=fs["kubernetes-namespace"],
        attribute_names=parse_attribute_names(fs["attribute-names"]),
        poll_period_ns=fs["poll-period"],
        scale_down_cool_down_ns=fs["scale-down-cool-down"],
        scale_up_cool_down_ns=fs["scale-up-cool-down"],
        scale_up_messages=fs["scale-up-messages"],
        scale_down_messages=fs["scale-down-messages"],
        scale_up_pods=fs["scale-up-pods"],
        scale_down_pods=fs["scale-down-pods"],
        max_pods=fs["max-pods"],
        min_pods=fs["min-pods"],
    )
    targets: List[TargetConfig] = []
    queue_specs: List[str] = fs["queue"]
    # The single-queue reference form is always honoured when --sqs-queue-url is given or no
    # --queue is used (the reference accepts an empty URL and fails on every poll instead).
    if fs.was_set("sqs-queue-url") or not queue_specs:
        targets.append(base)
    for spec in queue_specs:
        targets.append(parse_queue_spec(spec, base))
    cfg = Config(
        targets=targets,
        aws_region=fs["aws-region"],
        scale_mode=fs["scale-mode"],
        sqs_endpoint=fs["sqs-endpoint"],
        sqs_protocol=fs["sqs-protocol"],
        api_timeout_ns=fs["api-timeout"],
        log_level=fs["log-level"],
        log_format=fs["log-format"],
        metrics_addr=fs["metrics-addr"],
        gpu_aware_max=fs["gpu-aware-max"],
        gpu_resource=fs["gpu-resource"],
        gpu_node_selector=fs["gpu-node-selector"],
        gpus_per_pod=fs["gpus-per-pod"],
        gpu_refresh_period_ns=fs["gpu-refresh-period"],
        kube_config_path=env.get("KUBE_CONFIG_PATH", ""),
        pipeline_reads=fs["pipeline-reads"],
        dry_run=fs["dry-run"],
        worker_threads=fs["worker-threads"],
        worker_processes=fs["worker-processes"],
        busy_poll_ns=fs["busy-poll"],
        busy_poll_budget_pct=fs["busy-poll-budget"],
        poll_prewarm_ns=fs["poll-prewarm"],
        poll_presend=fs["poll-presend"],
        kube_api_qps=fs["kube-api-qps"],
        kube_api_burst=fs["kube-api-burst"],
        trace_file=fs["trace-file"],
        leader_elect=fs["leader-elect"],
        leader_elect_lease_name=fs["leader-elect-lease-name"],
        leader_elect_namespace=fs["leader-elect-namespace"] or fs["kubernetes-namespace"],
        leader_elect_identity=fs["leader-elect-identity"],
        leader_elect_lease_duration_ns=fs["leader-elect-lease-duration"],
        leader_elect_renew_deadline_ns=fs["leader-elect-renew-deadline"],
        leader_elect_retry_period_ns=fs["leader-elect-retry-period"],
        readiness_failure_window_ns=fs["readiness-failure-window"],
    )
    if cfg.scale_mode not in SCALE_MODES:
        raise FlagError(f'invalid value "{cfg.scale_mode}" for flag -scale-mode: must be one of {", ".join(SCALE_MODES)}')
    if cfg.sqs_protocol not in SQS_PROTOCOLS:
        raise FlagError(f'invalid value "{cfg.sqs_protocol}" for flag -sqs-protocol: must be query or json')
    if cfg.metrics_addr:
        host, sep, port = cfg.metrics_addr.rpartition(":")
        if not sep or not port.isdigit() or int(port) > 65535 or (":" in host and not host.startswith("[")):
            raise FlagError(f'invalid value "{cfg.metrics_addr}" for flag -metrics-addr: want host:port, :port or [ipv6]:port')
    if cfg.log_format not in ("text", "json"):
        raise FlagError(f'invalid value "{cfg.log_format}" for flag -log-format: must be text or json')
    if cfg.leader_elect and not (cfg.leader_elect_lease_duration_ns > cfg.leader_elect_renew_deadline_ns
                                 > cfg.leader_elect_retry_period_ns > 0):
        raise FlagError("leader election needs lease-duration > renew-deadline > retry-period > 0")
    if cfg.gpu_aware_max not in ("", "local", "cluster"):
        raise FlagError(f'invalid value "{cfg.gpu_aware_max}" for flag -gpu-aware-max: must be empty, local or cluster')
    if cfg.worker_processes and cfg.worker_threads > 0:
        raise FlagError("-worker-processes and -worker-threads cannot be combined")
    if not 0.0 <= cfg.busy_poll_budget_pct <= 100.0:
        raise FlagError(f'invalid value "{cfg.busy_poll_budget_pct:g}" for flag -busy-poll-budget: must be between 0 and 100')
    if cfg.poll_prewarm_ns < 0:
        raise FlagError(f'invalid value "{cfg.poll_prewarm_ns}ns" for flag -poll-prewarm: must not be negative')
    if cfg.gpus_per_pod < 1:
        raise FlagError(f'invalid value "{cfg.gpus_per_pod}" for flag -gpus-per-pod: must be >= 1')
    return cfg


def parse_args(argv: List[str], environ: Optional[Dict[str, str]] = None) -> Config:
    fs = new_flag_set()
    fs.parse(argv)
    return config_from_flags(fs, environ)
