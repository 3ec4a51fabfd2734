"""Process entry point: ``python -m kube_sqs_autoscaler_amd [flags]`` (the reference's ``main``).

/root/reference/main.go:82-116: parse flags -> ``NewPodAutoScaler`` (panics when no kube config
can be built, scale.go:35) -> attribute list -> ``NewSqsClient`` (panics when the AWS session's
configuration is invalid, ``session.Must``, sqs.go:36; sqs/session.py) -> log
``Starting kube-sqs-autoscaler`` -> ``Run`` forever. Exit codes follow Go: 2 for a flag error
(after printing the message and usage), 0 for ``-h``/``-help``, 2 for a start-up panic.
Extensions: several ``--queue`` targets, SIGTERM/SIGINT graceful stop (exit 0), optional
Prometheus endpoint and GPU-aware ``max-pods`` cap.
"""
from __future__ import annotations

import os
import signal
import sys
import threading
from typing import List, Mapping, Optional

from . import autoscaler
from .config import MI355X_MAX_PODS, REFERENCE_MAX_PODS, config_from_flags, new_flag_set
from .kube.config import KubeConfigError
from .sqs.session import SessionError, validate_session
from .utils.goflag import FlagError
from .utils.log import make_logger


def _program_name(argv0: str) -> str:
    base = os.path.basename(argv0 or "")
    return "kube-sqs-autoscaler" if base in ("", "__main__.py", "-c", "-m") else argv0


def _panic(msg: str, cause: str = "") -> int:
    # Go prints "panic: <msg>" plus the goroutine trace and exits with status 2.
    sys.stderr.write(f"panic: {msg}\n")
    if cause:
        sys.stderr.write(f"\ncause: {cause}\n")
    sys.stderr.flush()
    return 2


def main(argv: Optional[List[str]] = None, environ: Optional[Mapping[str, str]] = None,
         max_iterations: int = -1) -> int:
    argv = sys.argv[1:] if argv is None else argv
    env = os.environ if environ is None else environ
    fs = new_flag_set(_program_name(sys.argv[0] if sys.argv else ""))
    try:
        fs.parse(argv)
        cfg = config_from_flags(fs, env)
    except FlagError as e:
        if e.help:
            fs.print_usage(sys.stderr)
            return 0
        sys.stderr.write(f"{e}\n")
        fs.print_usage(sys.stderr)
        return 2

    from .ops import native

    nat = native()
    clock = nat.RealClock()
    log = make_logger(cfg.log_level, cfg.log_format, clock=None)

    # scale.NewPodAutoScaler -> clientcmd.BuildConfigFromFlags("", KUBE_CONFIG_PATH); client-go's
    # own warnings there are klog lines, as the reference's are (utils/klog.py)
    from .utils.klog import Klog

    try:
        rest = autoscaler.load_rest_config(cfg, env, klog=Klog())
    except KubeConfigError as e:
        return _panic("Failed to configure incluster or local config", str(e))
    try:
        w = autoscaler.prepare_kube_auth(rest, clock, cfg.api_timeout_ns)
    except autoscaler.KubeClientError as e:
        return _panic("Failed to configure client", str(e))
    if w:
        log.log("warning", w)
    # kubesqs.NewSqsClient -> sqs.New(session.Must(session.NewSession()), ...) (sqs/sqs.go:36):
    # the session's configuration is checked now; credentials are still fetched on first use.
    try:
        for w in validate_session(env):
            log.log("warning", f"AWS shared config: {w}")
    except SessionError as e:
        return _panic(str(e))

    if not fs.was_set("max-pods"):
        # the one default that differs from the reference (main.go:90: 5)
        log.log("warning", f"--max-pods not set: using {MI355X_MAX_PODS} (one GPU-worker pod per MI355X of an "
                           f"8-GPU node); the reference defaults to {REFERENCE_MAX_PODS}")

    multi = len(cfg.targets) > 1
    trace_fd = -1
    if cfg.trace_file:
        trace_fd = os.open(cfg.trace_file, os.O_WRONLY | os.O_CREAT | os.O_APPEND | os.O_CLOEXEC, 0o644)

    # One AWS credential source per region for the process's queues: a broker thread per region
    # runs the chain ahead of expiry and publishes each set into shared memory, where every queue reads it
    # (parallel/credbroker.py) -- worker threads here, or worker processes, which inherit the
    # mapping. No queue's poll or warm-up runs a fetch, one region's hung endpoint never delays
    # another's (a thread per region), a refresh that fails keeps the set while it still signs,
    # and a stop never waits for a fetch.
    from .parallel.credbroker import CredentialBroker

    broker = CredentialBroker({t.region or cfg.aws_region for t in cfg.targets}, env,
                              log=lambda lvl, m: log.log(lvl, m))
    if cfg.worker_processes:
        # fork the workers first: before this process starts threads or touches the GPU
        from .parallel.procfleet import ProcessFleet

        def build(t):
            def make():
                w = autoscaler.new_runner(t, cfg, rest, log, clock, environ=env, tag_queue=multi,
                                          credentials=broker.provider_for(t.region or cfg.aws_region))
                if trace_fd >= 0:
                    w.runner.set_trace_fd(trace_fd)
                return w
            return make

        fleet = ProcessFleet([build(t) for t in cfg.targets], cfg.targets)
        workers = fleet.workers
    else:
        workers = [autoscaler.new_runner(t, cfg, rest, log, clock, environ=env, tag_queue=multi,
                                         credentials=broker.provider_for(t.region or cfg.aws_region))
                   for t in cfg.targets]
        if trace_fd >= 0:
            for w in workers:
                w.runner.set_trace_fd(trace_fd)
        from .parallel.fleet import Fleet

        fleet = Fleet(workers, cfg.worker_threads)

    capper = None
    if cfg.gpu_aware_max:
        from .kube.gpus import ClusterGpuCapacity, MaxPodsCapper

        if cfg.gpu_aware_max == "local":
            from .ops import gpu

            def capacity() -> int:
                return gpu.healthy_gpu_count() // cfg.gpus_per_pod
        else:
            capacity = ClusterGpuCapacity(rest, cfg.gpu_resource, cfg.gpu_node_selector, cfg.gpus_per_pod).pod_capacity
        capper = MaxPodsCapper([w.runner.scaler for w in workers], [t.max_pods for t in cfg.targets], capacity,
                               cfg.gpu_refresh_period_ns / 1e9, log=lambda lvl, m: log.log(lvl, m),
                               min_pods=[t.min_pods for t in cfg.targets])
        capper.refresh()
        if cfg.gpu_aware_max == "cluster":
            capper.start()

    metrics = None
    health = None
    if cfg.metrics_addr:
        from .metrics import Health, MetricsServer

        health = Health(fleet, [Health.budget_ns(t.poll_period_ns, cfg.api_timeout_ns) for t in cfg.targets],
                        leader_elect=cfg.leader_elect, failure_window_ns=cfg.readiness_failure_window_ns)
        metrics = MetricsServer(fleet, cfg.metrics_addr, health, lambda: dict(broker.fetches_by_region),
                                broker.stale_signs_by_region)
        metrics.start()
        log.log("info", f"Serving metrics on {cfg.metrics_addr}")

    # Signals: stop whatever phase we are in (election wait, control loop) and exit 0.
    stop = threading.Event()
    got: List[int] = []

    def on_signal(signum, _frame):
        got.append(signum)
        log.log("info", f"Received signal {signum}, stopping")
        stop.set()
        fleet.stop()

    prev = {}
    if threading.current_thread() is threading.main_thread():
        for sig in (signal.SIGTERM, signal.SIGINT):
            prev[sig] = signal.signal(sig, on_signal)

    elector = None
    lost = threading.Event()
    renew_stop = threading.Event()
    renewer = None
    try:
        if cfg.leader_elect:
            from .kube.leader import LeaderElector, LeaseLock, default_identity

            lock = LeaseLock(rest, cfg.leader_elect_namespace, cfg.leader_elect_lease_name)
            elector = LeaderElector(lock, cfg.leader_elect_identity or default_identity(),
                                    cfg.leader_elect_lease_duration_ns / 1e9, cfg.leader_elect_renew_deadline_ns / 1e9,
                                    cfg.leader_elect_retry_period_ns / 1e9, log=lambda lvl, m: log.log(lvl, m))
            if not elector.acquire(stop):
                return 0

            def on_lost():
                lost.set()
                fleet.stop()

            renewer = threading.Thread(target=elector.renew_loop, args=(renew_stop, on_lost), name="ksa-lease", daemon=True)
            renewer.start()
            if health is not None:
                health.set_role("leader")

        log.log("info", "Starting kube-sqs-autoscaler")  # main.go:114
        broker.start()  # (after any worker process has forked) the queues' first sets
        fleet.start(max_iterations)
        worker_died = False
        while not fleet.wait(0.2):
            if cfg.worker_processes and not worker_died and fleet.failed():
                # One queue's worker died (a crash, an OOM kill): stop the rest and exit non-zero
                # so the pod restarts with every queue polled, as when a thread crash takes the
                # whole process down.
                worker_died = True
                log.log("error", f"worker process(es) {fleet.failed()} died (exit codes {fleet.exit_codes()}); "
                                 "stopping the other workers")
                fleet.stop()
        fleet.join()
        if cfg.worker_processes and any(c not in (0, None) for c in fleet.exit_codes()):
            log.log("error", f"worker process exit codes: {fleet.exit_codes()}")
            if not got:
                return 1
        if lost.is_set():
            log.log("fatal", "leaderelection lost")
            return 1
        if got:
            log.log("info", "Stopped kube-sqs-autoscaler")
    finally:
        renew_stop.set()
        if renewer is not None:
            renewer.join(timeout=5)
        if elector is not None and not lost.is_set():
            elector.release()
        for sig, h in prev.items():
            signal.signal(sig, h)
        if capper is not None:
            capper.stop()
        if metrics is not None:
            metrics.stop()
        if cfg.worker_processes:
            fleet.close()
        if cfg.worker_processes or fleet.wait(0):
            broker.close()  # no queue reads the slots any more
        else:
            broker.stop()  # threads still running (an exception left them): keep the slots mapped
        if trace_fd >= 0:
            os.close(trace_fd)
    return 0


def main_entry() -> None:
    """Console-script entry point (``kube-sqs-autoscaler`` on PATH, like the reference binary)."""
    sys.exit(main())


if __name__ == "__main__":
    sys.exit(main())
