"""Process-per-queue fleet: every tracked queue runs in a worker process of its own.

The reference is one process per queue (/root/reference/main.go:95-97, one URL and one
Deployment). :class:`~.fleet.Fleet` runs N queues as N threads of one process, and since each
runner keeps one thread for its life (``HomeThread``, csrc/core/runner.h; ``docs/HISTORY.md``
r02l) 8 thread queues poll as fast as 8 processes. ``--worker-processes`` keeps the
reference's isolation inside this build's single pod: separate address spaces, file tables
and allocators per queue, and per-process CPU and memory accounting. The supervisor forks one
worker per queue, each with its own native clients, connections, logger and ``Runner``, and
nothing mutable is shared except one
``SharedWorkerState`` slot per worker (csrc/core/runner.h) in an anonymous shared mapping:

* the worker mirrors its counters, latency ring and a heartbeat into its slot (lock-free);
* the supervisor reads the slots for ``/metrics`` and ``/healthz``, starts the workers together
  (``control = go``), stops them (``control = stop`` + SIGTERM), and forwards the GPU-capacity
  cap as a max-pods override the worker applies before its next poll.

Workers are forked when the fleet is built, before the supervisor starts any thread of its own
(metrics server, lease renewal) or touches the GPU; they wait for ``go``. A worker whose parent
dies gets SIGTERM (``PR_SET_PDEATHSIG``) and stops like on a graceful shutdown.
"""
from __future__ import annotations

import ctypes
import mmap
import os
import signal
import sys
import threading
import time
import traceback
from typing import Callable, List, Optional, Sequence

from ..ops import native

_PR_SET_PDEATHSIG = 1


class _SlotScaler:
    """What MaxPodsCapper needs of a scaler, for a worker in another process."""

    def __init__(self, addr: int, min_pods: int, max_pods: int):
        self._addr = addr
        self.min = min_pods
        self._max = max_pods

    @property
    def max(self) -> int:
        return self._max

    @max.setter
    def max(self, v: int) -> None:
        self._max = int(v)
        native().set_shared_worker_max(self._addr, int(v))


class SlotRunner:
    """Read-only view of a worker process' runner (the parts metrics and health use)."""

    def __init__(self, addr: int, scaler: _SlotScaler):
        self._addr = addr
        self.scaler = scaler

    def state(self) -> dict:
        return native().read_shared_worker_state(self._addr)

    def stats(self) -> dict:
        return self.state()

    def latencies(self) -> List[int]:
        return native().shared_worker_latencies(self._addr)

    def idle_ns(self) -> int:
        p = self.state()["progress_ns"]
        return max(0, time.monotonic_ns() - p) if p else 0

    def failing_ns(self) -> int:
        st = self.state()
        if not st["consecutive_failed_polls"] or not st["last_good_ns"]:
            return 0
        return max(0, time.monotonic_ns() - st["last_good_ns"])

    def last_error(self) -> str:
        """The worker's last poll error, as the thread fleet's Runner.last_error() gives it
        (carried through the shared slot, truncated to 511 bytes)."""
        return native().read_shared_worker_error(self._addr)


class ProcWorker:
    def __init__(self, target, runner: SlotRunner, pid: int):
        self.target = target
        self.runner = runner
        self.pid = pid
        self.kube_api = None  # the clients live in the worker process
        self.sqs_api = None


def _child(build: Callable[[], object], addr: int, cpus: Optional[List[int]]) -> None:
    """Body of a worker process (never returns)."""
    nat = native()
    code = 0
    try:
        try:
            ctypes.CDLL(None, use_errno=True).prctl(_PR_SET_PDEATHSIG, signal.SIGTERM, 0, 0, 0)
        except (OSError, AttributeError):
            pass
        sup_box: List[object] = []

        def on_signal(signum, frame):
            for s in sup_box:
                s.stop()
            nat.set_shared_worker_control(addr, 2)

        if threading.current_thread() is threading.main_thread():
            signal.signal(signal.SIGTERM, on_signal)
            signal.signal(signal.SIGINT, on_signal)
        worker = build()
        runner = worker.runner
        if cpus:
            runner.cpus = cpus
        runner.set_shared_state(addr)
        nat.set_shared_worker_progress(addr, time.monotonic_ns())
        nat.set_shared_worker_status(addr, 1)  # ready
        while True:
            st = nat.read_shared_worker_state(addr)
            if st["control"] != 0:
                break
            time.sleep(0.0005)
        if st["control"] == 1:
            sup = nat.Supervisor()
            sup.add(runner)
            sup_box.append(sup)
            sup.start(st["iterations"])
            nat.set_shared_worker_status(addr, 2)  # running
            while not sup.wait(200_000_000):
                nat.set_shared_worker_progress(addr, time.monotonic_ns() - runner.idle_ns())
                if nat.read_shared_worker_state(addr)["control"] == 2:
                    sup.stop()
            sup.join()
            nat.set_shared_worker_progress(addr, time.monotonic_ns())
        nat.set_shared_worker_status(addr, 3)  # exited
    except BaseException:  # noqa: BLE001 -- a worker process must always report and exit
        traceback.print_exc()
        try:
            nat.set_shared_worker_status(addr, 4)  # failed
        except Exception:
            pass
        code = 1
    finally:
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(code)


class ProcessFleet:
    """The :class:`~.fleet.Fleet` interface over one worker process per queue.

    ``builds[i]()`` runs in worker i's process and returns an object with ``.runner`` (a native
    ``Runner``); ``targets[i]`` is the matching TargetConfig (names, clamp bounds for the cap).
    ``cpus[i]`` optionally pins worker i's loop thread."""

    def __init__(self, builds: Sequence[Callable[[], object]], targets: Sequence, cpus: Optional[Sequence] = None):
        nat = native()
        n = len(builds)
        size = nat.shared_worker_state_size()
        self._slot = (size + mmap.PAGESIZE - 1) // mmap.PAGESIZE * mmap.PAGESIZE
        self._mm = mmap.mmap(-1, max(1, n) * self._slot, flags=mmap.MAP_SHARED | mmap.MAP_ANONYMOUS)
        self._buf = ctypes.c_char.from_buffer(self._mm)
        base = ctypes.addressof(self._buf)
        self.addrs = [base + i * self._slot for i in range(n)]
        for a in self.addrs:
            nat.init_shared_worker_state(a)
        sys.stdout.flush()
        sys.stderr.flush()
        self.workers: List[ProcWorker] = []
        for i, (build, t) in enumerate(zip(builds, targets)):
            pid = os.fork()
            if pid == 0:
                _child(build, self.addrs[i], list(cpus[i]) if cpus is not None else None)
            scaler = _SlotScaler(self.addrs[i], getattr(t, "min_pods", 0), getattr(t, "max_pods", 0))
            self.workers.append(ProcWorker(t, SlotRunner(self.addrs[i], scaler), pid))
        self._started = False
        self._stopped = False
        self._stop_at = 0.0
        self._reaped = {}
        self._lock = threading.Lock()

    pooled = False

    def late_polls(self) -> int:
        return 0

    def _states(self) -> List[dict]:
        return [w.runner.state() for w in self.workers]

    def wait_ready(self, timeout_s: float = 60.0) -> None:
        """Blocks until every worker has built its clients (raises if one failed or died)."""
        deadline = time.monotonic() + timeout_s
        while True:
            self._reap()
            st = self._states()
            bad = [i for i, s in enumerate(st)
                   if s["status"] == 4 or (self.workers[i].pid in self._reaped and s["status"] < 1)]
            if bad:
                raise RuntimeError(f"worker process(es) {bad} failed to start")
            if all(s["status"] >= 1 for s in st):
                return
            if time.monotonic() > deadline:
                raise TimeoutError("worker processes did not become ready")
            time.sleep(0.001)

    def start(self, max_iterations: int = -1) -> None:
        with self._lock:
            if self._started:
                raise RuntimeError("fleet already started")
            self._started = True
        self.wait_ready()
        nat = native()
        for a in self.addrs:
            nat.set_shared_worker_iterations(a, max_iterations)
        for a in self.addrs:  # the workers start together
            nat.set_shared_worker_control(a, 1)

    # A worker still alive this long after a stop is stuck in something a stop does not end; it
    # is killed, so the pod's shutdown never rests on the kubelet's SIGKILL after the grace
    # period (30 s by default).
    KILL_AFTER_S = 10.0

    def stop(self) -> None:
        if not self._stopped:
            self._stop_at = time.monotonic()
        self._stopped = True
        nat = native()
        for a in self.addrs:
            nat.set_shared_worker_control(a, 2)
        for w in self.workers:
            if w.pid not in self._reaped:
                try:
                    os.kill(w.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass

    @property
    def started(self) -> bool:
        return self._started

    @property
    def stopped(self) -> bool:
        return self._stopped

    def _reap(self) -> None:
        for w in self.workers:
            if w.pid in self._reaped:
                continue
            try:
                pid, status = os.waitpid(w.pid, os.WNOHANG)
            except ChildProcessError:
                self._reaped[w.pid] = 0
                continue
            if pid:
                self._reaped[w.pid] = status

    def wait(self, timeout_s: float) -> bool:
        """True when every worker process has exited."""
        deadline = time.monotonic() + max(timeout_s, 0.0)
        while True:
            self._reap()
            if len(self._reaped) == len(self.workers):
                return True
            if time.monotonic() >= deadline:
                return False
            time.sleep(min(0.002, max(0.0, deadline - time.monotonic())))

    def join(self) -> None:
        if not self._started:
            self.stop()
        while not self.wait(0.2):
            if self._stopped and time.monotonic() - self._stop_at > self.KILL_AFTER_S:
                for w in self.workers:
                    if w.pid not in self._reaped:
                        try:
                            os.kill(w.pid, signal.SIGKILL)
                        except ProcessLookupError:
                            pass

    def failed(self) -> List[int]:
        """Indices of workers that exited with an error or were killed (an OOM kill, a crash).

        Threads of one process die together and the pod restarts; a worker process can die alone,
        so the supervisor asks this and brings the whole fleet down instead of letting one queue
        go unpolled while the others carry on."""
        self._reap()
        return [i for i, w in enumerate(self.workers)
                if w.pid in self._reaped and os.waitstatus_to_exitcode(self._reaped[w.pid]) != 0]

    def exit_codes(self) -> List[int]:
        self._reap()
        return [os.waitstatus_to_exitcode(self._reaped[w.pid]) if w.pid in self._reaped else None for w in self.workers]

    def stats(self) -> List[dict]:
        out = []
        for w in self.workers:
            s = dict(w.runner.stats())
            s["deployment"] = w.target.name
            s["queue"] = w.target.queue_url
            out.append(s)
        return out

    def close(self) -> None:
        """Stops and reaps the workers, then unmaps the slots."""
        if len(self._reaped) < len(self.workers):
            self.stop()
            self.join()
        del self._buf
        self._mm.close()
