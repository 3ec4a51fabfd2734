"""Multi-queue execution: one native worker thread per tracked queue.

The reference runs exactly one loop per process (``Run`` never returns, /root/reference/main.go:35-80;
one URL and one Deployment, main.go:95-97). BASELINE.json asks for 1/2/4/8 concurrently tracked
queues, so a :class:`Fleet` owns N independent ``Runner`` objects and drives them from the
native ``Supervisor`` (csrc/core/runner.h): each worker has its own clients, connections,
timers and stats, and nothing is shared between workers (SURVEY.md §5.2 -- no cross-queue
locks, so no races by construction). Stopping is cooperative: a stop request interrupts every
worker's poll sleep, so SIGTERM ends the process within one in-flight API call (the reference
has no graceful shutdown, main.go:36).
"""
from __future__ import annotations

import threading
from typing import List, Sequence

from ..ops import native


class Fleet:
    """``threads`` <= 0 or >= len(workers): one native thread per queue (``Supervisor``, with a
    staggered start: each queue's Run() entry, main.go:37-38, is spread over its first period);
    otherwise ``threads`` workers share the queues through the native ``Scheduler`` (a timer
    heap that keeps every queue's sleep-then-poll cadence), for processes tracking hundreds of
    queues."""

    def __init__(self, workers: Sequence, threads: int = 0) -> None:
        self.workers = list(workers)
        nat = native()
        self.pooled = 0 < threads < len(self.workers)
        if self.pooled:
            self._sup = nat.Scheduler(threads)  # staggered by default
        else:
            # queue i of N starts i/N of its poll period late (as the pooled Scheduler does), so N
            # queues at one cadence do not all poll in the same instant every period
            self._sup = nat.Supervisor()
            self._sup.stagger = True
        for w in self.workers:
            self._sup.add(w.runner)
        self._started = False
        self._lock = threading.Lock()

    def start(self, max_iterations: int = -1) -> None:
        with self._lock:
            if self._started:
                raise RuntimeError("fleet already started")
            self._started = True
        self._sup.start(max_iterations)

    def stop(self) -> None:
        self._sup.stop()

    @property
    def started(self) -> bool:
        return self._started

    @property
    def stopped(self) -> bool:
        return self._sup.stopped()

    def wait(self, timeout_s: float) -> bool:
        """True when every worker has exited (max_iterations reached or stopped)."""
        return self._sup.wait(max(int(timeout_s * 1e9), 1))

    def join(self) -> None:
        self._sup.join()

    def late_polls(self) -> int:
        """Polls a pooled scheduler started >1 ms after they were due (0 for thread-per-queue)."""
        return self._sup.late_polls() if self.pooled else 0

    def stats(self) -> List[dict]:
        out = []
        for w in self.workers:
            s = dict(w.runner.stats())
            s["deployment"] = w.target.name
            s["queue"] = w.target.queue_url
            out.append(s)
        return out
