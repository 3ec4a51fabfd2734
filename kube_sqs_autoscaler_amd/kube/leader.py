"""Lease-based leader election (extension: high availability).

The reference has no leader election: two replicas would both scale, so its README deploys
``replicas: 1`` (/root/reference/README.md:27). With ``--leader-elect`` several
autoscaler replicas can run and exactly one drives the Deployments.

The algorithm is client-go's ``leaderelection`` with a ``coordination.k8s.io/v1`` Lease lock:

* ``try_acquire_or_renew``: read the Lease. Create it if it is missing. If another holder's
  record is still valid, give up. Validity is measured with the *local* clock from when this
  replica last saw the record change, never the remote ``renewTime``, so clock skew cannot
  cause two leaders. Otherwise write ourselves as holder, guarded by ``resourceVersion``; a 409
  means another candidate won.
* the leader renews every ``retry_period``; if no renewal succeeds within ``renew_deadline`` it
  has lost the lease and must stop scaling;
* on graceful shutdown the leader releases the lease (empty holder, 1 s duration), so a standby
  takes over without waiting ``lease_duration``.

Timers follow the reference: a replica that becomes leader starts its control loop fresh, with
cool-downs armed at that moment (main.go:37-38), the same as a restart.
"""
from __future__ import annotations

import json
import os
import socket
import threading
import time
from dataclasses import dataclass
from datetime import datetime, timezone
from typing import Callable, Optional, Tuple

from ..ops import native
from .config import RestConfig

LEASE_API = "/apis/coordination.k8s.io/v1/namespaces/{ns}/leases"


def micro_time(unix_s: float) -> str:
    """metav1.MicroTime wire format (RFC3339 with microseconds)."""
    return datetime.fromtimestamp(unix_s, tz=timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def default_identity() -> str:
    # client-go examples use the pod name; fall back to hostname + pid
    return os.environ.get("POD_NAME") or f"{socket.gethostname()}_{os.getpid()}"


class LeaseError(RuntimeError):
    def __init__(self, msg: str, status: int = 0):
        super().__init__(msg)
        self.status = status


@dataclass
class LeaderElectionRecord:
    holder: str = ""
    lease_duration_s: int = 15
    acquire_time: str = ""
    renew_time: str = ""
    transitions: int = 0

    def spec(self) -> dict:
        s = {"holderIdentity": self.holder, "leaseDurationSeconds": self.lease_duration_s,
             "leaseTransitions": self.transitions}
        if self.acquire_time:
            s["acquireTime"] = self.acquire_time
        if self.renew_time:
            s["renewTime"] = self.renew_time
        return s

    @staticmethod
    def from_spec(spec: dict) -> "LeaderElectionRecord":
        return LeaderElectionRecord(
            holder=spec.get("holderIdentity") or "", lease_duration_s=int(spec.get("leaseDurationSeconds") or 0),
            acquire_time=spec.get("acquireTime") or "", renew_time=spec.get("renewTime") or "",
            transitions=int(spec.get("leaseTransitions") or 0))


class LeaseLock:
    """Lease CRUD over the native keep-alive HTTP client (TLS, CA, bearer/basic auth)."""

    def __init__(self, rest: RestConfig, namespace: str, name: str, timeout_s: float = 10.0):
        from ..autoscaler import new_http_client

        self.rest = rest
        self.namespace = namespace
        self.name = name
        self.http = new_http_client(rest, int(timeout_s * 1e9))
        self._rv = ""
        # Instant by which every call must have returned, on ``self.monotonic`` (the elector's
        # clock: LeaderElector points it at its own, so the renew deadline and the per-call limit
        # share one time base); None: each call only has the client's own timeout.
        self.deadline: Optional[float] = None
        self.monotonic: Callable[[], float] = time.monotonic

    def _headers(self, body: bool = False):
        from ..autoscaler import auth_headers

        h = [("Accept", "application/json")] + auth_headers(self.rest)
        if body:
            h.append(("Content-Type", "application/json"))
        return h

    def _path(self, with_name: bool = True) -> str:
        base = LEASE_API.format(ns=self.namespace)
        return f"{base}/{self.name}" if with_name else base

    def _call(self, method: str, path: str, body: Optional[dict] = None) -> Tuple[int, dict]:
        nat = native()
        from ..autoscaler import note_status

        timeout_ns = -1
        if self.deadline is not None:
            left = self.deadline - self.monotonic()
            if left <= 0:
                raise LeaseError("renew deadline exceeded")
            timeout_ns = max(1, int(left * 1e9))
        try:
            headers = self._headers(body is not None)
            status, _, raw = self.http.request(method, path, headers,
                                               json.dumps(body).encode() if body is not None else b"", timeout_ns)
        except nat.NativeError as e:
            raise LeaseError(str(e))
        note_status(self.rest, headers, status)
        try:
            return status, json.loads(raw) if raw else {}
        except ValueError:
            return status, {}

    def get(self) -> Optional[LeaderElectionRecord]:
        status, obj = self._call("GET", self._path())
        if status == 404:
            return None
        if status != 200:
            raise LeaseError(obj.get("message") or f"GET lease: HTTP {status}", status)
        self._rv = obj.get("metadata", {}).get("resourceVersion", "")
        return LeaderElectionRecord.from_spec(obj.get("spec") or {})

    def create(self, rec: LeaderElectionRecord) -> None:
        body = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                "metadata": {"name": self.name, "namespace": self.namespace}, "spec": rec.spec()}
        status, obj = self._call("POST", self._path(False), body)
        if status not in (200, 201):
            raise LeaseError(obj.get("message") or f"POST lease: HTTP {status}", status)
        self._rv = obj.get("metadata", {}).get("resourceVersion", "")

    def update(self, rec: LeaderElectionRecord) -> None:
        body = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                "metadata": {"name": self.name, "namespace": self.namespace, "resourceVersion": self._rv},
                "spec": rec.spec()}
        status, obj = self._call("PUT", self._path(), body)
        if status != 200:
            raise LeaseError(obj.get("message") or f"PUT lease: HTTP {status}", status)
        self._rv = obj.get("metadata", {}).get("resourceVersion", "")

    def describe(self) -> str:
        return f"{self.namespace}/{self.name}"


class LeaderElector:
    def __init__(self, lock: LeaseLock, identity: str, lease_duration_s: float = 15.0, renew_deadline_s: float = 10.0,
                 retry_period_s: float = 2.0, monotonic: Callable[[], float] = time.monotonic,
                 wall: Callable[[], float] = time.time, log: Optional[Callable[[str, str], None]] = None):
        if not lease_duration_s > renew_deadline_s > retry_period_s > 0:
            raise ValueError("need lease_duration > renew_deadline > retry_period > 0")
        self.lock = lock
        self.identity = identity
        self.lease_duration = lease_duration_s
        self.renew_deadline = renew_deadline_s
        self.retry_period = retry_period_s
        self.monotonic = monotonic
        lock.monotonic = monotonic  # the lock's per-call deadline is set on this clock
        self.wall = wall
        self.log = log or (lambda level, msg: None)
        self.observed: Optional[LeaderElectionRecord] = None
        self.observed_at = 0.0
        self._leader = False

    @property
    def is_leader(self) -> bool:
        return self._leader

    def try_acquire_or_renew(self) -> bool:
        now_wall = micro_time(self.wall())
        desired = LeaderElectionRecord(self.identity, int(self.lease_duration), now_wall, now_wall, 0)
        try:
            old = self.lock.get()
        except LeaseError as e:
            self.log("error", f"error retrieving resource lock {self.lock.describe()}: {e}")
            return False
        if old is None:
            try:
                self.lock.create(desired)
            except LeaseError as e:
                self.log("error", f"error initially creating leader election record: {e}")
                return False
            self._observe(desired)
            return True
        if self.observed is None or old.spec() != self.observed.spec():
            self._observe(old)
        held_by_other = old.holder and old.holder != self.identity
        if held_by_other and self.observed_at + max(old.lease_duration_s, 1) > self.monotonic():
            return False  # another replica holds a valid lease
        if old.holder == self.identity:
            desired.acquire_time = old.acquire_time
            desired.transitions = old.transitions
        else:
            desired.transitions = old.transitions + 1
        try:
            self.lock.update(desired)
        except LeaseError as e:
            if e.status != 409:
                self.log("error", f"Failed to update lock: {e}")
            return False  # lost the race
        self._observe(desired)
        return True

    def _observe(self, rec: LeaderElectionRecord) -> None:
        self.observed = rec
        self.observed_at = self.monotonic()

    def acquire(self, stop: threading.Event) -> bool:
        """Blocks until this replica holds the lease (True) or ``stop`` is set (False)."""
        self.log("info", f"attempting to acquire leader lease {self.lock.describe()}...")
        while not stop.is_set():
            if self.try_acquire_or_renew():
                self._leader = True
                self.log("info", f"successfully acquired lease {self.lock.describe()}")
                return True
            stop.wait(self.retry_period)
        return False

    def renew_loop(self, stop: threading.Event, on_lost: Callable[[], None]) -> None:
        """Renews every retry_period. Leadership ends ``renew_deadline`` after the last successful
        renewal, at that instant, even while a renewal is still in flight: a watchdog calls
        ``on_lost`` when the deadline passes, and each attempt's lease calls only get the time
        left before it (client-go bounds every renew with a RenewDeadline context). A standby
        takes over ``lease_duration`` after it saw that last renewal, so the two never scale
        together (lease_duration > renew_deadline)."""
        mu = threading.Lock()
        lost = threading.Event()
        finished = threading.Event()
        last_ok = [self.monotonic()]

        def left() -> float:
            with mu:
                return last_ok[0] + self.renew_deadline - self.monotonic()

        def lose() -> None:
            with mu:
                if lost.is_set():
                    return
                lost.set()
                self._leader = False
            self.log("error", f"failed to renew lease {self.lock.describe()}: timed out waiting for the condition")
            on_lost()

        def watchdog() -> None:
            while not finished.is_set() and not stop.is_set():
                remaining = left()
                if remaining <= 0:
                    lose()
                    return
                finished.wait(min(remaining, self.retry_period))

        wd = threading.Thread(target=watchdog, name="ksa-lease-watchdog", daemon=True)
        wd.start()
        try:
            while not lost.is_set() and not stop.wait(self.retry_period):
                remaining = left()
                if remaining <= 0:
                    lose()
                    break
                self.lock.deadline = self.monotonic() + remaining
                ok = self.try_acquire_or_renew()
                with mu:
                    if ok and not lost.is_set():  # a success after the deadline does not count
                        last_ok[0] = self.monotonic()
        finally:
            self.lock.deadline = None
            finished.set()
            wd.join()

    def release(self) -> bool:
        """Gives the lease up (ReleaseOnCancel) so a standby can take over at once."""
        if not self._leader:
            return False
        self._leader = False
        try:
            old = self.lock.get()
            if old is None or old.holder != self.identity:
                return False
            now_wall = micro_time(self.wall())
            self.lock.update(LeaderElectionRecord("", 1, now_wall, now_wall, old.transitions))
            return True
        except LeaseError as e:
            self.log("error", f"Failed to release lock: {e}")
            return False
