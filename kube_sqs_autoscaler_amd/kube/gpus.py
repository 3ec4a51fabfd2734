"""GPU-capacity cap for ``--max-pods`` (extension: the MI355X specialisation).

The scaled Deployment is GPU-worker pods, one (or ``--gpus-per-pod``) MI355X each. Scaling past
the GPUs the scheduler can place only creates Pending pods, so ``--gpu-aware-max`` caps the
effective max-pods:

* ``local`` -- GPUs on this node that pass the gfx950 HBM probe (``ops/gpu.py``), measured once
  at start-up (sidecar deployments on the GPU node);
* ``cluster`` -- the sum of ``status.allocatable[--gpu-resource]`` (default ``amd.com/gpu``, what
  the AMD GPU device plugin advertises) over schedulable nodes matching ``--gpu-node-selector``,
  divided by ``--gpus-per-pod``, refreshed every ``--gpu-refresh-period``.

The cap is ``min(--max-pods, capacity)``, never below ``--min-pods``, and is applied through
the native actuator's atomic ``set_max``, so a refresh never races a running scale decision. A
failed refresh keeps the last good cap; no capacity read yet means no cap. A capacity of 0 (no
GPU visible, every GPU node cordoned) is treated as "unknown": it is logged as a warning and the
configured ``--max-pods`` stays in force -- a cap of 0 would silently turn every scale-up into a
no-op at max.

``local`` only sees the GPUs allocated to the autoscaler's own pod: under the AMD GPU device
plugin a pod that requests no ``amd.com/gpu`` sees none, so a ``local`` sidecar must request
the GPUs it is meant to count (``cluster`` has no such constraint).
"""
from __future__ import annotations

import json
import threading
import urllib.parse
from typing import Callable, Optional, Sequence

from ..ops import native
from .config import RestConfig


class CapacityError(RuntimeError):
    pass


def _quantity(v) -> int:
    """Integer resource quantity ("8", 8, "8000m" -> 8)."""
    if isinstance(v, int):
        return v
    s = str(v).strip()
    if s.endswith("m"):
        return int(s[:-1]) // 1000
    for suffix, mul in (("k", 1000), ("Ki", 1024)):
        if s.endswith(suffix):
            return int(s[: -len(suffix)]) * mul
    return int(s)


class ClusterGpuCapacity:
    def __init__(self, rest: RestConfig, resource: str = "amd.com/gpu", node_selector: str = "",
                 gpus_per_pod: int = 1, timeout_s: float = 10.0):
        from ..autoscaler import new_http_client

        if gpus_per_pod < 1:
            raise ValueError("gpus-per-pod must be >= 1")
        self.rest = rest
        self.resource = resource
        self.selector = node_selector
        self.gpus_per_pod = gpus_per_pod
        self.http = new_http_client(rest, int(timeout_s * 1e9))

    def _headers(self):
        from ..autoscaler import auth_headers

        return [("Accept", "application/json")] + auth_headers(self.rest)

    def allocatable_gpus(self) -> int:
        path = "/api/v1/nodes"
        if self.selector:
            path += "?labelSelector=" + urllib.parse.quote(self.selector, safe="=,!")
        from ..autoscaler import note_status

        try:
            headers = self._headers()
            status, _, body = self.http.request("GET", path, headers)
        except native().NativeError as e:
            raise CapacityError(f"list nodes: {e}")
        note_status(self.rest, headers, status)
        if status != 200:
            raise CapacityError(f"list nodes: HTTP {status}: {body[:200]!r}")
        total = 0
        for node in json.loads(body).get("items", []):
            if (node.get("spec") or {}).get("unschedulable"):
                continue
            alloc = (node.get("status") or {}).get("allocatable") or {}
            if self.resource in alloc:
                total += _quantity(alloc[self.resource])
        return total

    def pod_capacity(self) -> int:
        return self.allocatable_gpus() // self.gpus_per_pod


class MaxPodsCapper:
    """Applies ``min(configured max, capacity)`` to actuators, periodically."""

    def __init__(self, scalers: Sequence, configured_max: Sequence[int], capacity: Callable[[], int],
                 refresh_s: float = 60.0, log: Optional[Callable[[str, str], None]] = None,
                 min_pods: Optional[Sequence[int]] = None):
        self.scalers = list(scalers)
        self.configured = list(configured_max)
        self.floor = list(min_pods) if min_pods is not None else [getattr(s, "min", 0) for s in self.scalers]
        self.capacity = capacity
        self.refresh_s = refresh_s
        self.log = log or (lambda lvl, m: None)
        self.cap: Optional[int] = None
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def refresh(self) -> Optional[int]:
        try:
            cap = self.capacity()
        except Exception as e:  # keep the last good cap
            self.log("warning", f"GPU capacity refresh failed, keeping max-pods cap {self.cap}: {e}")
            return self.cap
        if cap <= 0:
            if cap != self.cap:
                self.log("warning", f"GPU capacity reads {cap} pods (no GPU visible to --gpu-aware-max?); "
                                    f"keeping the configured max-pods {self.configured}")
            self.cap = cap
            for s, m in zip(self.scalers, self.configured):
                s.max = m
            return cap
        eff = [max(min(m, cap), lo) for m, lo in zip(self.configured, self.floor)]
        if cap != self.cap:
            self.log("info", f"GPU capacity: {cap} pods; effective max-pods {eff}")
        self.cap = cap
        for s, e in zip(self.scalers, eff):
            s.max = e
        return cap

    def start(self) -> None:
        self._thread = threading.Thread(target=self._loop, name="ksa-gpu-capacity", daemon=True)
        self._thread.start()

    def _loop(self) -> None:
        while not self._stop.wait(self.refresh_s):
            self.refresh()

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
