"""What-if policy sweep: evaluate many autoscaler configurations against one queue-depth trace.

Extension (an operator tool, not a reference capability). Tuning cool-downs and thresholds of
the reference algorithm against a recorded queue means replaying the same trace
under thousands of candidate settings. Every candidate is an independent integer state machine.
The gfx950 kernel (csrc/hip/policy_sweep.hip) runs one per lane; the CPU path (csrc/core/sweep.cc)
runs the identical code (csrc/sim/policy_sim.h) on threads. Both agree exactly with each other
and with the Python oracle (``models/oracle.py``).

Inputs:

* a depth trace: piecewise-constant ``(t_ns, depth)`` segments, from a ``--trace-file`` span
  log, a CSV ``seconds,depth``, or synthetic arrays;
* a parameter grid: every combination of the listed values;
* a latency model (constant per SQS / GET / write call) and a horizon.

Outputs per configuration:

* ``pod_ms`` (cost), ``backlog`` (msg-ms per pod, queue pressure; one integer division per run
  of constant replicas, see csrc/sim/policy_sim.h);
* scale-up/down counts and no-ops;
* final and peak replicas, first scale-up time, poll count.
"""
from __future__ import annotations

import ctypes
import itertools
import json
import os
from dataclasses import dataclass
from typing import Dict, Iterable, Optional, Sequence, Tuple

import numpy as np

PARAM_FIELDS = ("poll_ns", "up_cool_ns", "down_cool_ns", "up_msgs", "down_msgs", "up_pods", "down_pods",
                "max_pods", "min_pods")
OUT64 = ("pod_ms", "backlog", "first_up_ns")
OUT32 = ("ups", "downs", "noop_ups", "noop_downs", "final_replicas", "max_replicas", "polls")

# the reference defaults (main.go:83-91) with this build's max-pods
DEFAULTS = dict(poll_ns=5_000_000_000, up_cool_ns=10_000_000_000, down_cool_ns=30_000_000_000, up_msgs=100,
                down_msgs=10, up_pods=1, down_pods=1, max_pods=8, min_pods=1)


@dataclass
class Trace:
    t_ns: np.ndarray  # int64, sorted, t_ns[0] == 0
    depth: np.ndarray  # int64

    def __post_init__(self):
        self.t_ns = np.ascontiguousarray(self.t_ns, dtype=np.int64)
        self.depth = np.ascontiguousarray(self.depth, dtype=np.int64)
        if self.t_ns.ndim != 1 or self.t_ns.shape != self.depth.shape or len(self.t_ns) == 0:
            raise ValueError("trace needs equal-length non-empty 1-D t_ns and depth")
        if self.t_ns[0] != 0 or np.any(np.diff(self.t_ns) < 0):
            raise ValueError("trace times must start at 0 and be sorted")

    @staticmethod
    def from_segments(segments: Sequence[Tuple[int, int]]) -> "Trace":
        return Trace(np.array([s[0] for s in segments]), np.array([s[1] for s in segments]))

    @staticmethod
    def from_spans(path: str, queue: Optional[str] = None) -> "Trace":
        """A ``--trace-file`` span log: depth observed at each poll, held until the next poll."""
        ts, ds = [], []
        with open(path) as f:
            for line in f:
                s = json.loads(line)
                if queue and s.get("queue") != queue and s.get("deployment") != queue:
                    continue
                if s.get("depth") is None:
                    continue
                ts.append(int(s["ts"]))
                ds.append(int(s["depth"]))
        if not ts:
            raise ValueError(f"no spans with a depth in {path}")
        order = np.argsort(ts, kind="stable")
        t = np.array(ts, dtype=np.int64)[order]
        return Trace(t - t[0], np.array(ds, dtype=np.int64)[order])

    @staticmethod
    def from_csv(path: str) -> "Trace":
        """``seconds,depth`` rows (header optional)."""
        rows = []
        with open(path) as f:
            for line in f:
                parts = line.strip().split(",")
                if len(parts) < 2:
                    continue
                try:
                    rows.append((float(parts[0]), int(float(parts[1]))))
                except ValueError:
                    continue  # header
        rows.sort()
        t0 = rows[0][0]
        return Trace(np.array([int(round((t - t0) * 1e9)) for t, _ in rows]), np.array([d for _, d in rows]))


def grid(**values: Iterable[int]) -> np.ndarray:
    """Cartesian product of parameter values -> ``(9, m)`` int64, poll period outermost (so
    neighbouring GPU lanes share loop trip counts). Unlisted fields take the defaults."""
    lists = [list(values.get(f, [DEFAULTS[f]])) for f in PARAM_FIELDS]
    unknown = set(values) - set(PARAM_FIELDS)
    if unknown:
        raise ValueError(f"unknown parameters {sorted(unknown)}; expected {PARAM_FIELDS}")
    combos = np.array(list(itertools.product(*lists)), dtype=np.int64)
    return np.ascontiguousarray(combos.T)


# ---------------------------------------------------------------------------------------------


MAX_TOTAL_POLLS = 2e11  # ~tens of seconds of GPU time; every lane also stops at kMaxPolls


def estimated_polls(params: np.ndarray, horizon_ns: int, latency_ns: Tuple[int, int, int]) -> float:
    step = np.maximum(params[0], 0) + latency_ns[0]
    step = np.maximum(step, 1)
    return float(np.minimum(horizon_ns // step, 1 << 26).sum())


def _gpu_lib():
    from ..ops import gpu

    lib = gpu.load()
    if not getattr(lib, "_sweep_ready", False):
        lib.ksa_sweep_gpu.restype = ctypes.c_int
        lib.ksa_sweep_gpu.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int32,
                                      ctypes.POINTER(ctypes.c_int32)]
        lib.ksa_sweep_last_error.restype = ctypes.c_char_p
        lib._sweep_ready = True
    return lib


def gpu_available() -> bool:
    try:
        from ..ops import gpu

        return gpu.device_count() > 0
    except Exception:
        return False


@dataclass
class SweepResult:
    params: np.ndarray  # (9, m)
    out: Dict[str, np.ndarray]
    device: str
    kernel_ms: float = 0.0
    ms_clock: bool = False  # the native path ran policy_sim.h's simulate_ms (whole-ms periods and latencies)
    skip: bool = False  # ... with the steady-stretch skip (policy_sim.h steady_limit; same results)

    def __len__(self) -> int:
        return self.params.shape[1]

    def config(self, i: int) -> Dict[str, int]:
        return {f: int(self.params[k, i]) for k, f in enumerate(PARAM_FIELDS)}

    def row(self, i: int) -> Dict[str, int]:
        r = self.config(i)
        r.update({k: int(v[i]) for k, v in self.out.items()})
        return r


def run(trace: Trace, params: np.ndarray, init_replicas: int = 1, horizon_ns: int = 3600 * 10**9,
        latency_ns: Tuple[int, int, int] = (1_000_000, 1_000_000, 1_000_000), device: str = "auto",
        threads: int = 0, gpu_index: int = 0, clock: str = "auto", skip: str = "auto") -> SweepResult:
    """Runs the sweep. ``clock``: ``"auto"`` simulates on 32-bit millisecond clocks when every
    period that can fire and every latency is a whole number of milliseconds (policy_sim.h
    ``ms_path_ok``; identical results), else on 64-bit nanosecond clocks; ``"ns"`` always uses
    the latter. ``skip``: adding up a stretch of polls that call nothing at once (policy_sim.h
    ``steady_limit``; identical results) -- ``"auto"`` when a trace segment spans several polls
    (``skip_pays``), ``"on"`` / ``"off"`` to force it."""
    if clock not in ("auto", "ns"):
        raise ValueError(f"clock must be auto or ns, not {clock!r}")
    skip_mode = {"auto": 0, "on": 1, "off": 2}.get(skip)
    if skip_mode is None:
        raise ValueError(f"skip must be auto, on or off, not {skip!r}")
    params = np.ascontiguousarray(params, dtype=np.int64)
    if params.ndim != 2 or params.shape[0] != len(PARAM_FIELDS):
        raise ValueError("params must have shape (9, m); build it with grid()")
    if not 0 < horizon_ns < 2**60:
        raise ValueError("horizon must be positive and below 2^60 ns (36 years)")
    if any(not 0 <= int(x) <= 3600 * 10**9 for x in latency_ns):
        raise ValueError("latencies must be within [0, 1 h] (ksa_sim::kMaxLatencyNs)")
    if np.any((params[0] <= 0) & (latency_ns[0] <= 0)):
        raise ValueError("a zero poll period needs a positive SQS latency (time would not advance)")
    lat = np.array(latency_ns, dtype=np.int64)
    m = params.shape[1]
    est = estimated_polls(params, horizon_ns, latency_ns)
    if est > MAX_TOTAL_POLLS:
        raise ValueError(f"sweep too large: ~{est:.3g} simulated polls (limit {MAX_TOTAL_POLLS:.3g}); "
                         "shorten the horizon, coarsen the grid or raise the poll period")
    if device == "auto":
        device = "gpu" if gpu_available() else "cpu"
    if device == "gpu":
        lib = _gpu_lib()
        out64 = np.zeros((3, m), dtype=np.int64)
        out32 = np.zeros((7, m), dtype=np.int32)
        ms = ctypes.c_double(0)
        used = ctypes.c_int32(0)
        rc = lib.ksa_sweep_gpu(gpu_index, trace.t_ns.ctypes.data, trace.depth.ctypes.data, len(trace.t_ns), init_replicas,
                               horizon_ns, lat.ctypes.data, params.ctypes.data, m, out64.ctypes.data, out32.ctypes.data,
                               ctypes.byref(ms), (1 if clock == "ns" else 0) | (skip_mode << 2), ctypes.byref(used))
        if rc != 0:
            raise RuntimeError("GPU sweep failed: " + (lib.ksa_sweep_last_error() or b"").decode())
        kernel_ms = ms.value
        ms_clock, skipped = bool(used.value & 1), bool(used.value & 2)
    elif device == "cpu":
        from ..ops import native

        out64, out32, ms_clock, skipped = native().sweep_cpu(trace.t_ns, trace.depth, init_replicas, horizon_ns, lat,
                                                             params, threads or (os.cpu_count() or 8), clock == "ns",
                                                             skip_mode)
        kernel_ms = 0.0
    else:
        raise ValueError(f"device must be auto, gpu or cpu, not {device!r}")
    out = {k: out64[i] for i, k in enumerate(OUT64)}
    out.update({k: out32[i] for i, k in enumerate(OUT32)})
    return SweepResult(params, out, device, kernel_ms, ms_clock, skipped)


def pareto_front(pod_ms: np.ndarray, backlog: np.ndarray) -> np.ndarray:
    """Indices of configurations not dominated on (pod_ms, backlog), cheapest first."""
    order = np.lexsort((backlog, pod_ms))  # by cost, then pressure
    front = []
    best = None
    for i in order:
        b = backlog[i]
        if best is None or b < best:
            front.append(int(i))
            best = b
    return np.array(front, dtype=np.int64)


def oracle_row(trace: Trace, cfg: Dict[str, int], init_replicas: int, horizon_ns: int,
               latency_ns: Tuple[int, int, int]) -> Dict[str, int]:
    """The same metrics from the independent Python oracle (exactness tests)."""
    from ..models import oracle

    names = ["ApproximateNumberOfMessages"]
    tr = [(int(t), {names[0]: str(int(d))}) for t, d in zip(trace.t_ns, trace.depth)]
    p = oracle.Params(cfg["poll_ns"], cfg["up_cool_ns"], cfg["down_cool_ns"], cfg["up_msgs"], cfg["down_msgs"],
                      cfg["up_pods"], cfg["down_pods"], cfg["max_pods"], cfg["min_pods"])
    step = max(cfg["poll_ns"], 0) + latency_ns[0]
    polls = int(horizon_ns // step) + 2 if step > 0 else 0
    ev = [e for e in oracle.simulate(p, tr, names, polls, init_replicas, oracle.Latency(*latency_ns))
          if e.t_poll_ns <= horizon_ns]
    r = {"pod_ms": 0, "backlog": 0, "first_up_ns": -1, "ups": 0, "downs": 0, "noop_ups": 0, "noop_downs": 0}
    prev_t, prev_r, prev_d = 0, oracle.int32(init_replicas), int(trace.depth[0])
    peak = prev_r
    run = {"sum": 0, "r": prev_r}

    def flush():
        x, y = run["sum"], max(run["r"], 1)
        r["backlog"] += x // y if x >= 0 else -((-x) // y)  # C++ integer division truncates
        run["sum"] = 0

    def acc(dt_ns, reps, d):
        dt_ms = dt_ns // 1_000_000
        r["pod_ms"] += reps * dt_ms
        if reps != run["r"]:
            flush()
            run["r"] = reps
        run["sum"] += d * dt_ms

    for e in ev:
        acc(e.t_poll_ns - prev_t, prev_r, prev_d)
        r["ups"] += e.up == "scaled"
        r["downs"] += e.down == "scaled"
        r["noop_ups"] += e.up == "noop"
        r["noop_downs"] += e.down == "noop"
        if e.up == "scaled" and r["first_up_ns"] < 0:
            r["first_up_ns"] = e.t_poll_ns
        prev_t, prev_r, prev_d = e.t_poll_ns, e.replicas, e.depth
        peak = max(peak, e.replicas)
    if horizon_ns > prev_t:
        acc(horizon_ns - prev_t, prev_r, prev_d)
    flush()
    r.update(final_replicas=prev_r, max_replicas=peak, polls=len(ev))
    return r
