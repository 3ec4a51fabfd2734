"""Closed-loop what-if sweep: autoscaler settings against a queue the replicas actually drain.

Extension (an operator tool, not a reference capability). :mod:`.sweep` replays a recorded depth
trace, so a candidate's decisions cannot change the depth it sees. Tuning cool-downs for GPU
workers that take minutes to start needs the feedback loop: more replicas drain the queue, which
changes the next decision. ``csrc/sim/queue_sim.h`` models it:

* arrivals at a piecewise-constant rate (msgs/s), random per poll interval (integer normal
  approximation of Poisson -- an Irwin-Hall sum of four 16-bit draws -- counter-based per seed,
  the same seeds for every configuration);
* each ready pod drains ``service_rate`` msgs/s; a scale-up's pods take work only
  ``startup`` after the write returned; a scale-down removes starting pods first;
* the decisions are the reference's rules (``KSA_DECIDE`` in ``policy_sim.h``, shared with the open-loop
  simulator that is exact against ``models/oracle.py``), on the same virtual clock and latency
  model.

The gfx950 kernel (``csrc/hip/queue_sweep.hip``) runs one (configuration, seed) per lane; the CPU
path runs the same header on threads; both are bit-identical. :func:`reference_lane` is an
independent pure-Python statement of the model for the tests.

Per configuration the result reports means and 95th percentiles over the seeds of: pod cost,
mean backlog, time above the SLO backlog, peak backlog, and scaling activity.
"""
from __future__ import annotations

import csv
import ctypes
import math
import os
from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import numpy as np

from .sweep import PARAM_FIELDS, _gpu_lib as _open_loop_lib, gpu_available

OUT64 = ("pod_ms", "backlog_msg_ms", "violation_ms", "peak_backlog", "arrived", "served", "final_backlog")
OUT32 = ("ups", "downs", "final_replicas", "max_replicas", "polls")
MAX_LANE_POLLS = 2e11  # work budget (lanes x polls), as sweep.MAX_TOTAL_POLLS
S = 1_000_000_000


@dataclass
class ArrivalTrace:
    """Piecewise-constant arrival rate: segment i starts at ``t_ms[i]`` (ms) with ``rate`` msgs/s."""

    t_ms: np.ndarray  # int64, sorted, t_ms[0] == 0
    rate_milli: np.ndarray  # int64, msgs/s x 1000

    def __post_init__(self):
        self.t_ms = np.ascontiguousarray(self.t_ms, dtype=np.int64)
        self.rate_milli = np.ascontiguousarray(self.rate_milli, dtype=np.int64)
        if self.t_ms.ndim != 1 or self.t_ms.shape != self.rate_milli.shape or len(self.t_ms) == 0:
            raise ValueError("arrival trace needs equal-length non-empty 1-D t_ms and rates")
        if self.t_ms[0] != 0 or np.any(np.diff(self.t_ms) < 0):
            raise ValueError("arrival trace times must start at 0 and be sorted")
        if np.any(self.rate_milli < 0) or np.any(self.rate_milli > 10**9):
            raise ValueError("arrival rates must be within [0, 1e6] msgs/s")

    @staticmethod
    def from_segments(segments: Sequence[Tuple[float, float]]) -> "ArrivalTrace":
        """``[(start_seconds, msgs_per_second), ...]``."""
        return ArrivalTrace(np.array([round(t * 1000) for t, _ in segments]),
                            np.array([round(r * 1000) for _, r in segments]))

    @staticmethod
    def from_csv(path: str) -> "ArrivalTrace":
        """``seconds,msgs_per_second`` rows (a header row is skipped)."""
        rows: List[Tuple[float, float]] = []
        with open(path, newline="") as f:
            for rec in csv.reader(f):
                if not rec or rec[0].strip().startswith("#"):
                    continue
                try:
                    rows.append((float(rec[0]), float(rec[1])))
                except ValueError:
                    if rows:
                        raise
        if not rows:
            raise ValueError(f"no seconds,rate rows in {path}")
        t0 = rows[0][0]
        return ArrivalTrace.from_segments([(t - t0, r) for t, r in rows])


@dataclass
class QueueModel:
    service_rate: float  # msgs/s drained per ready pod
    startup_ns: int = 60 * S  # scale-up write -> pods taking work
    slo_backlog: int = 1000  # msgs; time above it counts as a violation
    init_backlog: int = 0

    def packed(self) -> np.ndarray:
        if not 0 <= self.service_rate <= 1e6:
            raise ValueError("service rate must be within [0, 1e6] msgs/s per pod")
        if not 0 <= self.startup_ns <= 86400 * S:
            raise ValueError("startup delay must be within [0, 24 h]")
        if not 0 <= self.init_backlog <= 10**12 or self.slo_backlog < 0:
            raise ValueError("backlogs must be non-negative (initial backlog <= 1e12)")
        return np.array([round(self.service_rate * 1000), self.startup_ns, self.slo_backlog, self.init_backlog],
                        dtype=np.int64)


@dataclass
class ClosedLoopResult:
    params: np.ndarray  # (9, m)
    seeds: int
    out: Dict[str, np.ndarray]  # each (m, seeds)
    device: str
    horizon_ns: int
    kernel_ms: float = 0.0
    fast_arith: bool = False  # the native path ran queue_sim.h's FastArith (bounds proven)
    ms_clock: bool = False  # ... with its decisions on the millisecond clock (simulate_queue_ms)

    def __len__(self) -> int:
        return self.params.shape[1]

    def config(self, i: int) -> Dict[str, int]:
        return {f: int(self.params[k, i]) for k, f in enumerate(PARAM_FIELDS)}

    def summary(self) -> Dict[str, np.ndarray]:
        """Per-configuration means and 95th percentiles over the seeds."""
        h_ms = max(self.horizon_ns // 1_000_000, 1)
        mean_backlog = self.out["backlog_msg_ms"] / h_ms
        return {
            "pod_hours_mean": self.out["pod_ms"].mean(axis=1) / 3.6e6,
            "backlog_mean": mean_backlog.mean(axis=1),
            "backlog_p95": np.percentile(mean_backlog, 95, axis=1),
            "violation_s_mean": self.out["violation_ms"].mean(axis=1) / 1e3,
            "violation_s_p95": np.percentile(self.out["violation_ms"], 95, axis=1) / 1e3,
            "peak_backlog_p95": np.percentile(self.out["peak_backlog"], 95, axis=1),
            "ups_mean": self.out["ups"].mean(axis=1),
            "downs_mean": self.out["downs"].mean(axis=1),
            "max_replicas_max": self.out["max_replicas"].max(axis=1),
        }

    def row(self, i: int) -> Dict[str, float]:
        r: Dict[str, float] = dict(self.config(i))
        for k, v in self.summary().items():
            r[k] = float(v[i])
        return r


def _queue_lib():
    lib = _open_loop_lib()
    if not getattr(lib, "_queue_ready", False):
        lib.ksa_queue_sweep_gpu.restype = ctypes.c_int
        lib.ksa_queue_sweep_gpu.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int32,
                                            ctypes.POINTER(ctypes.c_int32)]
        lib.ksa_queue_sweep_last_error.restype = ctypes.c_char_p
        lib._queue_ready = True
    return lib


def run(trace: ArrivalTrace, params: np.ndarray, model: QueueModel, init_replicas: int = 1,
        horizon_ns: int = 3600 * S, latency_ns: Tuple[int, int, int] = (1_000_000, 1_000_000, 1_000_000),
        seeds: int = 32, seed0: int = 1, device: str = "auto", threads: int = 0, gpu_index: int = 0,
        arith: str = "auto") -> ClosedLoopResult:
    """Runs the sweep. ``arith``: ``"auto"`` runs queue_sim.h's FastArith (plain integer ops,
    32-bit times) when ``fast_path_ok`` proves that no quantity can saturate -- identical results --
    with the decisions on 32-bit millisecond clocks when every period and latency is a whole
    millisecond (``ms_clock_ok``), and the saturating arithmetic otherwise; ``"saturating"``
    always runs the latter; ``"fast-ns"`` allows FastArith but keeps the nanosecond decision
    clock (A/B and tests)."""
    codes = {"auto": 0, "saturating": 1, "fast-ns": 2}
    if arith not in codes:
        raise ValueError(f"arith must be auto, saturating or fast-ns, not {arith!r}")
    code = codes[arith]
    params = np.ascontiguousarray(params, dtype=np.int64)
    if params.ndim != 2 or params.shape[0] != len(PARAM_FIELDS):
        raise ValueError("params must have shape (9, m); build it with sweep.grid()")
    if not 0 < horizon_ns <= 30 * 86400 * S:
        raise ValueError("horizon must be within (0, 30 days]")
    if any(not 0 <= int(x) <= 3600 * S for x in latency_ns):
        raise ValueError("latencies must be within [0, 1 h]")
    if np.any((params[0] <= 0) & (latency_ns[0] <= 0)):
        raise ValueError("a zero poll period needs a positive SQS latency (time would not advance)")
    if not 1 <= seeds <= 1 << 20:
        raise ValueError("seeds must be within [1, 2^20]")
    packed = model.packed()
    lat = np.array(latency_ns, dtype=np.int64)
    m = params.shape[1]
    step = np.maximum(params[0], 0) + latency_ns[0]
    est = float(np.sum(horizon_ns / step)) * seeds
    if est > MAX_LANE_POLLS:
        raise ValueError(f"sweep too large: ~{est:.3g} simulated polls (limit {MAX_LANE_POLLS:.3g})")
    if device == "auto":
        device = "gpu" if gpu_available() else "cpu"
    lanes = m * seeds
    if device == "gpu":
        lib = _queue_lib()
        out64 = np.zeros((len(OUT64), lanes), dtype=np.int64)
        out32 = np.zeros((len(OUT32), lanes), dtype=np.int32)
        ms = ctypes.c_double(0)
        used = ctypes.c_int32(0)
        rc = lib.ksa_queue_sweep_gpu(gpu_index, trace.t_ms.ctypes.data, trace.rate_milli.ctypes.data, len(trace.t_ms),
                                     init_replicas, horizon_ns, lat.ctypes.data, packed.ctypes.data, params.ctypes.data,
                                     m, seeds, seed0, out64.ctypes.data, out32.ctypes.data, ctypes.byref(ms),
                                     code, ctypes.byref(used))
        if rc != 0:
            raise RuntimeError("GPU closed-loop sweep failed: " + (lib.ksa_queue_sweep_last_error() or b"").decode())
        kernel_ms = ms.value
        fast, ms_clock = bool(used.value & 1), bool(used.value & 2)
    elif device == "cpu":
        from ..ops import native

        out64, out32, fast, ms_clock = native().queue_sweep_cpu(trace.t_ms, trace.rate_milli, init_replicas, horizon_ns,
                                                                lat, packed, params, seeds, seed0,
                                                                threads or (os.cpu_count() or 8), code)
        kernel_ms = 0.0
    else:
        raise ValueError(f"device must be auto, gpu or cpu, not {device!r}")
    out = {k: out64[i].reshape(m, seeds) for i, k in enumerate(OUT64)}
    out.update({k: out32[i].reshape(m, seeds) for i, k in enumerate(OUT32)})
    return ClosedLoopResult(params, seeds, out, device, horizon_ns, kernel_ms, fast, ms_clock)


# ---------------------------------------------------------------------------------------------
# Independent pure-Python statement of the model (tests compare the native paths against it).

_MASK64 = (1 << 64) - 1
_SAT = 1 << 62


def _mix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK64
    return z ^ (z >> 31)


def _sample(mean: int, seed: int, k: int) -> int:
    if mean <= 0:
        return 0
    w = _mix64((seed * 0xD1B54A32D192ED03 + k) & _MASK64)
    u = sum((w >> (16 * i)) & 0xFFFF for i in range(4)) - 131070  # Irwin-Hall(4), centred
    z = (u * 113512) >> 16  # x sqrt(3): standard deviation 2^16; >> floors, as the C++ shift
    sd = math.isqrt(mean) * 1000  # micro-messages: 1000 sqrt(mean)
    a = mean + ((sd * z) >> 16)  # floors, as the C++ arithmetic shift
    return max(a, 0)


def _trunc_div(a: int, b: int) -> int:
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def _i32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


def reference_lane(trace: ArrivalTrace, cfg: Dict[str, int], model: QueueModel, init_replicas: int, horizon_ns: int,
                   latency_ns: Tuple[int, int, int], seed: int) -> Dict[str, int]:
    """One (configuration, seed) of the closed-loop model, in plain Python integers."""
    t_ms = [int(x) for x in trace.t_ms]
    rate = [int(x) for x in trace.rate_milli]
    service = round(model.service_rate * 1000)
    sqs, get, upd = latency_ns
    bound = 1 << 61
    period = min(max(cfg["poll_ns"], 0), bound)
    up_cool = max(min(cfg["up_cool_ns"], bound), -bound)
    down_cool = max(min(cfg["down_cool_ns"], bound), -bound)
    max32, min32 = _i32(cfg["max_pods"]), _i32(cfg["min_pods"])
    up32, down32 = _i32(cfg["up_pods"]), _i32(cfg["down_pods"])
    r = dict(pod_ms=0, backlog_msg_ms=0, violation_ms=0, peak_backlog=0, arrived=0, served=0, final_backlog=0, ups=0,
             downs=0, final_replicas=0, max_replicas=init_replicas, polls=0)
    st = {"q": model.init_backlog * 10**6, "ready": init_replicas, "pending": 0, "pending_at": 0, "draws": 0}

    def sat_add(a: int, b: int) -> int:  # the C++ accumulators saturate at 2^62
        return min(a + b, _SAT)

    def sat_mul(a: int, b: int) -> int:
        return 0 if a <= 0 or b <= 0 else min(a * b, _SAT)

    def per_ms(x_milli: int, dt: int) -> int:  # milli-msgs/s x ms = micro-messages
        return sat_mul(x_milli, dt)

    def expected(t0: int, t1: int) -> int:
        total = 0
        for i, start in enumerate(t_ms):
            end = t_ms[i + 1] if i + 1 < len(t_ms) else max(t1, start)
            a, b = max(start, t0), min(end, t1)
            if b > a:
                total = sat_add(total, per_ms(rate[i], b - a))
        return total

    def advance(t0: int, t1: int, replicas: int) -> None:
        if t1 <= t0:
            return
        dt = t1 - t0
        q0 = st["q"] // 10**6
        r["pod_ms"] = sat_add(r["pod_ms"], sat_mul(replicas, dt))
        r["backlog_msg_ms"] = sat_add(r["backlog_msg_ms"], sat_mul(q0, dt))
        if q0 > model.slo_backlog:
            r["violation_ms"] += dt
        a = _sample(expected(t0, t1), seed, st["draws"])
        st["draws"] += 1
        st["q"] = sat_add(st["q"], a)
        r["arrived"] = sat_add(r["arrived"], a)
        cap = sat_mul(st["ready"], per_ms(service, dt))
        if st["pending"] > 0 and st["pending_at"] < t1:
            cap = sat_add(cap, sat_mul(st["pending"], per_ms(service, t1 - max(st["pending_at"], t0))))
        served = min(st["q"], cap)
        st["q"] -= served
        r["served"] = sat_add(r["served"], served)
        if st["pending"] > 0 and st["pending_at"] <= t1:
            st["ready"] += st["pending"]
            st["pending"] = 0

    now = last_up = last_down = 0
    replicas = init_replicas
    prev_ms = 0
    while (period > 0 or sqs > 0) and r["polls"] < (1 << 26):
        t_poll = now + period
        if t_poll > horizon_ns:
            break
        advance(prev_ms, t_poll // 1_000_000, replicas)
        prev_ms = t_poll // 1_000_000
        now = t_poll
        r["polls"] += 1
        d = st["q"] // 10**6
        now += sqs
        before = replicas
        cont = False
        if d >= cfg["up_msgs"]:  # main.go:51
            if last_up + up_cool > now:
                cont = True
            else:
                now += get
                if replicas < max32:
                    replicas = min(_i32(replicas + up32), max32)
                    now += upd
                    r["ups"] += 1
                last_up = now
        if not cont and d <= cfg["down_msgs"]:  # main.go:65
            if not last_down + down_cool > now:
                now += get
                if replicas > min32:
                    replicas = max(_i32(replicas - down32), min32)
                    now += upd
                    r["downs"] += 1
                last_down = now
        delta = _i32(replicas - before)
        if delta > 0:
            st["pending"] += delta
            st["pending_at"] = _trunc_div(now + model.startup_ns, 1_000_000)
        elif delta < 0:
            drop = -delta
            take = min(drop, st["pending"])
            st["pending"] -= take
            st["ready"] = max(st["ready"] - (drop - take), 0)
        r["max_replicas"] = max(r["max_replicas"], replicas)
        r["peak_backlog"] = max(r["peak_backlog"], st["q"] // 10**6)
    horizon_ms = horizon_ns // 1_000_000
    if horizon_ms > prev_ms:
        advance(prev_ms, horizon_ms, replicas)
    r.update(final_replicas=replicas, final_backlog=st["q"] // 10**6, arrived=r["arrived"] // 10**6,
             served=r["served"] // 10**6)
    return r
