"""User-mode cycles, instructions and cache misses per poll of the thread fleet
(perf_event_open on the process' own threads; user mode only, as perf_event_paranoid allows).

Counters open on this thread with ``inherit`` before the fleet's worker threads are created,
so they count every worker (plus this thread, idle in join), warm-up polls included. Endpoint processes are started
first, in the BenchEnv, and never counted. If cycles per poll rise with N at the same
instructions per poll, the workers stall on memory that another core wrote.

Variants for 8 queues: ``shared`` (one clock and one logger for all queues, objects built on
the main thread: the CLI's layout), ``isolated`` (a clock and a logger per queue, each queue's
objects built on a thread of its own so they come from separate malloc arenas). One JSON line
per measurement, three interleaved rounds of 2000 polls per queue."""
import ctypes
import json
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.bench.latency import BenchEnv  # noqa: E402

libc = ctypes.CDLL(None, use_errno=True)
SYS_perf_event_open = 298
HW = 0  # PERF_TYPE_HARDWARE
SW = 1  # PERF_TYPE_SOFTWARE
EVENTS = {"cycles": (HW, 0), "instructions": (HW, 1), "cache_refs": (HW, 2), "cache_misses": (HW, 3),
          "task_clock_ns": (SW, 1)}


def open_counter(typ: int, config: int) -> int:
    attr = bytearray(128)
    struct.pack_into("IIQ", attr, 0, typ, 128, config)
    flags = (1 << 1) | (1 << 5) | (1 << 6)  # inherit, exclude_kernel, exclude_hv
    struct.pack_into("Q", attr, 40, flags)
    buf = ctypes.create_string_buffer(bytes(attr), 128)
    fd = libc.syscall(SYS_perf_event_open, buf, 0, -1, -1, 0)
    if fd < 0:
        raise OSError(ctypes.get_errno(), os.strerror(ctypes.get_errno()))
    return fd


def read_counter(fd: int) -> int:
    return struct.unpack("Q", os.read(fd, 8))[0]


VARIANTS = {"shared": {}, "isolated": {"build_on_threads": True, "clock_per_queue": True, "loggers": "per-queue"},
            "one_run": {}}
print(json.dumps({"perf_event_paranoid": open("/proc/sys/kernel/perf_event_paranoid").read().strip()}), flush=True)
quick = "--quick" in sys.argv  # 1 and 8 queues in the CLI layout only (for GLIBC_TUNABLES A/B runs)
configs = ((1, "shared"), (8, "shared")) if quick else ((1, "shared"), (8, "shared"), (8, "isolated"), (8, "one_run"))
tunables = os.environ.get("GLIBC_TUNABLES", "")
for rnd in range(2 if quick else 3):
    for q, variant in configs:
        env = BenchEnv(q, "scale", busy_poll_ns=25_000, servers="process" if q == 1 else "processes",
                       **VARIANTS[variant])
        try:
            # Counters open before the first run: a fleet's threads (HomeThread, one per runner,
            # kept across runs) are created by it, and only threads created after an inherited
            # counter opens are counted. one_run: warm-up and timed polls in one run.
            fds, errs = {}, {}
            for name, (typ, cfg) in EVENTS.items():
                try:
                    fds[name] = open_counter(typ, cfg)
                except OSError as e:
                    errs[name] = e.strerror
            before = {k: read_counter(fd) for k, fd in fds.items()}
            steps = 2000
            if variant != "one_run":
                env.run(200)
                env.clear()
            wall = env.run(steps + (200 if variant == "one_run" else 0))
            after = {k: read_counter(fd) for k, fd in fds.items()}
            for fd in fds.values():
                os.close(fd)
            res = env.collect(steps, wall)
            if variant == "one_run":
                res.samples = [x for r in env.runners for x in r.latencies()[-steps:]]
        finally:
            env.close()
        polls = q * (steps + 200)
        print(json.dumps({"round": rnd, "queues": q, "variant": variant, "glibc_tunables": tunables, "p50_ms": res.summary()["p50_ms"],
                          "user_per_poll": {k: round((after[k] - before[k]) / polls, 1) for k in fds}, "errors": errs}),
              flush=True)
