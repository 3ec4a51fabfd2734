"""Is the thread fleet's residual automatic NUMA balancing?

Threads of one process share one address space; the kernel's NUMA balancing scans it and
unmaps pages so the next touch takes a hinting fault (and maybe a migration), and with workers
on both sockets the shared pages bounce. Worker processes each own an address space and never
share a page. This probe runs N queues as threads and as worker processes (each queue against
its own fake endpoint process) and records /proc/vmstat's numa_* counters around each run,
plus a third mode: threads whose task memory policy is MPOL_LOCAL (set before the workers
are created, so they inherit it) -- a policy without MPOL_F_MOF, which the balancing scan skips.
One JSON line per measurement; three interleaved rounds of 2000 polls per queue."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.bench.latency import measure  # noqa: E402

SYS_set_mempolicy = 238  # x86_64
MPOL_DEFAULT, MPOL_LOCAL = 0, 4
libc = ctypes.CDLL(None, use_errno=True)


def set_policy(mode: int) -> None:
    if libc.syscall(SYS_set_mempolicy, mode, None, 0) != 0:
        raise OSError(ctypes.get_errno(), "set_mempolicy")


def vmstat() -> dict:
    out = {}
    with open("/proc/vmstat") as f:
        for line in f:
            k, v = line.split()
            if k.startswith("numa_") or k.startswith("pgmigrate"):
                out[k] = int(v)
    return out


def read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError as e:
        return f"unreadable: {e}"


print(json.dumps({"numa_balancing": read("/proc/sys/kernel/numa_balancing"),
                  "nodes": read("/sys/devices/system/node/online")}), flush=True)
for rnd in range(3):
    for q in (1, 4, 8):
        for mode in ("threads", "threads_mpol_local", "processes"):
            set_policy(MPOL_LOCAL if mode == "threads_mpol_local" else MPOL_DEFAULT)
            before = vmstat()
            r = measure(q, 2000, 200, "scale", pipeline=True, busy_poll_ns=25_000, servers="processes",
                        workers="processes" if mode == "processes" else "threads")
            after = vmstat()
            set_policy(MPOL_DEFAULT)
            s = r.summary()
            delta = {k: after[k] - before.get(k, 0) for k in after if after[k] != before.get(k, 0)}
            print(json.dumps({"round": rnd, "queues": q, "mode": mode, "p50_ms": s["p50_ms"], "p90_ms": s["p90_ms"],
                              "samples": s["samples"], "vmstat_delta": delta}), flush=True)
