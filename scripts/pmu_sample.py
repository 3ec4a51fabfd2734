"""Where the thread fleet's extra user-mode cycles go: a sampling profile of the worker threads.

perf_event_open (user mode only, as perf_event_paranoid allows) in sampling mode on each
worker thread (an inherited per-task event cannot have a ring buffer), attached right after
the fleet starts. Samples user cycles and cache misses at 1 and 8
queues (threads, each queue against its own endpoint process), keeps (ip -> count), and writes
the histogram plus /proc/self/maps to gpurun_out/ so the addresses can be symbolised against
the same .so files afterwards (scripts/pmu_symbolize.py). One JSON file per configuration."""
import collections
import ctypes
import json
import mmap
import os
import struct
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.bench.latency import BenchEnv  # noqa: E402

libc = ctypes.CDLL(None, use_errno=True)
SYS_perf_event_open = 298
PAGE = mmap.PAGESIZE
DATA_PAGES = 128  # 512 KiB of rings in all (the unprivileged mlock limit), split over the workers
SAMPLE_IP, SAMPLE_TID = 1 << 0, 1 << 1
RECORD_SAMPLE, RECORD_LOST = 9, 2
EVENTS = ({"cpu_clock": (1, 0, 20_000)} if os.environ.get("KSA_PMU_SW") else
          {"cycles": (0, 0, 200_000), "cache_misses": (0, 3, 200)})


def open_sampler(typ: int, config: int, period: int, tid: int) -> int:
    attr = bytearray(128)
    struct.pack_into("IIQQQQQ", attr, 0, typ, 128, config, period, SAMPLE_IP | SAMPLE_TID, 0,
                     (1 << 5) | (1 << 6))  # exclude_kernel, exclude_hv
    buf = ctypes.create_string_buffer(bytes(attr), 128)
    fd = libc.syscall(SYS_perf_event_open, buf, tid, -1, -1, 0)
    if fd < 0:
        raise OSError(ctypes.get_errno(), os.strerror(ctypes.get_errno()))
    return fd


def worker_tids() -> list:
    out = []
    for t in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{t}/comm") as f:
                if f.read().strip() == "ksa-worker":
                    out.append(int(t))
        except OSError:
            pass
    return out


def drain(ring: mmap.mmap, pages: int) -> tuple:
    head = struct.unpack_from("Q", ring, 1024)[0]
    data_off, data_size = struct.unpack_from("QQ", ring, 1040)
    if data_off == 0:
        data_off, data_size = PAGE, pages * PAGE
    hist, lost, pos = collections.Counter(), 0, 0
    if head > data_size:
        lost = -1  # wrapped: the oldest records are gone; count what is left
        pos = head - data_size
    while pos < head:
        base = data_off + (pos % data_size)
        typ, _misc, size = struct.unpack_from("IHH", ring, base)
        if size == 0:
            break
        if typ == RECORD_SAMPLE:
            ip = struct.unpack_from("Q", ring, base + 8)[0]
            hist[ip] += 1
        elif typ == RECORD_LOST:
            lost += struct.unpack_from("Q", ring, base + 16)[0]
        pos += size
    return hist, lost


os.makedirs("gpurun_out/pmu_sample", exist_ok=True)
TLS = "--tls" in sys.argv  # one queue over keep-alive TLS 1.3 instead of 1 and 8 plain queues
for q in ((1,) if TLS else (1, 8)):
    pages = DATA_PAGES // q  # the rings of all workers together stay within the mlock limit
    for event, (typ, cfg, period) in EVENTS.items():
        env = BenchEnv(q, "scale", busy_poll_ns=25_000, servers="process" if q == 1 else "processes", tls=TLS)
        try:
            env.run(200)
            env.clear()
            # env.run, with samplers attached to the worker threads once they exist
            steps = 20000  # long enough to attach
            sup = env.nat.Supervisor()
            for r in env.runners:
                sup.add(r)
            t0 = time.perf_counter()
            sup.start(steps)
            tids = []
            while len(tids) < q and time.perf_counter() - t0 < 5:
                tids = worker_tids()
            rings = []
            for tid in tids:
                try:
                    fd = open_sampler(typ, cfg, period * q, tid)  # 8 rings 1/8 the size: no wrap
                except ProcessLookupError:  # a thread of the warm-up run, gone since the listing
                    continue
                rings.append((fd, mmap.mmap(fd, (1 + pages) * PAGE, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)))
            sup.join()
            wall = time.perf_counter() - t0
            hist, lost = collections.Counter(), 0
            for fd, ring in rings:
                h, lo = drain(ring, pages)
                hist.update(h)
                lost = -1 if lo < 0 or lost < 0 else lost + lo
                ring.close()
                os.close(fd)
            res = env.collect(steps, wall)
            with open("/proc/self/maps") as f:
                maps_text = f.read()
        finally:
            env.close()
        out = {"queues": q, "tls": TLS, "event": event, "period": period * q, "polls": q * steps, "p50_ms": res.summary()["p50_ms"],
               "threads_sampled": len(rings), "samples": sum(hist.values()), "lost": lost,
               "hist": {hex(k): v for k, v in hist.most_common()}, "maps": maps_text}
        with open(f"gpurun_out/pmu_sample/q{q}{'_tls' if TLS else ''}_{event}.json", "w") as f:
            json.dump(out, f)
        print(json.dumps({k: out[k] for k in ("queues", "event", "polls", "p50_ms", "threads_sampled", "samples", "lost")}),
              flush=True)
