"""Where do the 8-queue fleet's threads run? Thread fleet vs worker processes.

While ``measure`` runs 8 queues (each against its own endpoint process), a sampler reads every
task's ``/proc/<pid>/task/<tid>/stat`` every few ms: for each worker thread (``ksa-worker``)
that is running, which CPU it is on, and whether another of our running threads (another
worker, or an endpoint thread ``ksa-serve``) is on the same physical core (SMT sibling) or
the same L3 domain. User-mode cycles per instruction rise when an SMT sibling is busy, which
would show as the thread fleet's extra user cycles at the same instruction count.
One JSON line per (round, mode)."""
import collections
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.bench.latency import measure  # noqa: E402


def topology():
    core, llc = {}, {}
    base = "/sys/devices/system/cpu"
    for d in os.listdir(base):
        if not (d.startswith("cpu") and d[3:].isdigit()):
            continue
        c = int(d[3:])
        try:
            with open(f"{base}/{d}/topology/core_id") as f:
                cid = int(f.read())
            with open(f"{base}/{d}/topology/physical_package_id") as f:
                pkg = int(f.read())
            core[c] = (pkg, cid)
        except OSError:
            continue
        try:
            with open(f"{base}/{d}/cache/index3/id") as f:
                llc[c] = (pkg, int(f.read()))
        except OSError:
            llc[c] = (pkg, -1)
    return core, llc


def snapshot():
    out = []  # (comm, pid, tid, cpu, state)
    for pid in os.listdir("/proc"):
        if not pid.isdigit():
            continue
        try:
            tids = os.listdir(f"/proc/{pid}/task")
        except OSError:
            continue
        for tid in tids:
            try:
                with open(f"/proc/{pid}/task/{tid}/stat") as f:
                    s = f.read()
            except OSError:
                continue
            comm = s[s.index("(") + 1:s.rindex(")")]
            if not comm.startswith("ksa-"):
                continue
            rest = s[s.rindex(")") + 2:].split()
            out.append((comm, int(pid), int(tid), int(rest[36]), rest[0]))
    return out


core, llc = topology()
for rnd in range(2):
    for workers in ("threads", "processes"):
        stats = collections.Counter()
        done = threading.Event()
        result = {}

        def run():
            result["r"] = measure(8, 20000, 200, "scale", pipeline=True, busy_poll_ns=25_000, servers="processes",
                                  workers=workers)
            done.set()

        th = threading.Thread(target=run)
        th.start()
        time.sleep(1.0)  # past endpoint start-up and warm-up
        while not done.is_set():
            snap = snapshot()
            running = [t for t in snap if t[4] == "R"]
            for comm, pid, tid, cpu, _ in running:
                if comm != "ksa-worker":
                    continue
                stats["worker_samples"] += 1
                others = [t for t in running if t[2] != tid]
                if any(core.get(o[3]) == core.get(cpu) for o in others):
                    stats["smt_sibling_busy"] += 1
                    if any(core.get(o[3]) == core.get(cpu) and o[0] == "ksa-worker" for o in others):
                        stats["smt_sibling_is_worker"] += 1
                if any(llc.get(o[3]) == llc.get(cpu) and o[0] == "ksa-worker" for o in others):
                    stats["llc_shared_with_worker"] += 1
                stats[f"pkg{core.get(cpu, (-1,))[0]}"] += 1
            time.sleep(0.003)
        th.join()
        s = result["r"].summary()
        n = max(1, stats["worker_samples"])
        print(json.dumps({"round": rnd, "workers": workers, "p50_ms": s["p50_ms"], "samples": stats["worker_samples"],
                          "smt_sibling_busy": round(stats["smt_sibling_busy"] / n, 3),
                          "smt_sibling_is_worker": round(stats["smt_sibling_is_worker"] / n, 3),
                          "llc_shared_with_worker": round(stats["llc_shared_with_worker"] / n, 3),
                          "by_package": {k: v for k, v in stats.items() if k.startswith("pkg")}}), flush=True)
