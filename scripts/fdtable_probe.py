"""N queues as threads of one process with the workers on the shared file table vs each on a
private one (Supervisor, KSA_WORKER_FD_TABLE), next to N worker processes; each queue against
its own fake endpoint process. Three interleaved rounds of 2000 polls per queue; one JSON line
per measurement. ``--ccd``: queue i's worker and its endpoint process pinned to L3 domain i
(utils/topology.py), for threads and processes alike."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.bench.latency import measure  # noqa: E402

affinity = "ccd" if "--ccd" in sys.argv else "none"
for rnd in range(3):
    for q in (1, 2, 4, 8):
        for mode in ("shared", "private", "processes"):
            os.environ["KSA_WORKER_FD_TABLE"] = "shared" if mode == "shared" else "private"  # Supervisor reads it
            workers = "processes" if mode == "processes" else "threads"
            r = measure(q, 2000, 200, "scale", pipeline=True, busy_poll_ns=25_000, servers="processes", workers=workers,
                        affinity=affinity)
            s = r.summary()
            print(json.dumps({"round": rnd, "queues": q, "mode": mode, "affinity": affinity, "p50_ms": s["p50_ms"], "p90_ms": s["p90_ms"],
                              "samples": s["samples"]}), flush=True)
