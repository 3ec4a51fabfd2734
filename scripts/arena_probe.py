"""Does the thread fleet pay for queues' heap data sharing cache lines?

The thread fleet builds every queue's clients on the main thread, so their heap buffers come
from one malloc arena, interleaved queue after queue; a worker process builds only its own.
This runs N queues as threads with the objects built on the main thread (``main``) and each
queue's built on a thread of its own, all alive together so each gets its own arena
(``threads``, BenchEnv ``build_on_threads``), next to worker processes; each queue against its own fake
endpoint process. One JSON line per measurement, three interleaved rounds of 2000 polls."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.bench.latency import measure  # noqa: E402

for rnd in range(3):
    for q in (1, 4, 8):
        for mode in ("main", "threads", "processes"):
            kw = {} if mode == "processes" else {"build_on_threads": mode == "threads"}
            r = measure(q, 2000, 200, "scale", pipeline=True, busy_poll_ns=25_000, servers="processes",
                        workers="processes" if mode == "processes" else "threads", **kw)
            s = r.summary()
            print(json.dumps({"round": rnd, "queues": q, "build": mode, "p50_ms": s["p50_ms"], "p90_ms": s["p90_ms"],
                              "samples": s["samples"]}), flush=True)
