"""Thread fleet at 4 and 8 queues: one shared logger vs one per queue vs no log lines, on shared
and private worker file tables (r02j follow-up). One JSON line per measurement."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kube_sqs_autoscaler_amd.bench.latency import measure
for rnd in range(3):
    for q in (4, 8):
        for loggers, level in (("shared", "info"), ("per-queue", "info"), ("shared", "error")):
            for fdt in ("shared", "private"):
                os.environ["KSA_WORKER_FD_TABLE"] = fdt
                r = measure(q, 2000, 200, "scale", pipeline=True, busy_poll_ns=25_000, servers="processes", workers="threads",
                            loggers=loggers, log_level=level)
                print(json.dumps({"round": rnd, "queues": q, "loggers": loggers, "level": level, "fd_table": fdt,
                                  "p50_ms": r.summary()["p50_ms"]}), flush=True)
