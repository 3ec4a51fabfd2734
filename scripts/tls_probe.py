"""TLS latency rows on the box: default path with and without adaptive busy-poll, and the
reference-equivalent path, three interleaved rounds each (p50 ms)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kube_sqs_autoscaler_amd.bench.latency import measure  # noqa: E402

rows = {"tls_busy_poll": ("scale", True, 25_000), "tls_no_busy_poll": ("scale", True, 0),
        "tls_reference_equivalent": ("deployment", False, 0)}
out = {k: [] for k in rows}
for _ in range(3):
    for k, (mode, pl, bp) in rows.items():
        out[k].append(measure(1, 2000, 200, mode, pipeline=pl, busy_poll_ns=bp, tls=True).summary()["p50_ms"])
print(json.dumps(out), flush=True)
