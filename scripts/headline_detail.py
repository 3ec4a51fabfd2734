"""Where the single-queue poll->patch time goes: per-phase medians plus the scheduler's view of
the worker thread and the fake endpoints (CPU per poll, voluntary context switches per poll)
for in-process fakes and for fakes in their own process. One JSON line per configuration."""
import json
import sys

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

from kube_sqs_autoscaler_amd.bench.latency import measure_detailed  # noqa: E402

for servers in ("shared", "process"):
    r = measure_detailed(1, 4000, 400, "scale", servers=servers, busy_poll_ns=25000)
    print(json.dumps(r), flush=True)
