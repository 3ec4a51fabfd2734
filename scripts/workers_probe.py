#!/usr/bin/env python3
"""1/2/4/8 tracked queues as threads of one process vs --worker-processes, each queue against its
own endpoint process, three interleaved rounds. One JSON line per run."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kube_sqs_autoscaler_amd.bench.latency import measure  # noqa: E402

for rnd in range(3):
    for q in (1, 2, 4, 8):
        for workers in ("threads", "processes"):
            kw = dict(servers="processes") if workers == "threads" else {}
            r = measure(q, 2000, 200, "scale", workers=workers, pipeline=True, busy_poll_ns=25000, **kw)
            print(json.dumps({"round": rnd, "queues": q, "workers": workers, **r.summary(),
                              "signature_failures": r.signature_failures}), flush=True)
