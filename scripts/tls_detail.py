"""Per-phase medians and worker CPU of the default path over keep-alive TLS 1.3, next to plain
TCP, fake endpoints in their own process. One JSON line per configuration, two rounds."""
import json
import sys

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

from kube_sqs_autoscaler_amd.bench.latency import measure_detailed  # noqa: E402

for rnd in range(2):
    for tls in (False, True):
        r = measure_detailed(1, 4000, 400, "scale", servers="process", busy_poll_ns=25000, tls=tls)
        r["tls"] = tls
        r["round"] = rnd
        print(json.dumps(r), flush=True)
