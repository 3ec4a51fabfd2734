"""Is the first headline measurement of a fresh process slow, and why? p50 of 5 back-to-back
1-queue measurements, with and without HIP runtime initialisation first (argv[1] = gpu|nogpu)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

t0 = time.perf_counter()
if sys.argv[1] == "gpu":
    import torch

    torch.cuda.set_device(0)
    torch.cuda.synchronize()
from kube_sqs_autoscaler_amd.bench.latency import measure  # noqa: E402

out = []
for i in range(5):
    r = measure(1, 2000, 200, "scale", pipeline=True, busy_poll_ns=25_000)
    out.append((round(time.perf_counter() - t0, 2), r.summary()["p50_ms"]))
print(json.dumps({"mode": sys.argv[1], "t_s_p50_ms": out}), flush=True)
