"""HBM probe benchmark (profiled by rocprofv3 in scripts/gpu_check.sh): one JSON line per size."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.ops import gpu  # noqa: E402

for size in (64 << 20, 1 << 30, 4 << 30):
    h = gpu.health_check(0, size, reps=5)
    print(json.dumps({"bytes": h.bytes, "ok": h.ok, "write_GBps": round(h.write_gbps, 1), "read_verify_GBps": round(h.read_gbps, 1),
                      "fill_ms": round(h.fill_ms, 4), "verify_ms": round(h.verify_ms, 4)}), flush=True)
