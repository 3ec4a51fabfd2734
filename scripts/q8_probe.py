"""Where does multi-queue latency go on the box? q1/q8 p50 under CPU-affinity variants."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r'''
import json, os, sys
sys.path.insert(0, sys.argv[1])
cpus = sys.argv[2]
if cpus != "all":
    a, b = map(int, cpus.split("-"))
    os.sched_setaffinity(0, range(a, b + 1))
from kube_sqs_autoscaler_amd.bench.latency import measure
q = int(sys.argv[3])
r = measure(q, 2000, 200, "scale", pipeline=True, busy_poll_ns=25_000)
print(json.dumps({"cpus": cpus, "q": q, **r.summary()}), flush=True)
'''

if __name__ == "__main__":
    try:
        numa = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        print(json.dumps({"lscpu": [l for l in numa.splitlines() if "NUMA" in l or "Socket" in l or "Thread" in l]}), flush=True)
    except OSError:
        pass
    for cpus in ("all", "0-15", "0-31", "0-7"):
        for q in (1, 8):
            subprocess.run([sys.executable, "-c", CHILD, ROOT, cpus, str(q)], check=True, timeout=120)
