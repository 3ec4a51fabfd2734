"""The benchmark's fake SQS + kube-apiserver endpoints, in a process of their own.

``python -m kube_sqs_autoscaler_amd.bench.fakeserve --queues Q --pairs N`` starts N fake SQS +
apiserver pairs serving Q bench queues (latency.start_fake_endpoints), prints one JSON line
with their URLs and certificates, then answers commands on stdin, one per line:
``stats`` -> a JSON line of request / connection / signature counters, the replicas of every
bench Deployment, and this process's thread count and CPU time (``threads``, ``cpu_ns``); ``timings`` -> a JSON line with every served request's (wake-up delay, service
time) in ns, per endpoint kind (HttpServer::timings), and clears them; ``quit`` -> stop the
servers and exit (EOF on stdin does the same).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

from .latency import deployment_name, start_fake_endpoints, thread_count


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--queues", type=int, required=True)
    ap.add_argument("--pairs", type=int, default=1)
    ap.add_argument("--tls", type=int, default=0)
    ap.add_argument("--sqs-latency-ns", type=int, default=0)
    ap.add_argument("--kube-latency-ns", type=int, default=0)
    ap.add_argument("--cpus", default="", help="JSON list: the CPU list of each pair's threads")
    ap.add_argument("--queue-offset", type=int, default=0, help="number of the first bench queue served")
    ap.add_argument("--only", default="both", choices=["both", "sqs", "kube"],
                    help="serve one kind alone (the bench's split endpoints: SQS and the apiserver in two processes)")
    ap.add_argument("--hot", action="store_true", help="busy-polling servers that never sleep (HttpServer::set_hot)")
    ap.add_argument("--timing", action="store_true", help="record per-request timings (HttpServer::set_timing)")
    a = ap.parse_args(argv)
    cpus = json.loads(a.cpus) if a.cpus else None
    sqs, kube = start_fake_endpoints(a.queues, a.pairs, bool(a.tls), a.sqs_latency_ns, a.kube_latency_ns, cpus,
                                     a.queue_offset, hot=a.hot, timing=a.timing, only=a.only)
    try:
        info = {"pid": os.getpid(), "sqs": [{"url": s.url, "cert_pem": s.cert_pem} for s in sqs],
                "kube": [{"url": k.url, "cert_pem": k.cert_pem} for k in kube]}
        print(json.dumps(info), flush=True)
        for line in sys.stdin:
            cmd = line.strip()
            if cmd == "stats":
                print(json.dumps({
                    "sqs_requests": sum(s.requests() for s in sqs), "kube_requests": sum(k.requests() for k in kube),
                    "sqs_connections": sum(s.connections() for s in sqs),
                    "kube_connections": sum(k.connections() for k in kube),
                    "signature_failures": sum(s.signature_failures() for s in sqs),
                    "replicas": [kube[q % len(kube)].replicas("bench", deployment_name(a.queue_offset + q))
                                 for q in range(a.queues)] if kube else [],
                    "threads": thread_count(), "cpu_ns": time.process_time_ns(),
                }), flush=True)
            elif cmd == "timings":
                out = {"sqs": [t for s in sqs for t in s.timings()], "kube": [t for k in kube for t in k.timings()]}
                for s in (*sqs, *kube):
                    s.clear_timings()
                print(json.dumps(out), flush=True)
            elif cmd == "quit":
                break
    finally:
        for s in sqs:
            s.stop()
        for k in kube:
            k.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
