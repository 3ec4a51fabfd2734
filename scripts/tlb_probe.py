"""The thread fleet's residual, seen from the worker threads' CPU split and the machine's IPIs.

N queues as threads of one process, each queue against its own fake endpoint process: per poll,
the workers' user and system CPU and minor faults (getrusage RUSAGE_THREAD as each exits), and the
machine's TLB-shootdown / function-call / reschedule IPIs over the timed run (/proc/interrupts).
If the penalty is system time with TLB IPIs rising with N, something in the process is
changing its mappings while the workers run (every thread of the address space is interrupted
to flush); if it is user time, it is memory contention in user space. One JSON line each;
three interleaved rounds of 2000 polls per queue."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.bench.latency import measure_detailed  # noqa: E402

servers = sys.argv[1] if len(sys.argv) > 1 else "processes"
for rnd in range(3):
    for q in (1, 4, 8):
        r = measure_detailed(q, 2000, 200, "scale", servers=servers if q > 1 else "process", busy_poll_ns=25_000)
        w = r["sched"]["autoscaler/ksa-worker"]
        print(json.dumps({"round": rnd, "queues": q, "p50_ms": r["summary"]["p50_ms"], "p90_ms": r["summary"]["p90_ms"],
                          "worker": w, "autoscaler_other": {k: v for k, v in r["sched"].items()
                                                            if k.startswith("autoscaler/") and k != "autoscaler/ksa-worker"},
                          "system": r["system"], "wall_s": r["wall_s"], "phases_median_us": r["phases_median_us"]}),
              flush=True)
