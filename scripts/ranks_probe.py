#!/usr/bin/env python3
"""N queues in one autoscaler process vs N autoscaler processes with one queue each, same
placement (queue i, its worker and its endpoint process on L3 domain i). If the processes stay
flat where the threads do not, the multi-queue cost is something the threads of one process
share. One JSON line per run."""
import json
import multiprocessing as mp
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rank(i, n, barrier, out, samples):
    from kube_sqs_autoscaler_amd.bench.latency import measure_detailed
    from kube_sqs_autoscaler_amd.utils.topology import plan_queue_ccds

    w, e = plan_queue_ccds(n)
    aff = json.dumps({"workers": [w[i]], "servers": [e[i]]})
    d = measure_detailed(1, samples, 200, "scale", sync=barrier.wait, pipeline=True, busy_poll_ns=25000,
                         servers="processes", affinity=aff)
    out.put((i, d["summary"]["p50_ms"], d["phases_median_us"], d["sched"]["autoscaler/ksa-worker"]))


def main():
    from kube_sqs_autoscaler_amd.bench.latency import measure_detailed

    print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith(("MALLOC", "GLIBC", "LD_", "OMP"))}}),
          flush=True)
    samples = 2000
    ctx = mp.get_context("spawn")
    for rnd in range(3):
        for n in (1, 8):
            d = measure_detailed(n, samples, 200, "scale", pipeline=True, busy_poll_ns=25000, servers="processes",
                                 affinity="ccd")
            print(json.dumps({"kind": "threads", "n": n, "round": rnd, "p50_ms": d["summary"]["p50_ms"],
                              "phases": d["phases_median_us"], "worker": d["sched"]["autoscaler/ksa-worker"]}),
                  flush=True)
            barrier, out = ctx.Barrier(n), ctx.Queue()
            ps = [ctx.Process(target=_rank, args=(i, n, barrier, out, samples)) for i in range(n)]
            for p in ps:
                p.start()
            res = sorted(out.get(timeout=300) for _ in ps)
            for p in ps:
                p.join()
            print(json.dumps({"kind": "processes", "n": n, "round": rnd, "p50_ms_per_rank": [r[1] for r in res],
                              "phases_rank0": res[0][2], "workers": [r[3] for r in res]}), flush=True)


if __name__ == "__main__":
    main()
