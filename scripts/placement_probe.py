#!/usr/bin/env python3
"""CPU placements for 1/2/4/8 tracked queues (why do more queues in one process
cost more per poll?). Each layout pins every queue's worker thread and its endpoint process:

* ``none``  -- the kernel's placement;
* ``ccd``   -- one L3 domain (CCD) per queue: worker on its first core, endpoints on the next two;
* ``split`` -- workers on distinct physical cores of CCD 0, queue i's endpoints on core i of CCD 1;
* ``smt``   -- (2 queues) the two workers on SMT siblings of one core (the kernel sometimes does);
* ``sockets`` -- (2 queues) the two queues on different sockets.

One JSON line per run (`measure_detailed`)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.bench.latency import measure_detailed  # noqa: E402
from kube_sqs_autoscaler_amd.utils import topology  # noqa: E402


def layouts(q):
    doms = topology.llc_domains()
    out = {"none": "none", "ccd": "ccd"}
    c0, c1 = topology.physical_cores(doms[0]), topology.physical_cores(doms[1])
    if q <= len(c0) and q <= len(c1):
        out["split"] = json.dumps({"workers": [[c0[i][0]] for i in range(q)], "servers": [c1[i] for i in range(q)]})
    if q == 2 and len(c0[1]) > 1:
        out["smt"] = json.dumps({"workers": [[c0[1][0]], [c0[1][1]]], "servers": [c0[2], c0[3]]})
        far = topology.physical_cores(doms[len(doms) // 2])
        out["sockets"] = json.dumps({"workers": [[c0[1][0]], [far[1][0]]], "servers": [c0[2], far[2]]})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queues", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--samples", type=int, default=2000)
    ap.add_argument("--layouts", nargs="+", default=["none", "ccd", "split", "smt", "sockets"])
    a = ap.parse_args()
    print(json.dumps({"llc_domains": len(topology.llc_domains())}), flush=True)
    for rnd in range(a.rounds):
        for q in a.queues:
            for name, aff in layouts(q).items():
                if name not in a.layouts:
                    continue
                d = measure_detailed(q, a.samples, 200, "scale", pipeline=True, busy_poll_ns=25000, servers="processes",
                                     affinity=aff)
                d["layout"] = name
                d["round"] = rnd
                print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
