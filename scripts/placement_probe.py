#!/usr/bin/env python3
"""Explicit CPU placements for 1-2 tracked queues (what makes the second queue
slower?). Each queue's worker thread and its endpoint process are pinned to given CPUs:
same CCD, SMT siblings, different CCDs, different sockets. One JSON line per run."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_sqs_autoscaler_amd.bench.latency import measure_detailed  # noqa: E402
from kube_sqs_autoscaler_amd.utils.topology import llc_domains  # noqa: E402

doms = llc_domains()
print(json.dumps({"llc_domains": len(doms), "first": doms[:2], "smt_of_1": None}), flush=True)
PLACEMENTS = {
    "q1": (1, {"workers": [[1]], "servers": [[3, 4]]}),
    "q2_same_ccd": (2, {"workers": [[1], [2]], "servers": [[3, 4], [5, 6]]}),
    "q2_smt_siblings": (2, {"workers": [[1], [129]], "servers": [[3, 4], [5, 6]]}),
    "q2_two_ccds": (2, {"workers": [[1], [9]], "servers": [[3, 4], [11, 12]]}),
    "q2_two_sockets": (2, {"workers": [[1], [65]], "servers": [[3, 4], [67, 68]]}),
    "q2_floating": (2, None),
    "q1_floating": (1, None),
}
for rnd in range(3):
    for name, (q, spec) in PLACEMENTS.items():
        d = measure_detailed(q, 2000, 200, "scale", pipeline=True, busy_poll_ns=25000, servers="processes",
                             affinity=json.dumps(spec) if spec else "none")
        d["placement"] = name
        d["round"] = rnd
        print(json.dumps(d), flush=True)
