"""CPU topology for thread placement (csrc/core/affinity.h).

``llc_domains()`` groups the CPUs this process may run on by the last-level cache they share
(sysfs ``cache/index3/shared_cpu_list``; on EPYC one L3 per 8-core CCD, SMT siblings included).
``plan(n)`` assigns n workers round-robin to those domains, so every worker -- and whatever it
talks to most -- stays on one CCD.
"""
from __future__ import annotations

import os
from typing import List, Optional

SYS_CPU = "/sys/devices/system/cpu"


def parse_cpu_list(text: str) -> List[int]:
    """Kernel CPU list format: ``0-7,128-135``."""
    out: List[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def llc_domains(allowed: Optional[List[int]] = None, sys_cpu: str = SYS_CPU) -> List[List[int]]:
    """CPU lists sharing one last-level cache, restricted to ``allowed`` (default: this process's
    affinity), ordered by their lowest CPU. Falls back to one domain of all allowed CPUs when
    sysfs has no cache topology."""
    cpus = sorted(allowed if allowed is not None else os.sched_getaffinity(0))
    allowed_set = set(cpus)
    seen, domains = set(), []
    for c in cpus:
        if c in seen:
            continue
        shared = None
        for index in ("index3", "index2"):
            try:
                with open(f"{sys_cpu}/cpu{c}/cache/{index}/shared_cpu_list") as f:
                    shared = parse_cpu_list(f.read())
                break
            except OSError:
                continue
        dom = sorted(allowed_set.intersection(shared)) if shared else [c]
        if not shared:
            return [cpus]
        seen.update(dom)
        domains.append(dom)
    return domains


def plan(n: int, domains: Optional[List[List[int]]] = None) -> List[List[int]]:
    """CPU list for each of n workers: worker i gets domain i mod len(domains)."""
    doms = domains if domains is not None else llc_domains()
    if not doms:
        return [[] for _ in range(n)]
    return [doms[i % len(doms)] for i in range(n)]
