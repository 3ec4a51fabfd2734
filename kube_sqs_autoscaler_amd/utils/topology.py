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


def physical_cores(domain: List[int], sys_cpu: str = SYS_CPU) -> List[List[int]]:
    """The physical cores of one domain, each as its SMT sibling list (ordered by first CPU)."""
    allowed = set(domain)
    seen, cores = set(), []
    for c in sorted(domain):
        if c in seen:
            continue
        try:
            with open(f"{sys_cpu}/cpu{c}/topology/thread_siblings_list") as f:
                sib = sorted(allowed.intersection(parse_cpu_list(f.read())))
        except OSError:
            sib = [c]
        seen.update(sib)
        cores.append(sib)
    return cores


def plan_cores(n: int, domains: Optional[List[List[int]]] = None) -> List[List[int]]:
    """One logical CPU on a distinct physical core for each of n busy-polling workers, filling
    one L3 domain before the next (compact: whatever the workers share stays in one L3) and
    never putting two workers on SMT siblings of one core. Wraps around when n exceeds the
    cores available."""
    doms = domains if domains is not None else llc_domains()
    cores = [core for d in doms for core in physical_cores(d)]
    if not cores:
        return [[] for _ in range(n)]
    return [[cores[i % len(cores)][0]] for i in range(n)]


def plan_queue_ccds(n: int, endpoint_cores: int = 2,
                    domains: Optional[List[List[int]]] = None) -> "tuple[List[List[int]], List[List[int]]]":
    """Benchmark placement, one L3 domain per tracked queue (as one rank per queue gets):
    queue i's worker on the first core of domain i, its fake endpoints on the next
    ``endpoint_cores`` cores of that domain (SMT siblings included). Returns (workers, endpoints)."""
    doms = domains if domains is not None else llc_domains()
    workers, endpoints = [], []
    for i in range(n):
        cores = physical_cores(doms[i % len(doms)])
        workers.append([cores[0][0]])
        ep = [c for core in cores[1:1 + endpoint_cores] for c in core]
        endpoints.append(ep or cores[0])
    return workers, endpoints


def plan_rank(rank: int, nranks: int, endpoint_cores: int = 2,
              domains: Optional[List[List[int]]] = None) -> Optional["tuple[List[int], List[int]]"]:
    """Placement of one bench rank (one autoscaler process per GPU, its fake endpoints in the same
    process): rank r gets L3 domain r mod D, and within it a block of 1 + ``endpoint_cores``
    physical cores of its own -- the worker on the first core's first CPU, the fake servers on
    the rest (SMT siblings included) -- so ranks never share a core and each rank's round trips
    stay inside one L3. None when the domains cannot give every rank its own block (then the
    kernel places the threads)."""
    doms = domains if domains is not None else llc_domains()
    if not doms or rank < 0 or rank >= nranks:
        return None
    per = 1 + endpoint_cores
    d = rank % len(doms)
    slot = rank // len(doms)
    ranks_here = (nranks - d + len(doms) - 1) // len(doms)  # ranks that land on domain d
    cores = physical_cores(doms[d])
    if len(cores) < ranks_here * per:
        return None
    skip = 1 if len(cores) > ranks_here * per else 0  # leave a domain's first core (CPU 0's housekeeping) when it can
    block = cores[skip + slot * per:skip + (slot + 1) * per]
    return [block[0][0]], [c for core in block[1:] for c in core]
