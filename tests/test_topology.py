"""CPU placement helpers (kube_sqs_autoscaler_amd/utils/topology.py) on synthetic topologies: the
kernel's CPU-list format, one L3 domain per worker, distinct physical cores, and per-rank core
blocks that never overlap."""
import os

from kube_sqs_autoscaler_amd.utils import topology as t


def _sysfs(tmp_path, llc, smt):
    """A fake /sys/devices/system/cpu: llc and smt are lists of CPU lists."""
    for group, kind in ((llc, "cache/index3/shared_cpu_list"), (smt, "topology/thread_siblings_list")):
        for cpus in group:
            text = ",".join(str(c) for c in cpus)
            for c in cpus:
                p = tmp_path / f"cpu{c}" / kind
                p.parent.mkdir(parents=True, exist_ok=True)
                p.write_text(text + "\n")
    return str(tmp_path)


def test_parse_cpu_list():
    assert t.parse_cpu_list("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert t.parse_cpu_list("") == []


def test_domains_plans_and_rank_blocks(tmp_path, monkeypatch):
    # 2 L3 domains x 4 cores x 2 SMT threads: CPU c and c+16 are siblings
    llc = [[c for c in range(0, 4)] + [c + 16 for c in range(0, 4)],
           [c for c in range(4, 8)] + [c + 16 for c in range(4, 8)]]
    smt = [[c, c + 16] for c in range(8)]
    sys_cpu = _sysfs(tmp_path, llc, smt)
    import functools

    # plan_cores / plan_rank read sibling lists through physical_cores' default sysfs path
    monkeypatch.setattr(t, "physical_cores", functools.partial(t.physical_cores, sys_cpu=sys_cpu))
    allowed = sorted(c for d in llc for c in d)
    doms = t.llc_domains(allowed, sys_cpu=sys_cpu)
    assert doms == [sorted(llc[0]), sorted(llc[1])]
    assert t.plan(3, doms) == [doms[0], doms[1], doms[0]]
    cores = t.physical_cores(doms[0], sys_cpu=sys_cpu)
    assert cores == [[0, 16], [1, 17], [2, 18], [3, 19]]
    workers = t.plan_cores(8, doms)
    assert len({w[0] % 16 for w in workers}) == 8  # eight distinct physical cores

    # ranks: 2 per domain fit only without the spare first core
    plans = [t.plan_rank(r, 2, domains=doms) for r in range(2)]
    assert plans[0] == ([1], [2, 18, 3, 19]) and plans[1] == ([5], [6, 22, 7, 23])
    assert t.plan_rank(0, 4, domains=doms) is None  # 2 ranks x 3 cores do not fit in 4 cores
    small = [t.plan_rank(r, 2, endpoint_cores=1, domains=doms) for r in range(2)]
    used = [c for w, e in small for c in w + e]
    assert len(used) == len(set(used))
    assert t.plan_rank(2, 2, domains=doms) is None and t.plan_rank(-1, 2, domains=doms) is None
    assert os.path.isdir(sys_cpu)
