"""Opt-in private file tables for Supervisor workers (KSA_WORKER_FD_TABLE=private,
unshare(CLONE_FILES), csrc/core/runner.h): their sockets never appear in, leak into, or get
closed through the process' shared table, and the clients keep working across runs and from
other threads afterwards."""
import os

from kube_sqs_autoscaler_amd.bench.latency import BenchEnv


def _sockets(path="/proc/self/fd"):
    n = 0
    for fd in os.listdir(path):
        try:
            if os.readlink(f"{path}/{fd}").startswith("socket:"):
                n += 1
        except OSError:
            pass
    return n


def test_worker_sockets_stay_off_the_shared_table(nat, monkeypatch):
    monkeypatch.setenv("KSA_WORKER_FD_TABLE", "private")  # read by every Supervisor env.run() builds
    env = BenchEnv(4, "scale", servers="processes")  # endpoints in another process: only client sockets here
    try:
        assert nat.Supervisor().private_files
        before = _sockets()
        for _ in range(3):  # three runs, three supervisors, reconnecting each time
            env.run(50)
            assert _sockets() == before
        res = env.collect(50, 1.0)
        assert len(res.samples) > 0 and res.signature_failures == 0
        # the same clients from this (main) thread: they dial on this table, and work
        assert env.sqs_apis[0] is not None
        r = env.runners[0]
        assert r.sqs.num_messages() in (0, 200)
        assert _sockets() == before + 1
    finally:
        env.close()


def test_private_tables_are_opt_in(nat, monkeypatch):
    monkeypatch.delenv("KSA_WORKER_FD_TABLE", raising=False)
    assert not nat.Supervisor().private_files
    monkeypatch.setenv("KSA_WORKER_FD_TABLE", "shared")
    assert not nat.Supervisor().private_files
    s = nat.Supervisor()
    s.private_files = True
    assert s.private_files


def test_private_tables_under_dropped_connections(nat):
    """Workers on private tables reconnect on their own table when the servers drop every
    connection mid-run; no socket is left behind and the replicas stay in bounds."""
    import threading
    import time

    env = BenchEnv(4, "scale", servers="per-queue")  # in-process fakes: they can drop connections
    try:
        time.sleep(0.1)
        before = _sockets()
        sup = nat.Supervisor()
        sup.private_files = True
        for r in env.runners:
            sup.add(r)
        stop = threading.Event()

        def chaos():
            while not stop.is_set():
                for s in env.sqs_servers + env.kube_servers:
                    s.drop_connections()
                time.sleep(0.005)

        t = threading.Thread(target=chaos)
        t.start()
        try:
            sup.start(400)
            sup.join()
        finally:
            stop.set()
            t.join()
        assert sum(r.stats()["polls"] for r in env.runners) == 4 * 400
        deadline = time.time() + 5  # the servers close their side once they see the clients' EOF
        while _sockets() > before and time.time() < deadline:
            time.sleep(0.05)
        assert _sockets() <= before
        res = env.collect(400, 1.0)
        assert all(1 <= x <= 8 for x in res.final_replicas)
    finally:
        env.close()
