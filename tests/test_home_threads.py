"""Each Runner polls on one OS thread for its whole life (HomeThread, csrc/core/runner.h), across
Supervisor runs: a replaced thread would hand its malloc arena to another queue's new thread
and interleave two queues' hot buffers (docs/HISTORY.md, r02l)."""
import os

from kube_sqs_autoscaler_amd.bench.latency import BenchEnv


def _workers():
    out = set()
    for t in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{t}/comm") as f:
                if f.read().strip() == "ksa-worker":
                    out.add(int(t))
        except OSError:
            pass
    return out


def test_runner_keeps_its_thread_across_runs(nat):
    earlier = _workers()  # other tests' runners may still be alive in this process
    env = BenchEnv(3, "scale", servers="per-queue")
    try:
        env.run(20)
        first = _workers() - earlier
        assert len(first) == 3
        env.run(20)  # a new Supervisor, the same runners
        assert _workers() - earlier == first
        sched = env.last_thread_sched
        assert sched["threads"] == 3 and sched["cpu_ns"] > 0  # this run's share only
        res = env.collect(20, 1.0)
        assert len(res.samples) == 3 * 40 and res.signature_failures == 0
    finally:
        env.close()


def test_threads_end_with_their_runners(nat):
    import gc

    env = BenchEnv(2, "scale", servers="per-queue")
    try:
        earlier = _workers()
        env.run(5)
        mine = _workers() - earlier
        assert len(mine) == 2
        env.runners.clear()
        gc.collect()
        assert not (_workers() & mine)
    finally:
        env.close()
