"""Tests that need the MI355X: the gfx950 probe kernels and the driver smoke path."""
import pytest

pytestmark = pytest.mark.gpu


def test_probe_inventory():
    from kube_sqs_autoscaler_amd.ops import gpu

    n = gpu.device_count()
    assert n >= 1
    info = gpu.device_info(0)
    assert info.arch.startswith("gfx950"), info
    assert info.wavefront_size == 64
    assert info.compute_units >= 256
    assert info.total_mem_bytes > 250 << 30  # 288 GB HBM3E


def test_hbm_health_check_matches_host_checksum():
    from kube_sqs_autoscaler_amd.ops import gpu

    h = gpu.health_check(0, 2 << 30, reps=5)  # 2 GiB >> 256 MiB Infinity Cache: HBM-bound
    assert h.ok and h.mismatches == 0 and h.checksum == h.expected_checksum
    print(f"HBM write {h.write_gbps:.0f} GB/s, read+verify {h.read_gbps:.0f} GB/s")
    # streaming kernels should reach a large fraction of the ~6.3 TB/s achievable
    assert h.read_gbps > 3000 and h.write_gbps > 3000, h


def test_healthy_gpu_count():
    from kube_sqs_autoscaler_amd.ops import gpu

    assert gpu.healthy_gpu_count(16 << 20) == gpu.device_count()


def test_graft_smoke():
    import __graft_entry__ as g

    g.smoke()


def test_cli_gpu_aware_max_local(tmp_path, capfd):
    """--gpu-aware-max=local: the gfx950 probe counts healthy GPUs and caps max-pods at them."""
    import yaml

    from kube_sqs_autoscaler_amd.cli import main
    from kube_sqs_autoscaler_amd.ops import fakes, gpu

    fk = fakes()
    n_gpus = gpu.device_count()
    sqs, kube = fk.FakeSqsServer(), fk.FakeKubeServer()
    sqs.start()
    kube.start()
    try:
        url = sqs.url + "/1/q"
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": "1000"})
        kube.add_deployment("ml", "w", 1)
        kc = tmp_path / "kc"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": "x"}}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = {"AWS_ACCESS_KEY_ID": "a", "AWS_SECRET_ACCESS_KEY": "b", "KUBE_CONFIG_PATH": str(kc)}
        rc = main([f"--sqs-queue-url={url}", "--kubernetes-deployment=w", "--kubernetes-namespace=ml", "--aws-region=us-east-1",
                   f"--sqs-endpoint={sqs.url}", "--poll-period=1ms", "--scale-up-cool-down=0s", "--max-pods=64",
                   "--attribute-names=ApproximateNumberOfMessages", "--gpu-aware-max=local", "--kube-api-qps=0"],
                  environ=env, max_iterations=100)
        assert rc == 0
        assert kube.replicas("ml", "w") == min(64, n_gpus)
        assert f"GPU capacity: {n_gpus} pods" in capfd.readouterr().err
    finally:
        sqs.stop()
        kube.stop()


def test_cli_gpu_aware_max_local_with_worker_processes(tmp_path):
    """--gpu-aware-max=local with --worker-processes, in a fresh process as in production: the
    workers are forked first, then the supervisor runs the gfx950 probe and forwards the cap to
    every worker through its shared slot. Two queues, both capped at the healthy GPU count."""
    import os
    import signal
    import subprocess
    import sys
    import time

    import yaml

    from kube_sqs_autoscaler_amd.ops import fakes, gpu

    fk = fakes()
    n_gpus = gpu.device_count()
    sqs, kube = fk.FakeSqsServer(), fk.FakeKubeServer()
    sqs.start()
    kube.start()
    p = None
    try:
        specs = []
        for i in range(2):
            url = f"{sqs.url}/1/q{i}"
            sqs.set_attributes(url, {"ApproximateNumberOfMessages": "1000"})
            kube.add_deployment("ml", f"w{i}", 1)
            specs += ["--queue", f"url={url},deployment=w{i},namespace=ml,attribute-names=ApproximateNumberOfMessages"]
        kc = tmp_path / "kc"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": "x"}}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        env = dict(os.environ, AWS_ACCESS_KEY_ID="a", AWS_SECRET_ACCESS_KEY="b", KUBE_CONFIG_PATH=str(kc))
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        err_path = tmp_path / "stderr.log"  # a file, not a pipe: nobody drains a pipe while it runs
        err = open(err_path, "w")
        p = subprocess.Popen([sys.executable, "-m", "kube_sqs_autoscaler_amd", "--aws-region=us-east-1",
                              f"--sqs-endpoint={sqs.url}", "--poll-period=5ms", "--scale-up-cool-down=0s", "--max-pods=64",
                              "--gpu-aware-max=local", "--kube-api-qps=0", "--worker-processes", *specs],
                             cwd=root, env=env, stderr=err, text=True)
        err.close()
        want = min(64, n_gpus)
        deadline = time.time() + 90
        # both workers polling (the CLI imports and forks first), each far past the cap's reach
        while time.time() < deadline and p.poll() is None and sqs.requests() < 100:
            time.sleep(0.05)
        assert sqs.requests() >= 100, "the workers did not start polling"
        assert [kube.replicas("ml", f"w{i}") for i in range(2)] == [want, want]
        polled = sqs.requests()
        time.sleep(0.3)  # more polls: the cap holds
        assert sqs.requests() >= polled + 20
        assert [kube.replicas("ml", f"w{i}") for i in range(2)] == [want, want]
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=30) == 0
        assert f"GPU capacity: {n_gpus} pods" in err_path.read_text()
    finally:
        if p is not None and p.poll() is None:
            p.kill()
        sqs.stop()
        kube.stop()


def _random_walk_trace(n, seed):
    import numpy as np

    from kube_sqs_autoscaler_amd.tune import sweep

    rng = np.random.default_rng(seed)
    t = np.concatenate([[0], np.cumsum(rng.integers(1, 20, n - 1)) * 1_000_000_000])
    d = np.maximum(0, np.cumsum(rng.integers(-40, 41, n)) + 100)
    return sweep.Trace(t, d)


def test_sweep_kernel_equals_cpu_and_oracle():
    """gfx950 sweep kernel: bit-identical to the CPU path on a 30k-config grid (trace in LDS and
    trace in global memory), and to the Python oracle on a sample."""
    import numpy as np

    from kube_sqs_autoscaler_amd.tune import sweep

    S = 1_000_000_000
    grid = sweep.grid(poll_ns=[2 * S, 5 * S], up_cool_ns=list(range(0, 300 * S, 20 * S)),
                      down_cool_ns=list(range(0, 600 * S, 60 * S)), up_msgs=[50, 100, 200, 400, 800],
                      down_msgs=[5, 50], up_pods=[1, 2], max_pods=[8, 16], min_pods=[1])
    assert grid.shape[1] == 2 * 15 * 10 * 5 * 2 * 2 * 2
    # traces staged in LDS up to 32 KiB: <= 2048 int64 segments on the nanosecond clock, <= 4096
    # int32 ones on the millisecond clock; longer ones are read from global memory
    for n in (1000, 3000, 6000):
        tr = _random_walk_trace(n, n)
        horizon = int(tr.t_ns[-1]) + 5 * S
        lat = (2_000_000, 1_000_000, 1_000_000)
        c = sweep.run(tr, grid, 2, horizon, lat, device="cpu", clock="ns", skip="off")
        g = sweep.run(tr, grid, 2, horizon, lat, device="gpu")
        assert g.device == "gpu" and g.kernel_ms > 0 and g.ms_clock and g.skip and not c.ms_clock
        # every kernel instantiation: both clocks, with and without the steady-stretch skip
        for clock in ("auto", "ns"):
            for skip in ("on", "off"):
                gk = g if (clock, skip) == ("auto", "on") else sweep.run(tr, grid, 2, horizon, lat, device="gpu",
                                                                          clock=clock, skip=skip)
                assert gk.ms_clock == (clock == "auto") and gk.skip == (skip == "on")
                for k in g.out:
                    assert np.array_equal(gk.out[k], c.out[k]), (k, clock, skip)
        assert int(g.out["ups"].sum()) > 0 and int(g.out["downs"].sum()) > 0
        for i in range(0, len(g), len(g) // 7):
            o = sweep.oracle_row(tr, g.config(i), 2, horizon, (2_000_000, 1_000_000, 1_000_000))
            assert {k: g.row(i)[k] for k in o} == o


def test_closed_loop_kernel_equals_cpu_and_python_model():
    """gfx950 closed-loop sweep: bit-identical to the CPU path over a grid x seeds, and to the
    independent Python statement of the model on a sample of lanes."""
    import numpy as np

    from kube_sqs_autoscaler_amd.tune import closedloop as cl
    from kube_sqs_autoscaler_amd.tune import sweep

    S = 1_000_000_000
    tr = cl.ArrivalTrace.from_segments([(0, 0.5), (300, 40.0), (900, 1.5), (1500, 0.0)])
    grid = sweep.grid(poll_ns=[5 * S, 7 * S], up_cool_ns=list(range(0, 300 * S, 30 * S)),
                      down_cool_ns=[0, 60 * S, 300 * S], up_msgs=[20, 100, 400], max_pods=[4, 8, 16])
    model = cl.QueueModel(service_rate=5.0, startup_ns=60 * S, slo_backlog=200, init_backlog=10)
    lat = (2_000_000, 1_000_000, 1_000_000)
    g = cl.run(tr, grid, model, 1, 2400 * S, lat, seeds=64, device="gpu")
    gn = cl.run(tr, grid, model, 1, 2400 * S, lat, seeds=64, device="gpu", arith="fast-ns")
    gs = cl.run(tr, grid, model, 1, 2400 * S, lat, seeds=64, device="gpu", arith="saturating")
    c = cl.run(tr, grid, model, 1, 2400 * S, lat, seeds=64, device="cpu", arith="saturating")
    assert g.device == "gpu" and g.kernel_ms > 0
    # the bounds hold, so the GPU ran FastArith (on the millisecond decision clock: whole-ms
    # periods and latencies) -- and matches the saturating arithmetic exactly
    assert g.fast_arith and g.ms_clock and gn.fast_arith and not gn.ms_clock
    assert not gs.fast_arith and not c.fast_arith
    for k in g.out:
        assert np.array_equal(g.out[k], c.out[k]), k
        assert np.array_equal(gn.out[k], c.out[k]), k
        assert np.array_equal(gs.out[k], c.out[k]), k
    for i in range(0, len(g), 37):
        want = cl.reference_lane(tr, g.config(i), model, 1, 2400 * S, lat, 1 + 5)
        assert {k: int(v[i, 5]) for k, v in g.out.items()} == want


def test_closed_loop_kernel_equals_cpu_at_extremes():
    """The saturating / wide-operand paths of the closed-loop model on the GPU: maximum rates,
    20-day polls (intervals above 2^31 ms), a 1e12-message backlog."""
    import numpy as np

    from kube_sqs_autoscaler_amd.tune import closedloop as cl
    from kube_sqs_autoscaler_amd.tune import sweep

    S = 1_000_000_000
    for rate, service, poll_s, init in [(1e6, 1e6, 20 * 86400, 10**12), (1e6, 0.001, 3, 10**12), (0.001, 1e6, 1, 10**12)]:
        tr = cl.ArrivalTrace.from_segments([(0, rate), (7 * 86400, rate / 2)])
        grid = sweep.grid(poll_ns=[poll_s * S], up_cool_ns=[0], down_cool_ns=[0], up_msgs=[1, 10**15],
                          max_pods=[2**31 - 1, 50])
        model = cl.QueueModel(service_rate=service, startup_ns=86400 * S, slo_backlog=0, init_backlog=init)
        horizon = (30 * 86400 if poll_s > 86400 else 400) * S
        g = cl.run(tr, grid, model, 1, horizon, (0, 0, 0), seeds=4, device="gpu")
        c = cl.run(tr, grid, model, 1, horizon, (0, 0, 0), seeds=4, device="cpu")
        assert not g.fast_arith  # 2^31 - 1 pods: only the saturating arithmetic is safe
        for k in g.out:
            assert np.array_equal(g.out[k], c.out[k]), (rate, k)


def test_sharded_sweep_cli_on_gpu(tmp_path):
    """tune --distributed on the GPU under torchrun (one rank: the torch device / gpu_index
    plumbing), in a fresh process -- torch must initialise its HIP runtime before this test
    process's already-loaded kernels library could shadow it -- against the in-process CPU sweep."""
    import json
    import os
    import subprocess
    import sys

    from kube_sqs_autoscaler_amd.tune import closedloop as cl
    from kube_sqs_autoscaler_amd.tune import sweep

    S = 1_000_000_000
    csv = tmp_path / "rate.csv"
    csv.write_text("0,1\n300,25\n900,1\n")
    args = ["--arrivals", str(csv), "--horizon", "30m", "--service-rate", "5", "--seeds", "8", "--json", "--top", "0",
            "--slo-backlog", "100", "--grid", "scale-up-cool-down=0s,1m", "--grid", "max-pods=4,8,16", "--latency",
            "1ms,1ms,1ms", "--grid", "poll-period=2s,5s"]  # mixed periods: the cost-sorted shard is scattered back
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import socket

    with socket.socket() as sk:  # a free port, not a fixed one another job on the box may hold
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr=127.0.0.1", f"--master-port={port}", "-m", "kube_sqs_autoscaler_amd.tune",
                        "--distributed", "--device", "gpu", *args], cwd=root, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    info, rows = lines[0], lines[1:]
    assert info["device"] == "gpu" and info["ranks"] == 1 and len(rows) == 12
    tr = cl.ArrivalTrace.from_csv(str(csv))
    grid = sweep.grid(poll_ns=[2 * S, 5 * S], up_cool_ns=[0, 60 * S], max_pods=[4, 8, 16])
    c = cl.run(tr, grid, cl.QueueModel(5.0, 60 * S, 100), 1, 1800 * S, (1_000_000,) * 3, seeds=8, device="cpu")
    want = sorted((c.row(i) for i in range(len(c))), key=lambda x: x["pod_hours_mean"])
    assert sorted(rows, key=lambda x: x["pod_hours_mean"]) == want


def test_bench_pools_samples_over_rccl():
    """bench.py's job-wide pooling (``_pool``: padded all_gather of the samples, MAX all_reduce of
    the wall time) on this GPU's tensors over an RCCL process group. One GPU allows one rank, so
    the group has one; the collectives, dtypes (int64, float64) and the padding path are the ones
    an N-GPU job runs. In a fresh process, as above."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import json, os, sys, torch, torch.distributed as dist\n"
        f"sys.path.insert(0, {root!r}); import bench\n"
        "torch.cuda.set_device(0); dev = torch.device('cuda', 0)\n"
        "dist.init_process_group('nccl', device_id=dev)\n"
        "ns, wall = bench._pool([30, 10, 20], 1.5, dev, collective=True)\n"
        "empty, _ = bench._pool([], 0.25, dev, collective=True)\n"
        "print(json.dumps({'backend': dist.get_backend(), 'ns': ns, 'wall': wall, 'empty': empty}))\n"
        "dist.destroy_process_group()\n")
    import socket

    with socket.socket() as sk:  # a free port, not a fixed one another job on the box may hold
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert out == {"backend": "nccl", "ns": [10, 20, 30], "wall": 1.5, "empty": []}


def test_sweep_kernel_random_lanes_equal_oracle():
    """the gfx950 open-loop kernel against the independent Python oracle on 256 lanes
    per dispatch (adversarial + random configurations), with the trace in LDS and in global
    memory, plus GPU == CPU on every lane of the dispatch, in every kernel instantiation (both
    clocks, with and without the steady-stretch skip)."""
    import sys
    import os

    import numpy as np

    sys.path.insert(0, os.path.dirname(__file__))
    from _lanes import MS, S, lanes_to_check, random_params, random_walk_trace
    from kube_sqs_autoscaler_amd.tune import sweep

    lat = (2 * MS, MS, MS)
    params = random_params(16384, seed=21)  # >> 256 CUs x 64 lanes / 4: a full dispatch
    for n, seed in ((400, 1), (2600, 2)):
        tr = random_walk_trace(n, seed)
        horizon = min(int(tr.t_ns[-1]) + 10 * S, 1800 * S)
        c = sweep.run(tr, params, 2, horizon, lat, device="cpu", clock="ns", skip="off")
        # both clocks, each with the steady-stretch skip forced on and off
        runs = {(clock, skip): sweep.run(tr, params, 2, horizon, lat, device="gpu", clock=clock, skip=skip)
                for clock in ("auto", "ns") for skip in ("on", "off")}
        for (clock, skip), g in runs.items():
            assert g.device == "gpu" and g.ms_clock == (clock == "auto") and g.skip == (skip == "on")
            for k in g.out:
                assert np.array_equal(g.out[k], c.out[k]), (k, clock, skip)
        g = runs[("auto", "on")]
        for i in lanes_to_check(params.shape[1], 256, seed):
            o = sweep.oracle_row(tr, g.config(i), 2, horizon, lat)
            assert {k: g.row(i)[k] for k in o} == o, (i, g.config(i))


def test_closed_loop_kernel_random_lanes_equal_reference_model():
    import sys
    import os

    import numpy as np

    sys.path.insert(0, os.path.dirname(__file__))
    from _lanes import MS, S, lanes_to_check, random_params
    from kube_sqs_autoscaler_amd.tune import closedloop as cl

    lat = (2 * MS, MS, MS)
    params = random_params(4096, seed=31, min_poll_ms=2000)
    tr = cl.ArrivalTrace.from_segments([(0, 0.5), (120, 30.0), (400, 2.0), (700, 45.0), (800, 0.0)])
    model = cl.QueueModel(service_rate=4.0, startup_ns=45 * S, slo_backlog=150, init_backlog=20)
    seeds = 8
    g = cl.run(tr, params, model, 1, 1200 * S, lat, seeds=seeds, device="gpu")
    c = cl.run(tr, params, model, 1, 1200 * S, lat, seeds=seeds, device="cpu")
    for k in g.out:
        assert np.array_equal(g.out[k], c.out[k]), k
    rng = np.random.default_rng(9)
    for i in lanes_to_check(params.shape[1], 256, 13):
        s = int(rng.integers(0, seeds))
        want = cl.reference_lane(tr, g.config(i), model, 1, 1200 * S, lat, 1 + s)
        assert {k: int(v[i, s]) for k, v in g.out.items()} == want, (i, g.config(i))


def test_sweeps_reuse_device_buffers_across_sizes():
    """The sweep launchers keep grow-only device buffers and a stream per device
    (csrc/hip/device_arena.h): calls that shrink, grow and alternate kernels must still give
    exactly the CPU path's results (no stale tail of a larger earlier call leaks in)."""
    import numpy as np

    from kube_sqs_autoscaler_amd.tune import closedloop as cl
    from kube_sqs_autoscaler_amd.tune import sweep

    S = 1_000_000_000
    lat = (2_000_000, 1_000_000, 1_000_000)
    tr = cl.ArrivalTrace.from_segments([(0, 1.0), (200, 30.0), (500, 2.0)])
    model = cl.QueueModel(service_rate=4.0, startup_ns=30 * S, slo_backlog=100)
    big = sweep.grid(up_cool_ns=list(range(0, 240 * S, 30 * S)), max_pods=[4, 8, 16])
    small = big[:, :5]
    dtr = sweep.Trace.from_segments([(0, 0), (60 * S, 300), (400 * S, 5)])
    for grid, seeds in ((big, 16), (small, 3), (big, 16), (small, 40)):
        g = cl.run(tr, grid, model, 1, 900 * S, lat, seeds=seeds, device="gpu")
        c = cl.run(tr, grid, model, 1, 900 * S, lat, seeds=seeds, device="cpu")
        for k in g.out:
            assert np.array_equal(g.out[k], c.out[k]), (grid.shape, seeds, k)
        go = sweep.run(dtr, grid, 1, 900 * S, lat, device="gpu")
        co = sweep.run(dtr, grid, 1, 900 * S, lat, device="cpu")
        for k in go.out:
            assert np.array_equal(go.out[k], co.out[k]), (grid.shape, k)
