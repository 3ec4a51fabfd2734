"""Sharded what-if sweeps (tune/distributed.py): torchrun ranks over gloo on CPU must reproduce
the single-process sweep exactly (RCCL on an MI355X node runs the same code path with cuda
tensors)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from kube_sqs_autoscaler_amd.tune.distributed import shard_bounds

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("m,world", [(10, 3), (3, 8), (0, 2), (1000, 8), (7, 1)])
def test_shard_bounds_partition(m, world):
    bounds = [shard_bounds(m, r, world) for r in range(world)]
    assert bounds[0][0] == 0 and bounds[-1][1] == m
    assert all(a[1] == b[0] for a, b in zip(bounds, bounds[1:]))
    sizes = [hi - lo for lo, hi in bounds]
    assert max(sizes) - min(sizes) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args, world=None):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    if world is None:
        cmd = [sys.executable, "-m", "kube_sqs_autoscaler_amd.tune", *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "-m", "kube_sqs_autoscaler_amd.tune",
               "--distributed", *args]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    return lines[0], lines[1:]


def test_open_loop_three_ranks_equal_single_process(tmp_path):
    csv = tmp_path / "depth.csv"
    csv.write_text("seconds,depth\n" + "".join(f"{i * 5},{(i * 37) % 400}\n" for i in range(300)))
    args = ["--trace", str(csv), "--device", "cpu", "--json", "--top", "0", "--grid", "scale-up-cool-down=0s:2m:20s",
            "--grid", "scale-up-messages=50,100,200,400", "--grid", "max-pods=4,8,16"]  # 7 x 4 x 3 = 84 configs
    info1, rows1 = _run(args)
    info3, rows3 = _run(args, world=3)
    assert info3["ranks"] == 3 and info1["ranks"] == 1
    assert info1["configs"] == info3["configs"] == 84
    assert rows1 == rows3 and len(rows1) == 84


def test_closed_loop_two_ranks_equal_single_process(tmp_path):
    csv = tmp_path / "rate.csv"
    csv.write_text("seconds,msgs_per_second\n0,2\n600,30\n1200,2\n")
    args = ["--arrivals", str(csv), "--horizon", "40m", "--service-rate", "5", "--seeds", "6", "--device", "cpu",
            "--json", "--top", "0", "--grid", "scale-up-cool-down=0s:4m:1m", "--grid", "max-pods=2,8,9"]
    info1, rows1 = _run(args)
    info2, rows2 = _run(args, world=2)
    assert info2["ranks"] == 2 and info1["configs"] == info2["configs"] == 15
    assert rows1 == rows2 and len(rows1) == 15


def test_group_refuses_to_start_after_the_kernels_library(monkeypatch):
    import sys

    from kube_sqs_autoscaler_amd.ops import gpu
    from kube_sqs_autoscaler_amd.tune import distributed

    monkeypatch.setattr(gpu, "_LIB", object())
    monkeypatch.delitem(sys.modules, "torch", raising=False)
    with pytest.raises(RuntimeError, match="before the first GPU sweep"):
        distributed.Group("cpu")
