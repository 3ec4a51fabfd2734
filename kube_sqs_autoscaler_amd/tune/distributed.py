"""Multi-GPU what-if sweeps: one process per GPU, configurations sharded by rank.

Extension (an operator tool, like the rest of :mod:`kube_sqs_autoscaler_amd.tune`). Launch with
``torchrun`` (``python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m
kube_sqs_autoscaler_amd.tune --distributed ...``). Every rank:

1. takes a cost-balanced share of the configuration grid (:func:`shard_plan`). A lane's work is
   the number of polls it simulates, horizon / (poll period + SQS latency), so on a grid with
   poll periods 1 s..10 s the 1 s configurations cost ten times the 10 s ones: equal-count
   slices of the poll-sorted grid would leave the rank holding the shortest periods running
   long after the others. Configurations are dealt out in cost order so every rank's summed
   :func:`sweep.estimated_polls` is within a few % of the mean, and each rank's share stays
   poll-sorted (neighbouring lanes of a wave share loop trip counts);
2. runs it on its own GPU (``LOCAL_RANK``) with the same kernel a single-GPU sweep uses, or on
   CPU threads;
3. all-gathers the per-configuration outputs over ``torch.distributed`` and scatters them back
   into grid order. The backend is ``nccl`` (RCCL over xGMI on an MI355X node) when the GPUs
   run the sweep, ``gloo`` on CPU.

The outputs are a few dozen bytes per configuration: every field is packed into one int64
row per configuration, so a sweep makes one all-gather (plus one all-reduce of the kernel
time), not one per field; the simulation dominates. Every rank ends with the full result,
bit-identical to a single-process sweep of the whole grid (``tests/test_tune_distributed.py``).
"""
from __future__ import annotations

import os
from typing import Dict, List, Tuple

import numpy as np

from . import closedloop, sweep


def config_costs(params: np.ndarray, horizon_ns: int, latency_ns: Tuple[int, int, int]) -> np.ndarray:
    """Per-configuration simulated polls (the unit :func:`sweep.estimated_polls` sums): the work
    of one lane is proportional to it, whatever its other parameters."""
    # the poll period clipped to the horizon first: a huge period from a user grid must cost one
    # poll, not wrap negative in int64 when the latency is added (and cost horizon polls)
    period = np.clip(np.asarray(params[0], dtype=np.int64), 0, max(int(horizon_ns), 0))
    step = np.maximum(period + min(max(int(latency_ns[0]), 0), max(int(horizon_ns), 0)), 1)
    return np.maximum(np.minimum(horizon_ns // step, 1 << 26), 0).astype(np.int64)


def shard_plan(costs: np.ndarray, world: int) -> List[np.ndarray]:
    """Splits configurations 0..m-1 over `world` ranks so the per-rank cost sums are balanced.

    Configurations are sorted by decreasing cost (ties in grid order) and dealt out in a snake
    order, 0, 1, ..., w-1, w-1, ..., 1, 0, 0, 1, ...: within every round of `world` the rank that
    took the most expensive configuration takes the cheapest of the next round. Every rank gets
    the same number of configurations (+-1), and its cost sum is within about one configuration's
    cost of the mean. Each rank's index array comes out in decreasing-cost (= increasing poll)
    order, so lanes next to each other in a wave run similar trip counts. The plan depends only
    on the costs, so every rank computes the same one."""
    m = len(costs)
    order = np.lexsort((np.arange(m), -np.asarray(costs, dtype=np.int64)))
    pos = np.arange(m)
    rnd, k = np.divmod(pos, world)
    ranks = np.where(rnd % 2 == 0, k, world - 1 - k)
    return [order[ranks == r] for r in range(world)]


class Group:
    """The process group a sharded sweep runs in (initialised from the torchrun environment)."""

    def __init__(self, device: str = "auto"):
        import sys

        from ..ops import gpu as _gpu

        if "torch" not in sys.modules and _gpu._LIB is not None:
            # Measured on the MI355X image: once libksa_gpu.so has initialised the ROCm runtime,
            # a later `import torch` binds torch to that already-loaded runtime and
            # torch.cuda.is_available() turns False. Import order is the only fix.
            raise RuntimeError("create the sweep Group (it imports torch) before the first GPU sweep of the process")
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if device == "auto":
            device = "gpu" if sweep.gpu_available() else "cpu"
        self.device = device
        self.owned = False
        use_gpu = device == "gpu"
        if use_gpu:
            torch.cuda.set_device(self.local_rank)
            self.tensor_device = torch.device("cuda", self.local_rank)
        else:
            self.tensor_device = torch.device("cpu")
        if self.world > 1 and not dist.is_initialized():
            if use_gpu:
                dist.init_process_group("nccl", device_id=self.tensor_device)
            else:
                dist.init_process_group("gloo")
            self.owned = True

    def close(self) -> None:
        if self.owned:
            self.dist.destroy_process_group()
            self.owned = False

    def all_gather_rows(self, shard: np.ndarray, counts: List[int]) -> np.ndarray:
        """Concatenation over ranks of each rank's rows (axis 0), `counts[r]` rows from rank r."""
        if self.world == 1:
            return shard
        torch = self.torch
        longest = max(counts)
        pad = np.zeros((longest,) + shard.shape[1:], dtype=shard.dtype)
        pad[: shard.shape[0]] = shard
        t = torch.from_numpy(pad).to(self.tensor_device)
        parts = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t)
        return np.concatenate([p.cpu().numpy()[:n] for p, n in zip(parts, counts)], axis=0)

    def all_gather_fields(self, out: Dict[str, np.ndarray], counts: List[int]) -> Dict[str, np.ndarray]:
        """:meth:`all_gather_rows` of every output field at once: the fields (int32 / int64,
        one row per configuration) are packed side by side into one int64 array -- exact for
        both -- gathered in one collective, and split back to their own dtypes and shapes."""
        keys = sorted(out)  # the same order on every rank
        widths = [int(np.prod(out[k].shape[1:], dtype=np.int64)) for k in keys]
        rows = out[keys[0]].shape[0] if keys else 0
        packed = np.empty((rows, sum(widths)), dtype=np.int64)
        off = 0
        for k, w in zip(keys, widths):
            packed[:, off:off + w] = out[k].reshape(rows, w)
            off += w
        full = self.all_gather_rows(packed, counts)
        res, off = {}, 0
        for k, w in zip(keys, widths):
            res[k] = full[:, off:off + w].astype(out[k].dtype).reshape((full.shape[0],) + out[k].shape[1:])
            off += w
        return res

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.tensor_device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())


def _shards(g: Group, params: np.ndarray, horizon_ns: int,
            latency_ns: Tuple[int, int, int]) -> Tuple[np.ndarray, List[int], np.ndarray]:
    """This rank's configuration indices, every rank's count, and the rank-major concatenation
    of all ranks' indices (row i of the all-gathered output belongs to configuration
    ``gathered_order[i]``)."""
    plan = shard_plan(config_costs(params, horizon_ns, latency_ns), g.world)
    return plan[g.rank], [len(p) for p in plan], np.concatenate(plan) if plan else np.zeros(0, np.int64)


def _to_grid_order(full: Dict[str, np.ndarray], gathered_order: np.ndarray) -> Dict[str, np.ndarray]:
    res = {}
    for k, v in full.items():
        out = np.empty_like(v)
        out[gathered_order] = v
        res[k] = out
    return res


def run_open_loop(g: Group, trace: sweep.Trace, params: np.ndarray, init_replicas: int, horizon_ns: int,
                  latency_ns: Tuple[int, int, int]) -> sweep.SweepResult:
    """:func:`sweep.run` over the whole grid, sharded over the group's ranks."""
    params = np.ascontiguousarray(params, dtype=np.int64)
    mine, counts, order = _shards(g, params, horizon_ns, latency_ns)
    if len(mine):
        res = sweep.run(trace, np.ascontiguousarray(params[:, mine]), init_replicas, horizon_ns, latency_ns, g.device,
                        gpu_index=g.local_rank)
        out, kernel_ms, ns_clock, no_skip = res.out, res.kernel_ms, not res.ms_clock, not res.skip
    else:  # more ranks than configurations
        out = {k: np.zeros(0, dtype=np.int64 if k in sweep.OUT64 else np.int32) for k in sweep.OUT64 + sweep.OUT32}
        kernel_ms, ns_clock, no_skip = 0.0, False, False
    full = _to_grid_order(g.all_gather_fields(out, counts), order)
    # ms_clock / skip: every shard ran the millisecond clock / the steady-stretch skip (each shard
    # picks the skip for its own configurations; the results do not depend on it)
    return sweep.SweepResult(params, full, g.device, g.max(kernel_ms), g.max(float(ns_clock)) == 0.0,
                             g.max(float(no_skip)) == 0.0)


def run_closed_loop(g: Group, trace: closedloop.ArrivalTrace, params: np.ndarray, model: closedloop.QueueModel,
                    init_replicas: int, horizon_ns: int, latency_ns: Tuple[int, int, int], seeds: int,
                    seed0: int) -> closedloop.ClosedLoopResult:
    """:func:`closedloop.run` over the whole grid, sharded over the group's ranks. Seeds are
    common to all configurations, so every shard draws the same arrival sequences."""
    params = np.ascontiguousarray(params, dtype=np.int64)
    mine, counts, order = _shards(g, params, horizon_ns, latency_ns)
    if len(mine):
        res = closedloop.run(trace, np.ascontiguousarray(params[:, mine]), model, init_replicas, horizon_ns, latency_ns,
                             seeds, seed0, g.device, gpu_index=g.local_rank)
        out, kernel_ms, flags = res.out, res.kernel_ms, (res.fast_arith, res.ms_clock)
    else:
        out = {k: np.zeros((0, seeds), dtype=np.int64 if k in closedloop.OUT64 else np.int32)
               for k in closedloop.OUT64 + closedloop.OUT32}
        kernel_ms, flags = 0.0, (True, True)
    full = _to_grid_order(g.all_gather_fields(out, counts), order)
    # fast_arith / ms_clock: every shard ran it
    fast, ms_clock = (g.max(float(not f)) == 0.0 for f in flags)
    return closedloop.ClosedLoopResult(params, seeds, full, g.device, horizon_ns, g.max(kernel_ms), fast, ms_clock)
