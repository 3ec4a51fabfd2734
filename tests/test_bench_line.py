"""bench.py's result line fits the driver's capture.

The driver parses the last line of stdout out of its last 8,000 characters. Round 5's line was
24.6 KB: its head, with ``metric`` and ``value``, fell outside the tail and the round's headline
was recorded unparsed (BENCH_r05.json ``parsed: null``). The line now holds the headline and the
summary rows only (at most 4,096 bytes); the rest goes to the ``--detail-out`` file it names.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

HEADLINE = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config", "parallelism",
            "higher_is_better", "scaling", "vs_baseline", "data")
SUMMARY = ("p50_ms_by_tracked_queues", "decision_parity", "wan_cadenced_p50_ms", "cpu_ms_per_poll",
           "cadenced_reference_over_default", "cadenced_p50_ms_by_tracked_queues", "ranks", "collective_backend")


def _driver_parse(stdout: str) -> dict:
    """What the driver does: keep the last 8,000 characters, parse the last line."""
    tail = stdout[-8000:]
    return json.loads(tail.strip().splitlines()[-1])


def _full():
    with open(os.path.join(ROOT, "tests", "fixtures", "bench_line_r05ag_full.json")) as f:
        return json.load(f)


def test_round5_result_fits_and_parses_from_the_tail():
    """Round 5's own full result (24.6 KB; profiles/r05ag/bench.json at ee40be9) becomes a line of at most 4,096 bytes
    that parses from the tail with every headline key and every summary row."""
    out = _full()
    assert len(json.dumps(out)) > 20_000
    line = bench.result_line(out, "gpurun_out/bench_detail.json")
    assert len(line.encode()) <= bench.LINE_LIMIT
    stdout = "[bench] noise\n" * 500 + line + "\n"
    got = _driver_parse(stdout)
    for k in HEADLINE:
        assert k in got, k
    assert got["value"] == out["value"] and got["metric"] == bench.METRIC
    assert got["parallelism"] == "dp1" == got["config"]["parallelism"]
    for k in SUMMARY:
        assert k in got["extra"], k
    assert got["extra"]["decision_parity"] == {"fraction": 1.0, "polls": "2000/2000"}  # 4 wire configs x 500 polls
    assert got["extra"]["p50_ms_by_tracked_queues"] == out["extra"]["p50_ms_by_tracked_queues"]
    assert got["extra"]["detail"] == "gpurun_out/bench_detail.json"
    assert "dropped_from_line" not in got["extra"]
    assert "cadenced_rows" not in got["extra"]  # the 8.9 KB per-row detail stays in the file


def test_oversized_rows_are_dropped_least_important_first():
    out = _full()
    out["extra"]["cadenced_p50_ms_by_tracked_queues"] = {f"setup{i}": {"x" * 50: i} for i in range(100)}
    out["extra"]["section_errors"] = {"cadence_rows": "E" * 10_000}
    line = bench.result_line(out, None)
    assert len(line.encode()) <= bench.LINE_LIMIT
    got = json.loads(line)
    assert got["extra"]["dropped_from_line"] == ["cadenced_p50_ms_by_tracked_queues"]
    assert len(got["extra"]["section_errors"]["cadence_rows"]) == 200
    assert got["extra"]["p50_ms_by_tracked_queues"] and got["extra"]["detail"] is None
    # even free text past the limit cannot push the headline out
    out["data"] = "d" * 10_000
    out["config"]["model"] = "m" * 10_000
    got = json.loads(bench.result_line(out, None))
    assert got["value"] == out["value"] and len(json.dumps(got)) <= bench.LINE_LIMIT


def _run(args, env=None, tmp_path=None):
    detail = str(tmp_path / "detail.json")
    r = subprocess.run([sys.executable, "bench.py", *args, "--detail-out", detail], cwd=ROOT, capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    got = _driver_parse(r.stdout)
    assert len(r.stdout.strip().splitlines()[-1].encode()) <= bench.LINE_LIMIT
    for k in HEADLINE:
        assert k in got, k
    assert got["extra"]["detail"] == detail
    with open(detail) as f:
        full = json.load(f)
    assert full["value"] == got["value"] and full["extra"]["samples"] == got["extra"]["samples"]
    return got, full


def test_single_rank_line_and_detail_file(tmp_path):
    got, full = _run(["--steps", "100", "--warmup", "10", "--no-sweep"], tmp_path=tmp_path)
    assert got["extra"]["decision_parity"]["fraction"] == 1.0
    assert full["extra"]["decision_parity"]["configs"]  # the per-scenario rows are in the file


@pytest.mark.slow
def test_two_rehearsal_ranks_line(tmp_path):
    """`bench.py --gpus 2 --rehearse-shared-gpus` over gloo: rank 0's line parses from the tail
    and covers both ranks."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    got, _ = _run(["--gpus", "2", "--steps", "60", "--warmup", "5", "--no-sweep", "--rehearse-shared-gpus"],
                  env=env, tmp_path=tmp_path)
    assert got["extra"]["ranks"] == 2 and got["extra"]["collective_backend"] == "gloo"
    assert got["parallelism"] == "dp2" and got["extra"]["samples"] == 120


def test_rehearsal_checker_reads_the_driver_tail():
    """scripts/check_bench_line.py (the GPU-box rehearsal's check) accepts the compact line after
    10 KB of other output and rejects round 5's full line, whose head the tail cuts off."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import check_bench_line

    out = _full()
    ok = check_bench_line.check("x" * 10_000 + "\n" + bench.result_line(out, "d.json") + "\n")
    assert ok["ok"] and ok["missing"] == [] and ok["value"] == out["value"] and ok["bytes"] <= 4096
    bad = check_bench_line.check("x" * 10_000 + "\n" + json.dumps(out) + "\n")
    assert not bad["ok"] and "does not parse" in bad["error"]
