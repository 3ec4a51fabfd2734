"""Parses bench.py's result line the way the driver does and checks it.

Reads stdout of a ``bench.py`` run on stdin, keeps its last 8,000 characters (the driver's
capture), parses the last line and checks its size (at most 4,096 bytes), its headline keys and
its summary rows. Prints one JSON line: ok, the line's size, the headline value and any key that is
missing; exits 1 when the line does not parse or a key is missing.

    python3 bench.py --gpus 1 --steps 20 --warmup 5 | tail -c 8000 | python3 scripts/check_bench_line.py
"""
import json
import sys

HEADLINE = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config", "parallelism")
SUMMARY = ("p50_ms_by_tracked_queues", "decision_parity", "wan_cadenced_p50_ms", "cpu_ms_per_poll",
           "cadenced_reference_over_default", "cadenced_p50_ms_by_tracked_queues", "ranks", "collective_backend")


def check(stdout: str, sweep: bool = True) -> dict:
    tail = stdout[-8000:]
    lines = tail.strip().splitlines()
    if not lines:
        return {"ok": False, "error": "no stdout"}
    last = lines[-1]
    try:
        got = json.loads(last)
    except ValueError as e:
        return {"ok": False, "error": f"last line does not parse: {e}", "bytes": len(last.encode())}
    missing = [k for k in HEADLINE if k not in got]
    extra = got.get("extra") or {}
    # without the secondary sections (--no-sweep, or a world > 1) only the rows every run has
    wanted = SUMMARY if sweep else ("decision_parity", "ranks", "collective_backend")
    missing += [f"extra.{k}" for k in wanted if k not in extra]
    size = len(last.encode())
    return {"ok": not missing and size <= 4096, "bytes": size, "missing": missing, "value": got.get("value"),
            "unit": got.get("unit"), "n_gpus": got.get("n_gpus"), "parallelism": got.get("parallelism"),
            "decision_parity": extra.get("decision_parity"), "skipped_sections": extra.get("skipped_sections"),
            "dropped_from_line": extra.get("dropped_from_line"), "detail": extra.get("detail")}


def main() -> int:
    res = check(sys.stdin.read(), sweep="--no-sweep" not in sys.argv[1:])
    print(json.dumps(res))
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
