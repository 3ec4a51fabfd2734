# Closed-loop kernel on the box: GPU == CPU test, kernel time (rocprofv3 --stats), then PMC
# passes (--pmc only with --kernel-trace/--stats; per-block counter limits respected).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/queue}
mkdir -p "$OUT"
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k closed > "$OUT/pytest_closed.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o queue -- python3 scripts/queue_sweep_bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err" &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d "$OUT/pmc" -o queue -- python3 scripts/queue_sweep_bench.py > "$OUT/pmc.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc2" -o queue -- python3 scripts/queue_sweep_bench.py > "$OUT/pmc2.log" 2>&1
