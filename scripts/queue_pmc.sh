# Closed-loop kernel: A/B against the libraries given as arguments, then PMC passes
# (--pmc only with --kernel-trace/--stats; per-block counter limits respected).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH=scripts/queue_sweep_bench.py bash scripts/ab_sweep.sh "$@" &&
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k closed > gpurun_out/pytest_closed.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/qpmc -o queue -- python3 scripts/queue_sweep_bench.py > gpurun_out/qpmc.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/qpmc2 -o queue -- python3 scripts/queue_sweep_bench.py > gpurun_out/qpmc2.log 2>&1
